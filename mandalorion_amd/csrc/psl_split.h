// psl_split.h — the locus split's ordered-lines stage, shared by the host path (psl.cpp) and the GPU
// path (psl_kernel.hip): writes clean.sorted.psl (optional) and one <chrom>~<start>~<end>.psl per locus
// exactly as get_chromosomes (SpliceDefineConsensus.py:442-495) cuts the sorted lines.
#pragma once
#include <cstdint>
#include <string_view>
#include <vector>

namespace mando {
namespace psl {

struct Line {
    std::string_view text;   // without the trailing newline
    std::string_view chrom;  // field 14 (index 13)
    int64_t start = 0, end = 0;
    bool start_ok = false;
};

// lines in `sort -k 14,14 -k 16,17n` order (C locale; ties by the whole line)
int split_write_ordered(const std::vector<Line> &lines, const char *out_dir, const char *sorted_out,
                        int64_t *n_records, int64_t *n_loci);

}  // namespace psl
}  // namespace mando
