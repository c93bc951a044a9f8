// quant.h — module Q (assignReadsToIsoforms.py:27-105) pieces shared by the host path (module_f.cpp
// mando_quantify) and the device path (quant_kernel.hip mando_quantify_device): the read files' record
// names, the filtered PSL's isoform column and the two output tables, so both paths read and write alike.
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace mando {
namespace modq {

// mappy.fastx_read over one FASTA / FASTQ file (plain or gzip): buf holds the file, names each record's
// (offset into buf, length) in file order (name = header up to the first blank)
bool fastx_names(const char *path, std::string &buf, std::vector<std::pair<int64_t, int32_t>> &names);
// column 10 (a[9]) of every line of the filtered PSL, in line order; false on a line with < 10 fields
bool psl_isoforms(const std::string &buf, std::vector<std::string_view> &isos);
// .quant / .tpm: counts[k * samples + s] = reads of sample s assigned to isoform k
int write_tables(const std::vector<std::string> &samples, const std::vector<int64_t> &total,
                 const std::vector<std::string_view> &isos, const std::vector<int64_t> &counts, const char *out_quant,
                 const char *out_tpm);

}  // namespace modq
}  // namespace mando
