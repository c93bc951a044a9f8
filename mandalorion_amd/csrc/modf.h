// modf.h — module F (filterIsoforms.py:81-433) pieces shared by the host path (module_f.cpp
// mando_filter_isoforms) and the device path (modf_kernel.hip mando_filter_isoforms_device): the parsed
// isoforms, a chromosome's state after the absolute and relative-expression filters, and the per-isoform
// outcome of look_for_contained_isoforms' candidate search (filterIsoforms.py:125-278), which both paths
// turn into the same kept list and reason texts.
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include "../../include/mando.h"

namespace mando {
namespace modf {

struct Iso {
    std::string name;
    std::vector<std::string> fields;  // the clean PSL line, split on tabs
    std::vector<int64_t> coords;      // block start, block end, ...
    char dir = '+';
    int64_t abundance = 0;
};

// merged [s, e) intervals
using Ivs = std::vector<std::pair<int64_t, int64_t>>;

// a chromosome after parse_clean_psl, get_count and filter_isoforms
struct ChrState {
    std::vector<int> listed;  // isoforms passing the parse, line order (psl_dict)
    std::vector<int> kept1;   // passing the relative-expression filter, name order
    std::vector<Ivs> ext;     // per isoform (filled for kept1): merged blocks +- splice window
    std::vector<int> bydir[2];  // kept1 per direction (+, -), by first merged start
    int64_t maxspan[2] = {0, 0};
};

// look_for_contained_isoforms' search for isoform k: |status| and |extend| (k itself included), the
// extending isoform the reason names (smallest name), and the first isoform of status in name order
// (other than k) whose junctions contain k's and that decides: kind 1 the internal ratio, 2 near
// identical, 3 a zero abundance (the reference's ZeroDivisionError); trig -1 / kind 0 when none does
struct Contain {
    int64_t n_status = 0, n_extend = 0;
    int ext_first = -1, trig = -1, kind = 0;
};

// the containment search of every chromosome at once: dec[c][t] for isoform kept1[t] of chromosome c
using ContainStage = std::function<int(const mando_filter_params &, const std::vector<std::vector<Iso>> &,
                                       const std::vector<ChrState> &, std::vector<std::vector<Contain>> &)>;

// mando_filter_isoforms with the containment search done by `stage` (nullptr: on the host, per
// chromosome in threads)
int filter_isoforms_impl(const mando_filter_params *P, const char *isoform_fasta, const char *genome_fasta,
                         const char *clean_psl, const char *whitelist_bed, const char *out_fasta, const char *out_psl,
                         const char *reasons_path, int64_t *n_kept, const ContainStage *stage);

}  // namespace modf
}  // namespace mando
