// revcomp.h — the complement table mappy.revcomp applies (minimap2's seq_comp_table, used through
// mappy's revcomp binding): IUPAC complements in either case (A<->T, C<->G, U->A, R<->Y, K<->M, B<->V,
// D<->H, S, W and N map to themselves); every other byte is kept.  Shared by the read packer
// (cluster.cpp) and SAM -> PSL (sam.cpp).
#pragma once
#include <cstdint>

namespace mando {

struct CompTable {
    uint8_t t[256];
    CompTable() {
        for (int i = 0; i < 256; ++i) t[i] = (uint8_t)i;
        const char *a = "ACGTURYKMBVDHSWN", *b = "TGCAAYRMKVBHDSWN";
        for (int i = 0; a[i]; ++i) {
            t[(uint8_t)a[i]] = (uint8_t)b[i];
            t[(uint8_t)(a[i] + 32)] = (uint8_t)(b[i] + 32);
        }
    }
};

inline const CompTable &comp_table() {
    static const CompTable c;
    return c;
}

}  // namespace mando
