// CPU check: the closed forms of trees.c's length / distance code tables in pmc_trees.hpp
// (len_code_cf, len_base_cf, len_extra_cf, dist_code_cf, dist_base_cf, dist_extra_cf, bl_order_cf)
// equal the tables zlib 1.2.11 builds in tr_static_init (trees.c) and its bl_order, entry for entry.
#include <cstdio>

#include "../../poor-man-s-cache_amd/csrc/pmc_trees.hpp"

int main() {
    using namespace pmc;
    static const int extra_lbits[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                        2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
    static const int extra_dbits[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                        6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
    unsigned char length_code[256], dist_code[512];
    int base_length[29], base_dist[30], n, code, length = 0, dist = 0;
    for (code = 0; code < 28; code++) {
        base_length[code] = length;
        for (n = 0; n < (1 << extra_lbits[code]); n++) length_code[length++] = (unsigned char)code;
    }
    length_code[length - 1] = 28; // as zlib: length 258 gets its own code
    base_length[28] = 255;
    for (code = 0; code < 16; code++) {
        base_dist[code] = dist;
        for (n = 0; n < (1 << extra_dbits[code]); n++) dist_code[dist++] = (unsigned char)code;
    }
    dist >>= 7;
    for (; code < 30; code++) {
        base_dist[code] = dist << 7;
        for (n = 0; n < (1 << (extra_dbits[code] - 7)); n++) dist_code[256 + dist++] = (unsigned char)code;
    }
    int bad = 0;
    for (unsigned lc = 0; lc < 256; lc++) bad += len_code_cf(lc) != length_code[lc];
    for (unsigned c = 0; c < 29; c++)
        bad += len_base_cf(c) != (unsigned)base_length[c] || len_extra_cf(c) != (unsigned)extra_lbits[c];
    for (unsigned dm = 0; dm < 32768; dm++)
        bad += dist_code_cf(dm) != (dm < 256 ? dist_code[dm] : dist_code[256 + (dm >> 7)]);
    for (unsigned dc = 0; dc < 30; dc++)
        bad += dist_base_cf(dc) != (unsigned)base_dist[dc] || dist_extra_cf(dc) != (unsigned)extra_dbits[dc];
    static const int bl_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    for (int i = 0; i < 19; i++) bad += bl_order_cf(i) != (unsigned)bl_order[i];
    printf("closed forms: %d mismatches\n", bad);
    return bad != 0;
}
