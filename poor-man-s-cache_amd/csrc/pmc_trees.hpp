// pmc_trees.hpp -- per-block Huffman construction for the gfx950 deflate kernel.
//
// Restates zlib 1.2.11 trees.c (build_tree / pqdownheap / gen_bitlen / gen_codes /
// scan_tree / send_tree / build_bl_tree / _tr_flush_block's block-type choice), the code
// behind the reference's deflate(Z_FINISH) call (/root/reference/src/compressor/
// gzip_compressor.cpp:38).  The binary heap is kept exactly (including `smaller`'s
// freq-then-depth order and the Dad/Len field aliasing): which of two equal-frequency
// symbols gets the longer code is decided by heap positions, so any other Huffman
// construction would change output bytes.
//
// Written as __host__ __device__ so tests/host/host_pipeline.cpp (tests/test_host_pipeline.py) compiles it
// with g++ and diffs it against oracle/trees.c on the CPU; on the GPU one lane of the wave runs it on
// the wave's LDS-resident PmcTrees.
#pragma once
#include <stdint.h>

#ifndef PMC_HD
#if defined(__HIPCC__)
#define PMC_HD __host__ __device__
#else
#define PMC_HD
#endif
#endif

namespace pmc {

constexpr int kLengthCodes = 29, kLiterals = 256, kLCodes = 286, kDCodes = 30, kBLCodes = 19;
constexpr int kHeapSize = 2 * kLCodes + 1, kMaxBits = 15, kMaxBLBits = 7, kEndBlock = 256;
constexpr int kRep3_6 = 16, kRepz3_10 = 17, kRepz11_138 = 18;

struct CtData {
    uint16_t fc; // Freq | Code
    uint16_t dl; // Dad | Len
};

struct Tables {
    uint8_t length_code[256];
    uint8_t dist_code[512];
    uint8_t extra_lbits[kLengthCodes];
    uint8_t extra_dbits[kDCodes];
    uint8_t extra_blbits[kBLCodes];
    uint8_t bl_order[kBLCodes];
    uint16_t base_length[kLengthCodes];
    uint16_t base_dist[kDCodes];
    CtData static_ltree[kLCodes + 2];
    CtData static_dtree[kDCodes];
};

constexpr unsigned bi_reverse_c(unsigned code, int len) {
    unsigned res = 0;
    do {
        res |= code & 1;
        code >>= 1, res <<= 1;
    } while (--len > 0);
    return res >> 1;
}

// trees.c tr_static_init, evaluated at compile time.
constexpr Tables make_tables() {
    Tables t{};
    const uint8_t el[kLengthCodes] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
    const uint8_t ed[kDCodes] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
    const uint8_t eb[kBLCodes] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
    const uint8_t bo[kBLCodes] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    for (int k = 0; k < kLengthCodes; k++) t.extra_lbits[k] = el[k];
    for (int k = 0; k < kDCodes; k++) t.extra_dbits[k] = ed[k];
    for (int k = 0; k < kBLCodes; k++) t.extra_blbits[k] = eb[k], t.bl_order[k] = bo[k];
    int length = 0, code = 0;
    for (code = 0; code < kLengthCodes - 1; code++) {
        t.base_length[code] = (uint16_t)length;
        for (int n = 0; n < (1 << el[code]); n++) t.length_code[length++] = (uint8_t)code;
    }
    t.length_code[length - 1] = (uint8_t)code;
    t.base_length[kLengthCodes - 1] = 0;
    int dist = 0;
    for (code = 0; code < 16; code++) {
        t.base_dist[code] = (uint16_t)dist;
        for (int n = 0; n < (1 << ed[code]); n++) t.dist_code[dist++] = (uint8_t)code;
    }
    dist >>= 7;
    for (; code < kDCodes; code++) {
        t.base_dist[code] = (uint16_t)(dist << 7);
        for (int n = 0; n < (1 << (ed[code] - 7)); n++) t.dist_code[256 + dist++] = (uint8_t)code;
    }
    uint16_t bl_count[kMaxBits + 1] = {};
    int n = 0;
    while (n <= 143) t.static_ltree[n++].dl = 8, bl_count[8]++;
    while (n <= 255) t.static_ltree[n++].dl = 9, bl_count[9]++;
    while (n <= 279) t.static_ltree[n++].dl = 7, bl_count[7]++;
    while (n <= 287) t.static_ltree[n++].dl = 8, bl_count[8]++;
    uint16_t next_code[kMaxBits + 1] = {};
    unsigned c = 0;
    for (int bits = 1; bits <= kMaxBits; bits++) {
        c = (c + bl_count[bits - 1]) << 1;
        next_code[bits] = (uint16_t)c;
    }
    for (n = 0; n <= kLCodes + 1; n++) {
        int len = t.static_ltree[n].dl;
        t.static_ltree[n].fc = (uint16_t)bi_reverse_c(next_code[len]++, len);
    }
    for (n = 0; n < kDCodes; n++) {
        t.static_dtree[n].dl = 5;
        t.static_dtree[n].fc = (uint16_t)bi_reverse_c((unsigned)n, 5);
    }
    return t;
}

PMC_HD inline unsigned d_code(const Tables &T, unsigned dist) {
    return dist < 256 ? T.dist_code[dist] : T.dist_code[256 + (dist >> 7)];
}

// Closed forms of trees.c's _length_code / base_length / extra_lbits and _dist_code / base_dist /
// extra_dbits (RFC 1951 3.2.5; equal to the tables entry for entry, checked by the parity tests).
// They replace per-lane indexed loads from constant memory with a few VALU operations.
PMC_HD inline unsigned log2_floor(unsigned x) { return 31u - (unsigned)__builtin_clz(x | 1u); }
// length code (0..28) of lc = match length - 3 (0..255)
PMC_HD inline unsigned len_code_cf(unsigned lc) {
    if (lc < 8) return lc;
    if (lc == 255) return 28;
    const unsigned lx = log2_floor(lc) - 2;
    return 4 * lx + (lc >> lx);
}
PMC_HD inline unsigned len_extra_cf(unsigned c) { return c < 8 || c == 28 ? 0u : (c - 4) >> 2; }
PMC_HD inline unsigned len_base_cf(unsigned c) {
    return c < 8 ? c : c == 28 ? 255u : (4 + (c & 3)) << ((c - 4) >> 2);
}
// distance code (0..29) of dm = distance - 1 (0..32767)
PMC_HD inline unsigned dist_code_cf(unsigned dm) {
    if (dm < 4) return dm;
    const unsigned k = log2_floor(dm);
    return 2 * k + ((dm >> (k - 1)) & 1);
}
PMC_HD inline unsigned dist_extra_cf(unsigned dc) { return dc < 4 ? 0u : (dc >> 1) - 1; }
PMC_HD inline unsigned dist_base_cf(unsigned dc) { return dc < 4 ? dc : (2 + (dc & 1)) << ((dc >> 1) - 1); }
// trees.c bl_order[i] (= inflate's code-length order) from two packed constants of 5-bit fields
PMC_HD inline unsigned bl_order_cf(int i) {
    return i < 12 ? (unsigned)(0x22caa324e804a30ull >> (5 * i)) & 31u : (unsigned)(0x3c2e1346cull >> (5 * (i - 12))) & 31u;
}

// Per-wave Huffman workspace (4448 bytes).  Lives in LDS on the GPU.
struct Trees {
    CtData ltree[kHeapSize];       // dyn_ltree
    CtData dtree[2 * kDCodes + 1]; // dyn_dtree
    CtData bltree[2 * kBLCodes + 1];
    uint16_t heap[2 * kLCodes + 1];
    uint8_t depth[2 * kLCodes + 1];
    uint8_t pad_[3];
    uint16_t bl_count[kMaxBits + 1];
};

// Result of building one block's trees (_tr_flush_block up to the type decision).
struct BlockPlan {
    uint32_t opt_lenb, static_lenb;
    int l_max, d_max, max_blindex;
};

PMC_HD inline void init_block(Trees &s) {
    for (int n = 0; n < kLCodes; n++) s.ltree[n].fc = 0;
    for (int n = 0; n < kDCodes; n++) s.dtree[n].fc = 0;
    for (int n = 0; n < kBLCodes; n++) s.bltree[n].fc = 0;
    s.ltree[kEndBlock].fc = 1;
}

struct TreeDesc {
    CtData *tree;
    const CtData *stree; // nullptr for the bit-length tree
    const uint8_t *extra;
    int extra_base, elems, max_length;
};

PMC_HD inline bool smaller(const CtData *tree, int n, int m, const uint8_t *depth) {
    return tree[n].fc < tree[m].fc || (tree[n].fc == tree[m].fc && depth[n] <= depth[m]);
}

PMC_HD inline void pqdownheap(Trees &s, int heap_len, const CtData *tree, int k) {
    int v = s.heap[k];
    int j = k << 1;
    while (j <= heap_len) {
        if (j < heap_len && smaller(tree, s.heap[j + 1], s.heap[j], s.depth)) j++;
        if (smaller(tree, v, s.heap[j], s.depth)) break;
        s.heap[k] = s.heap[j];
        k = j;
        j <<= 1;
    }
    s.heap[k] = (uint16_t)v;
}

PMC_HD inline void gen_bitlen(Trees &s, const TreeDesc &d, int max_code, int heap_max, uint64_t &opt_len,
                              uint64_t &static_len) {
    CtData *tree = d.tree;
    int h, n, m, bits, xbits, overflow = 0;
    for (bits = 0; bits <= kMaxBits; bits++) s.bl_count[bits] = 0;
    tree[s.heap[heap_max]].dl = 0;
    for (h = heap_max + 1; h < kHeapSize; h++) {
        n = s.heap[h];
        bits = tree[tree[n].dl].dl + 1;
        if (bits > d.max_length) bits = d.max_length, overflow++;
        tree[n].dl = (uint16_t)bits;
        if (n > max_code) continue;
        s.bl_count[bits]++;
        xbits = 0;
        if (n >= d.extra_base) xbits = d.extra[n - d.extra_base];
        unsigned f = tree[n].fc;
        opt_len += (uint64_t)f * (unsigned)(bits + xbits);
        if (d.stree) static_len += (uint64_t)f * (unsigned)(d.stree[n].dl + xbits);
    }
    if (overflow == 0) return;
    do {
        bits = d.max_length - 1;
        while (s.bl_count[bits] == 0) bits--;
        s.bl_count[bits]--;
        s.bl_count[bits + 1] += 2;
        s.bl_count[d.max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    for (bits = d.max_length; bits != 0; bits--) {
        n = s.bl_count[bits];
        while (n != 0) {
            m = s.heap[--h];
            if (m > max_code) continue;
            if ((unsigned)tree[m].dl != (unsigned)bits) {
                opt_len += ((uint64_t)bits - tree[m].dl) * tree[m].fc;
                tree[m].dl = (uint16_t)bits;
            }
            n--;
        }
    }
}

PMC_HD inline void gen_codes(CtData *tree, int max_code, const uint16_t *bl_count) {
    uint16_t next_code[kMaxBits + 1];
    unsigned code = 0;
    for (int bits = 1; bits <= kMaxBits; bits++) {
        code = (code + bl_count[bits - 1]) << 1;
        next_code[bits] = (uint16_t)code;
    }
    for (int n = 0; n <= max_code; n++) {
        int len = tree[n].dl;
        if (len == 0) continue;
        unsigned c = next_code[len]++, r = 0;
        for (int k = 0; k < len; k++) r = (r << 1) | ((c >> k) & 1);
        tree[n].fc = (uint16_t)r;
    }
}

// build_tree; returns max_code.
PMC_HD inline int build_tree(Trees &s, const TreeDesc &d, uint64_t &opt_len, uint64_t &static_len) {
    CtData *tree = d.tree;
    int n, m, max_code = -1, node, heap_len = 0, heap_max = kHeapSize;
    for (n = 0; n < d.elems; n++) {
        if (tree[n].fc != 0) {
            s.heap[++heap_len] = (uint16_t)(max_code = n);
            s.depth[n] = 0;
        } else {
            tree[n].dl = 0;
        }
    }
    while (heap_len < 2) {
        node = max_code < 2 ? ++max_code : 0;
        s.heap[++heap_len] = (uint16_t)node;
        tree[node].fc = 1;
        s.depth[node] = 0;
        opt_len--;
        if (d.stree) static_len -= d.stree[node].dl;
    }
    for (n = heap_len / 2; n >= 1; n--) pqdownheap(s, heap_len, tree, n);
    node = d.elems;
    do {
        n = s.heap[1];
        s.heap[1] = s.heap[heap_len--];
        pqdownheap(s, heap_len, tree, 1);
        m = s.heap[1];
        s.heap[--heap_max] = (uint16_t)n;
        s.heap[--heap_max] = (uint16_t)m;
        tree[node].fc = (uint16_t)(tree[n].fc + tree[m].fc);
        s.depth[node] = (uint8_t)((s.depth[n] >= s.depth[m] ? s.depth[n] : s.depth[m]) + 1);
        tree[n].dl = tree[m].dl = (uint16_t)node;
        s.heap[1] = (uint16_t)node++;
        pqdownheap(s, heap_len, tree, 1);
    } while (heap_len >= 2);
    s.heap[--heap_max] = s.heap[1];
    gen_bitlen(s, d, max_code, heap_max, opt_len, static_len);
    gen_codes(tree, max_code, s.bl_count);
    return max_code;
}

PMC_HD inline void scan_tree(Trees &s, CtData *tree, int max_code) {
    int prevlen = -1, curlen, nextlen = tree[0].dl, count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    tree[max_code + 1].dl = 0xffff;
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[n + 1].dl;
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            s.bltree[curlen].fc = (uint16_t)(s.bltree[curlen].fc + count);
        } else if (curlen != 0) {
            if (curlen != prevlen) s.bltree[curlen].fc++;
            s.bltree[kRep3_6].fc++;
        } else if (count <= 10) {
            s.bltree[kRepz3_10].fc++;
        } else {
            s.bltree[kRepz11_138].fc++;
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

// Builds the three trees of the current block and computes the sizes _tr_flush_block
// compares.  Frequencies must already be in s.ltree/s.dtree (END_BLOCK counted).
PMC_HD inline BlockPlan plan_block(Trees &s, const Tables &T) {
    uint64_t opt_len = 0, static_len = 0;
    BlockPlan p;
    TreeDesc ld{s.ltree, T.static_ltree, T.extra_lbits, kLiterals + 1, kLCodes, kMaxBits};
    TreeDesc dd{s.dtree, T.static_dtree, T.extra_dbits, 0, kDCodes, kMaxBits};
    TreeDesc bd{s.bltree, nullptr, T.extra_blbits, 0, kBLCodes, kMaxBLBits};
    p.l_max = build_tree(s, ld, opt_len, static_len);
    p.d_max = build_tree(s, dd, opt_len, static_len);
    scan_tree(s, s.ltree, p.l_max);
    scan_tree(s, s.dtree, p.d_max);
    build_tree(s, bd, opt_len, static_len);
    int mbi;
    for (mbi = kBLCodes - 1; mbi >= 3; mbi--)
        if (s.bltree[T.bl_order[mbi]].dl != 0) break;
    opt_len += 3 * ((uint64_t)mbi + 1) + 5 + 5 + 4;
    p.max_blindex = mbi;
    p.opt_lenb = (uint32_t)((opt_len + 3 + 7) >> 3);
    p.static_lenb = (uint32_t)((static_len + 3 + 7) >> 3);
    if (p.static_lenb <= p.opt_lenb) p.opt_lenb = p.static_lenb;
    return p;
}

// send_tree with a caller-provided bit sink (Sink::put(value, nbits)).
template <class Sink>
PMC_HD inline void send_tree(Trees &s, Sink &out, const CtData *tree, int max_code) {
    int prevlen = -1, curlen, nextlen = tree[0].dl, count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[n + 1].dl;
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            do { out.put(s.bltree[curlen].fc, s.bltree[curlen].dl); } while (--count != 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) {
                out.put(s.bltree[curlen].fc, s.bltree[curlen].dl);
                count--;
            }
            out.put(s.bltree[kRep3_6].fc, s.bltree[kRep3_6].dl);
            out.put((unsigned)(count - 3), 2);
        } else if (count <= 10) {
            out.put(s.bltree[kRepz3_10].fc, s.bltree[kRepz3_10].dl);
            out.put((unsigned)(count - 3), 3);
        } else {
            out.put(s.bltree[kRepz11_138].fc, s.bltree[kRepz11_138].dl);
            out.put((unsigned)(count - 11), 7);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

// send_all_trees (trees.c)
template <class Sink>
PMC_HD inline void send_all_trees(Trees &s, const Tables &T, Sink &out, const BlockPlan &p) {
    int lcodes = p.l_max + 1, dcodes = p.d_max + 1, blcodes = p.max_blindex + 1;
    out.put((unsigned)(lcodes - 257), 5);
    out.put((unsigned)(dcodes - 1), 5);
    out.put((unsigned)(blcodes - 4), 4);
    for (int rank = 0; rank < blcodes; rank++) out.put(s.bltree[T.bl_order[rank]].dl, 3);
    send_tree(s, out, s.ltree, lcodes - 1);
    send_tree(s, out, s.dtree, dcodes - 1);
}

// Bits for one symbol-buffer entry (compress_block): token = dist<<16 | lc, dist==0 -> literal.
// Returns the bit pattern (LSB first) and sets nbits (<= 48).
PMC_HD inline uint64_t token_bits(const Tables &T, const CtData *ltree, const CtData *dtree, uint32_t tok,
                                  int &nbits) {
    unsigned dist = tok >> 16, lc = tok & 0xff;
    if (dist == 0) {
        nbits = ltree[lc].dl;
        return ltree[lc].fc;
    }
    unsigned code = T.length_code[lc];
    uint64_t v = ltree[code + kLiterals + 1].fc;
    int n = ltree[code + kLiterals + 1].dl;
    int extra = T.extra_lbits[code];
    v |= (uint64_t)((lc - T.base_length[code]) & ((1u << extra) - 1)) << n;
    n += extra;
    dist--;
    code = d_code(T, dist);
    v |= (uint64_t)dtree[code].fc << n;
    n += dtree[code].dl;
    extra = T.extra_dbits[code];
    v |= (uint64_t)((dist - T.base_dist[code]) & ((1u << extra) - 1)) << n;
    n += extra;
    nbits = n;
    return v;
}

} // namespace pmc
