// host_pipeline.cpp -- CPU twin of the gfx950 deflate kernel's back end (test only).
//
// Compiles poor-man-s-cache_amd/csrc/pmc_trees.hpp (the Huffman construction the kernel
// runs on lane 0, and token_bits which the kernel's lanes use to emit symbols) with g++
// and drives it the way pmc_deflate.hip does: serial lazy parse over a hash-sorted chain,
// 16383-symbol blocks, stored/fixed/dynamic choice, gzip framing.  tests/test_host_pipeline.py
// diffs the result against the golden vectors, so the device-side Huffman/emit code is
// pinned on a CPU before any GPU run.
//
// usage: host_pipeline <in> <out> [v2]   (writes the gzip member of <in> to <out>; v2 =
//        pmc_deflate_small.hip's Huffman formulation: packed-key heap, lengths from node
//        depths, closed-form per-run scan_tree/send_tree, serial fallback on overflow)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../poor-man-s-cache_amd/csrc/pmc_trees.hpp"

using namespace pmc;

static const Tables T = make_tables();

struct Bitbuf {
    std::vector<uint8_t> &out;
    uint64_t pos;
    void put(unsigned v, int n) {
        for (int k = 0; k < n; k++) {
            uint64_t p = pos + k;
            if ((p >> 3) >= out.size()) out.resize((p >> 3) + 1, 0);
            if ((v >> k) & 1) out[p >> 3] |= (uint8_t)(1u << (p & 7));
        }
        pos += n;
    }
    void put64(uint64_t v, int n) {
        for (int k = 0; k < n; k += 16) put((unsigned)(v >> k) & 0xffff, n - k < 16 ? n - k : 16);
    }
};

// ---- v2 (pmc_deflate_small.hip) algorithms, serial form -----------------------------------
// build_tree with heap entries (freq<<5|depth)<<10|node and a one-compare `smaller`, code
// lengths = node depths, canonical codes; returns overflow instead of fixing it.
struct V2Tree {
    int max_code;
    int64_t opt, stat;
    bool overflow;
    std::vector<uint32_t> code; // bitrev code | len << 16
};
static V2Tree v2_build(std::vector<uint32_t> freq, int elems, const CtData *stree, const uint8_t *extra, int base,
                       int max_length) {
    V2Tree t{};
    std::vector<uint32_t> heap(1);
    int max_code = -1;
    for (int s = 0; s < elems; s++)
        if (freq[s]) heap.push_back(((freq[s] << 5) << 10) | s), max_code = s;
    int64_t opt = 0, stat = 0;
    while (heap.size() - 1 < 2) {
        int node = max_code < 2 ? ++max_code : 0;
        heap.push_back(((1u << 5) << 10) | node);
        freq[node] = 1;
        opt -= 1;
        if (stree) stat -= stree[node].dl;
    }
    int heap_len = (int)heap.size() - 1;
    auto down = [&](int k) {
        uint32_t v = heap[k];
        int j = k << 1;
        while (j <= heap_len) {
            if (j < heap_len && (heap[j + 1] >> 10) <= (heap[j] >> 10)) j++;
            if ((v >> 10) <= (heap[j] >> 10)) break;
            heap[k] = heap[j];
            k = j;
            j <<= 1;
        }
        heap[k] = v;
    };
    for (int n = heap_len / 2; n >= 1; n--) down(n);
    std::vector<int> dad(2 * elems + 2, -1);
    int node = elems;
    do {
        uint32_t n = heap[1];
        heap[1] = heap[heap_len--];
        down(1);
        uint32_t m = heap[1];
        uint32_t kn = n >> 10, km = m >> 10, dn = kn & 31, dm = km & 31;
        uint32_t d = (dn >= dm ? dn : dm) + 1;
        dad[n & 1023] = dad[m & 1023] = node;
        heap[1] = (((((kn >> 5) + (km >> 5)) << 5) | d) << 10) | node;
        node++;
        down(1);
    } while (heap_len >= 2);
    std::vector<uint32_t> len(elems, 0);
    bool over = false;
    int64_t po = 0, ps = 0;
    for (int s = 0; s <= max_code; s++) {
        if (!freq[s]) continue;
        uint32_t d = 0;
        for (int x = s; dad[x] >= 0; x = dad[x]) d++;
        len[s] = d;
        over |= d > (uint32_t)max_length;
        uint32_t xb = s >= base ? extra[s - base] : 0;
        po += (int64_t)freq[s] * (d + xb);
        if (stree) ps += (int64_t)freq[s] * (stree[s].dl + xb);
    }
    t.overflow = over;
    t.opt = opt + po;
    t.stat = stat + ps;
    t.max_code = max_code;
    uint32_t bl_count[16] = {}, next_code[16] = {}, code = 0;
    for (int s = 0; s <= max_code; s++) bl_count[len[s]]++;
    bl_count[0] = 0;
    for (int L = 1; L <= 15; L++) {
        code = (code + bl_count[L - 1]) << 1;
        next_code[L] = code;
    }
    t.code.assign(elems, 0);
    for (int s = 0; s <= max_code; s++) {
        uint32_t L = len[s];
        if (!L) continue;
        uint32_t c = next_code[L]++, r = 0;
        for (uint32_t k = 0; k < L; k++) r = (r << 1) | ((c >> k) & 1);
        t.code[s] = r | (L << 16);
    }
    return t;
}
// closed-form scan_tree / send_tree of one maximal run (v, R)
template <class F>
static void v2_run(uint32_t v, uint32_t R, F put) {
    if (v) {
        uint32_t c1 = R < 7 ? R : 7, rem = R - c1, full = rem / 6, last = rem % 6;
        if (c1 < 4) {
            for (uint32_t k = 0; k < c1; k++) put(v, 0, 0);
        } else {
            put(v, 0, 0);
            put(16, c1 - 4, 2);
        }
        for (uint32_t k = 0; k < full; k++) put(16, 3, 2);
        if (last) {
            if (last < 3)
                for (uint32_t k = 0; k < last; k++) put(v, 0, 0);
            else
                put(16, last - 3, 2);
        }
    } else {
        uint32_t full = R / 138, last = R % 138;
        for (uint32_t k = 0; k < full; k++) put(18, 127, 7);
        if (last) {
            if (last < 3)
                for (uint32_t k = 0; k < last; k++) put(0, 0, 0);
            else if (last <= 10)
                put(17, last - 3, 3);
            else
                put(18, last - 11, 7);
        }
    }
}
template <class F>
static void v2_runs(const std::vector<uint32_t> &code, int max_code, F on_run) {
    int s = 0;
    while (s <= max_code) {
        uint32_t v = code[s] >> 16;
        int e = s + 1;
        while (e <= max_code && (code[e] >> 16) == v) e++;
        on_run(v, (uint32_t)(e - s));
        s = e;
    }
}

static uint32_t crc32(const uint8_t *p, size_t n) {
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) {
        c ^= p[i];
        for (int k = 0; k < 8; k++) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    }
    return ~c;
}

int main(int argc, char **argv) {
    if (argc != 3 && argc != 4) return 2;
    const bool use_v2 = argc == 4 && strcmp(argv[3], "v2") == 0;
    FILE *f = fopen(argv[1], "rb");
    std::vector<uint8_t> in;
    int ch;
    while ((ch = fgetc(f)) != EOF) in.push_back((uint8_t)ch);
    fclose(f);
    const uint64_t len = in.size();
    std::vector<uint8_t> b(in);
    b.resize(len + 64, 0);
    // hash + stable sort (the kernel: 3 x 5-bit LSD radix passes)
    const uint64_t npos = len >= 3 ? len - 2 : 0;
    std::vector<uint64_t> S(npos), rank(npos);
    {
        std::vector<uint32_t> cnt(32769, 0);
        std::vector<uint32_t> h(npos);
        for (uint64_t p = 0; p < npos; p++) {
            h[p] = ((uint32_t)b[p] << 10 ^ (uint32_t)b[p + 1] << 5 ^ b[p + 2]) & 0x7fff;
            cnt[h[p] + 1]++;
        }
        for (int k = 0; k < 32768; k++) cnt[k + 1] += cnt[k];
        for (uint64_t p = 0; p < npos; p++) {
            uint32_t r = cnt[h[p]]++;
            S[r] = (uint64_t)h[p] << 32 | p;
            rank[p] = r;
        }
    }
    auto search = [&](uint64_t i, uint32_t b0, uint64_t B, uint64_t *qo) -> uint32_t {
        uint32_t C = b0 >= 32 ? 1024 : 4096;
        uint32_t nice = (uint32_t)((len - i) < 258 ? (len - i) : 258);
        int64_t r = (int64_t)rank[i];
        uint64_t hi = S[r] >> 32;
        uint32_t ex = 0, best = 0;
        for (int64_t k = r - 1; k >= 0; k--) {
            if ((S[k] >> 32) != hi) break;
            uint64_t q = S[k] & 0xffffffffull, d = i - q;
            if (q <= B || (ex == 0 ? d > 32506 : d >= 32506) || ex >= C) break;
            ex++;
            uint32_t l = 0;
            while (l < nice && b[i + l] == b[q + l]) l++;
            if (l > best) {
                best = l;
                *qo = q;
                if (l >= nice) break;
            }
        }
        return best > b0 ? best : 0;
    };
    // v2 small-value path (pmc_deflate_small.hip match_all + search): every position's walk
    // over its first kPre chain candidates is done up front (best | q << 9 | cut << 31);
    // the parse resumes cut walks at candidate kPre.
    const uint32_t kPre = 32; // = 64 / PMC_GROUP (pmc_deflate_small.hip)
    const bool pre = use_v2 && len <= 16382;
    std::vector<uint32_t> M(pre ? npos : 0);
    for (uint64_t i = 0; pre && i < npos; i++) {
        uint32_t nice = (uint32_t)((len - i) < 258 ? (len - i) : 258), best = 0, bq = 0, s = 0;
        int64_t k = (int64_t)rank[i] - 1;
        for (; s < kPre && k >= 0; s++, k--) {
            uint64_t q = S[k] & 0xffffffffull;
            if (q == 0 || (S[k] >> 32) != (S[rank[i]] >> 32)) break;
            uint32_t l = 0;
            while (l < nice && b[i + l] == b[q + l]) l++;
            if (l > best) {
                best = l;
                bq = (uint32_t)q;
                if (best >= nice) break;
            }
        }
        M[i] = best | bq << 9 | ((s == kPre && best < nice) ? 1u << 31 : 0u);
    }
    auto search_pre = [&](uint64_t i, uint32_t b0, uint64_t *qo) -> uint32_t {
        uint32_t best = M[i] & 511;
        *qo = (M[i] >> 9) & 0x3fff;
        if (M[i] >> 31) {
            uint32_t C = b0 >= 32 ? 1024 : 4096;
            uint32_t nice = (uint32_t)((len - i) < 258 ? (len - i) : 258);
            int64_t r = (int64_t)rank[i];
            uint32_t ex = kPre;
            for (int64_t k = r - 1 - kPre; k >= 0 && ex < C; k--, ex++) {
                uint64_t q = S[k] & 0xffffffffull;
                if ((S[k] >> 32) != (S[r] >> 32) || q == 0) break;
                uint32_t l = 0;
                while (l < nice && b[i + l] == b[q + l]) l++;
                if (l > best) {
                    best = l;
                    *qo = q;
                    if (l >= nice) break;
                }
            }
        }
        return best > b0 ? best : 0;
    };
    std::vector<uint8_t> out(10, 0);
    const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 2, 3};
    memcpy(out.data(), hdr, 10);
    Bitbuf bb{out, 80};
    Trees *tr = (Trees *)calloc(1, sizeof(Trees));
    init_block(*tr);
    std::vector<uint32_t> tok;
    uint64_t block_start = 0, B = 0, wend = 0, i = 0;
    auto flush_v2 = [&](uint64_t end, bool last) -> bool {
        std::vector<uint32_t> lf(286), df(30), blf(19, 0);
        for (int s = 0; s < 286; s++) lf[s] = tr->ltree[s].fc;
        for (int s = 0; s < 30; s++) df[s] = tr->dtree[s].fc;
        V2Tree tl = v2_build(lf, 286, T.static_ltree, T.extra_lbits, 257, 15);
        V2Tree td = v2_build(df, 30, T.static_dtree, T.extra_dbits, 0, 15);
        if (tl.overflow || td.overflow) return false;
        auto count = [&](uint32_t v, uint32_t R) { v2_run(v, R, [&](uint32_t c, uint32_t, uint32_t) { blf[c]++; }); };
        v2_runs(tl.code, tl.max_code, count);
        v2_runs(td.code, td.max_code, count);
        V2Tree tb = v2_build(blf, 19, nullptr, T.extra_blbits, 0, 7);
        if (tb.overflow) return false;
        int mbi;
        for (mbi = 18; mbi >= 3; mbi--)
            if ((tb.code[T.bl_order[mbi]] >> 16) != 0) break;
        int64_t opt = tl.opt + td.opt + tb.opt + 3 * ((int64_t)mbi + 1) + 14, stat = tl.stat + td.stat;
        uint64_t optb = ((uint64_t)opt + 10) >> 3, statb = ((uint64_t)stat + 10) >> 3;
        if (statb <= optb) optb = statb;
        uint64_t stored_len = end - block_start;
        if (stored_len + 4 <= optb && block_start >= B) {
            bb.put((0u << 1) + last, 3);
            bb.pos = (bb.pos + 7) & ~7ull;
            bb.put((unsigned)stored_len & 0xffff, 16);
            bb.put((~(unsigned)stored_len) & 0xffff, 16);
            for (uint64_t k = 0; k < stored_len; k++) bb.put(b[block_start + k], 8);
        } else {
            bool fixed = statb == optb;
            std::vector<uint32_t> lc(288), dc(32);
            for (int s = 0; s < 286; s++)
                lc[s] = fixed ? (T.static_ltree[s].fc | (uint32_t)T.static_ltree[s].dl << 16) : tl.code[s];
            for (int s = 0; s < 30; s++)
                dc[s] = fixed ? (T.static_dtree[s].fc | (uint32_t)T.static_dtree[s].dl << 16) : td.code[s];
            bb.put(((fixed ? 1u : 2u) << 1) + last, 3);
            if (!fixed) {
                bb.put(tl.max_code + 1 - 257, 5);
                bb.put(td.max_code + 1 - 1, 5);
                bb.put(mbi + 1 - 4, 4);
                for (int k = 0; k <= mbi; k++) bb.put(tb.code[T.bl_order[k]] >> 16, 3);
                auto send = [&](uint32_t v, uint32_t R) {
                    v2_run(v, R, [&](uint32_t c, uint32_t xv, uint32_t xn) {
                        bb.put(tb.code[c] & 0xffff, tb.code[c] >> 16);
                        bb.put(xv, xn);
                    });
                };
                v2_runs(tl.code, tl.max_code, send);
                v2_runs(td.code, td.max_code, send);
            }
            for (uint32_t t : tok) {
                uint32_t dist = t >> 16, l8 = t & 0xff;
                if (!dist) {
                    bb.put(lc[l8] & 0xffff, lc[l8] >> 16);
                } else {
                    uint32_t code = T.length_code[l8];
                    bb.put(lc[code + 257] & 0xffff, lc[code + 257] >> 16);
                    bb.put((l8 - T.base_length[code]) & ((1u << T.extra_lbits[code]) - 1), T.extra_lbits[code]);
                    uint32_t dm = dist - 1, dcd = d_code(T, dm);
                    bb.put(dc[dcd] & 0xffff, dc[dcd] >> 16);
                    bb.put((dm - T.base_dist[dcd]) & ((1u << T.extra_dbits[dcd]) - 1), T.extra_dbits[dcd]);
                }
            }
            bb.put(lc[256] & 0xffff, lc[256] >> 16);
            if (last) bb.pos = (bb.pos + 7) & ~7ull;
        }
        init_block(*tr);
        tok.clear();
        block_start = end;
        return true;
    };
    auto flush = [&](uint64_t end, bool last) {
        if (use_v2 && flush_v2(end, last)) return;
        BlockPlan p = plan_block(*tr, T);
        uint64_t stored_len = end - block_start;
        if (stored_len + 4 <= p.opt_lenb && block_start >= B) {
            bb.put((0u << 1) + last, 3);
            bb.pos = (bb.pos + 7) & ~7ull;
            bb.put((unsigned)stored_len & 0xffff, 16);
            bb.put((~(unsigned)stored_len) & 0xffff, 16);
            for (uint64_t k = 0; k < stored_len; k++) bb.put(b[block_start + k], 8);
        } else {
            bool fixed = p.static_lenb == p.opt_lenb;
            const CtData *lt = fixed ? T.static_ltree : tr->ltree;
            const CtData *dt = fixed ? T.static_dtree : tr->dtree;
            bb.put(((fixed ? 1u : 2u) << 1) + last, 3);
            if (!fixed) send_all_trees(*tr, T, bb, p);
            for (uint32_t t : tok) {
                int nb = 0;
                uint64_t v = token_bits(T, lt, dt, t, nb);
                bb.put64(v, nb);
            }
            bb.put(lt[kEndBlock].fc, lt[kEndBlock].dl);
            if (last) bb.pos = (bb.pos + 7) & ~7ull;
        }
        init_block(*tr);
        tok.clear();
        block_start = end;
    };
    auto emit = [&](uint32_t t) {
        tok.push_back(t);
        uint32_t dist = t >> 16, lc = t & 0xff;
        if (!dist) tr->ltree[lc].fc++;
        else {
            tr->ltree[T.length_code[lc] + kLiterals + 1].fc++;
            tr->dtree[d_code(T, dist - 1)].fc++;
        }
    };
    uint32_t match_length = 2, prev_length;
    uint64_t match_start = 0, prev_match;
    bool avail = false;
    if (pre) {
        // v2 on-demand parse (pmc_deflate_small.hip parse_ondemand()): with no pending match,
        // positions without chain candidates are skipped as literals; every other position
        // steps deflate_slow exactly with longest_match = M (resumed by search_pre if cut).
        auto has_cand = [&](uint64_t x) {
            if (x >= npos || rank[x] == 0) return false;
            uint64_t q = S[rank[x] - 1] & 0xffffffffull;
            return q != 0 && (S[rank[x] - 1] >> 32) == (S[rank[x]] >> 32);
        };
        uint64_t ii = 0;
        uint32_t ml = 2;
        uint64_t ms = 0;
        bool av = false;
        while (ii < len) {
            if (ml == 2) {
                uint64_t j = ii;
                while (j < npos && !has_cand(j)) j++;
                if (j >= npos) j = len;
                if (j > ii) {
                    uint64_t from = av ? ii - 1 : ii;
                    for (uint64_t k = from; k + 1 < j; k++) emit(b[k]);
                    av = true;
                    ii = j;
                    if (ii >= len) break;
                }
            }
            uint32_t pl = ml;
            uint64_t pm = ms;
            ml = 2;
            if (ii < npos && pl < 258 && has_cand(ii)) {
                uint64_t q = 0;
                uint32_t m = search_pre(ii, pl, &q);
                if (m) {
                    ml = m;
                    ms = q;
                    if (m == 3 && ii - q > 4096) ml = 2;
                }
            }
            if (pl >= 3 && ml <= pl) {
                emit((uint32_t)(ii - 1 - pm) << 16 | (pl - 3));
                ii += pl - 1;
                ml = 2;
                av = false;
            } else if (av) {
                emit(b[ii - 1]);
                ii++;
            } else {
                av = true;
                ii++;
            }
        }
        if (av) emit(b[ii - 1]);
        i = len;
        avail = false;
    }
    for (; !pre;) {
        if (wend - i < 262) {
            do {
                if (i - B >= 32768 + 32506) B += 32768;
                if (wend == len) break;
                wend = len < B + 65536 ? len : B + 65536;
            } while (wend - i < 262 && wend < len);
            if (wend == i) break;
        }
        prev_length = match_length;
        prev_match = match_start;
        match_length = 2;
        if (i + 3 <= len && prev_length < 258) {
            uint64_t q = 0;
            uint32_t m = pre ? search_pre(i, prev_length, &q) : search(i, prev_length, B, &q);
            if (m) {
                match_length = m;
                match_start = q;
                if (m == 3 && i - q > 4096) match_length = 2;
            }
        }
        if (prev_length >= 3 && match_length <= prev_length) {
            emit((uint32_t)(i - 1 - prev_match) << 16 | (prev_length - 3));
            i += prev_length - 1;
            avail = false;
            match_length = 2;
            if (tok.size() == 16383) flush(i, false);
        } else if (avail) {
            emit(b[i - 1]);
            if (tok.size() == 16383) flush(i, false);
            i++;
        } else {
            avail = true;
            i++;
        }
    }
    if (avail) emit(b[i - 1]);
    flush(i, true);
    out.resize(bb.pos >> 3);
    uint32_t c = crc32(in.data(), len);
    for (int k = 0; k < 4; k++) out.push_back((uint8_t)(c >> (8 * k)));
    for (int k = 0; k < 4; k++) out.push_back((uint8_t)(len >> (8 * k)));
    FILE *g = fopen(argv[2], "wb");
    fwrite(out.data(), 1, out.size(), g);
    fclose(g);
    free(tr);
    return 0;
}
