// pmc_deflate_large.hip -- gzip level-9 compression of values above the split pipeline's large pass
// (deflate_big_limit(), ~31.8 KB): the reference accepts values up to 512 MiB
// (/root/reference/src/server/constants.hpp:8) and compresses each with zlib 1.2.11 deflate_slow
// (gzip_compressor.cpp:12,38).  Output is bit-identical to it.
//
// A long value is one serial lazy parse in zlib.  Here it is cut into segments of kLvSeg positions:
//
//  1. sort (lv_sort_*_kernel, lv_rank_kernel): every position of the value is sorted stably by its
//     15-bit hash into S in HBM (2-pass LSD radix, 8 + 7 bits, per-chunk digit histograms, one scan
//     per value, stable scatter by ballot match masks -- no reliance on atomic lane order), with the
//     rank array R (R[S[k]] = k) and HC[x] = zlib would search at x (the nearest same-hash earlier
//     position exists, is not NIL position 0 and lies within MAX_DIST).  zlib's chain of x is then the
//     run S[R[x] - 1], S[R[x] - 2], ... of equal hash, cut at MAX_DIST (deflate_dp.c restates this).
//     Window slides never change a match: after the first slide every search position lies more than
//     MAX_DIST past the window base, so the base's NIL only ever hides candidates the distance limit
//     hides anyway.
//  2. parse (lv_parse_kernel): one wave per segment runs deflate_slow from a fresh state at the
//     segment start over global memory, longest_match 64 chain candidates per step (lane per
//     candidate, nearest wins ties), and on through kLvOverlap positions of the next segment.  At each
//     loop-top position of its first and its last kLvOverlap positions it records the parse state
//     (fresh after a match / a literal pending, both with no pending match) and its token count.
//  3. stitch (lv_stitch_kernel): the first segment's parse is exact.  If segment j's parse is exact
//     from some position on, the first position of the next segment's start region where both parses
//     recorded the same state is a point from which they are identical (the state there is the whole
//     of deflate_slow's state: chains depend on the input only); segment j's tokens end there and
//     segment j + 1's begin there.  A boundary without such a position (not seen on any input so far:
//     JSON converges within ~60 bytes, at most 300) sends the value to the HBM kernel.
//  4. emit (deflate_lv_emit_kernel, pmc_deflate.hip): one wave per value streams the stitched tokens
//     in zlib's 16383-symbol blocks through the general kernel's _tr_flush_block.
#include <hip/hip_runtime.h>

#include "pmc_device.hpp"
#include "pmc_kernels.hpp"

namespace pmc {

constexpr uint32_t kLvMaxDist = 32768 - 262, kLvTooFar = 4096;

__device__ __forceinline__ uint32_t lv_hash(uint32_t w) {
    return ((w & 0xff) << 10 ^ ((w >> 8) & 0xff) << 5 ^ ((w >> 16) & 0xff)) & 0x7fffu;
}

// The value's bytes, read in place from the batch: only dwords that hold at least one byte of the
// value are loaded (bytes past its end read as whatever shares their dword, never used: every
// comparison is capped at the value's end).  (Clamping the address instead of predicating the load --
// unconditional loads, no exec-masked branch per dword -- measured 3 % slower in round 5.)
struct LvBytes {
    const uint8_t *base;
    uint32_t len;
    __device__ uint32_t dw(uintptr_t a) const { // a: dword-aligned address
        return a < (uintptr_t)(base + len) ? *(PMC_GLB const uint32_t *)a : 0u;
    }
    __device__ uint32_t load4(uint32_t p) const {
        const uintptr_t a = (uintptr_t)(base + p), a0 = a & ~(uintptr_t)3;
        return __builtin_amdgcn_alignbyte(dw(a0 + 4), dw(a0), (uint32_t)(a & 3));
    }
    __device__ void load16(uint32_t p, uint64_t &lo, uint64_t &hi) const {
        const uintptr_t a = (uintptr_t)(base + p), a0 = a & ~(uintptr_t)3;
        const uint32_t sh = (uint32_t)(a & 3);
        const uint32_t w0 = dw(a0), w1 = dw(a0 + 4), w2 = dw(a0 + 8), w3 = dw(a0 + 12), w4 = dw(a0 + 16);
        lo = (uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32 | __builtin_amdgcn_alignbyte(w1, w0, sh);
        hi = (uint64_t)__builtin_amdgcn_alignbyte(w4, w3, sh) << 32 | __builtin_amdgcn_alignbyte(w3, w2, sh);
    }
    __device__ uint32_t byte(uint32_t p) const { return base[p]; }
};

__device__ __forceinline__ LvBytes lv_bytes(const LargeArgs &a, uint32_t ov) {
    const uint32_t v = a.lv_val[ov];
    return LvBytes{a.src + a.src_off[v], a.src_len[v]};
}
__device__ __forceinline__ uint32_t lv_npos(uint32_t len) { return len >= 3 ? len - 2 : 0; }

// ---- 1. sort --------------------------------------------------------------------------------------
// chunk c of value ov: positions (or, in pass 1, pass-0 output slots) [c0, c1) of the value
struct LvChunk {
    uint32_t ov, c0, c1;
    uint64_t pb;
};
__device__ __forceinline__ LvChunk lv_chunk(const LargeArgs &a, uint32_t c, uint32_t npos_of_ov_len) {
    LvChunk k;
    k.ov = a.ch_val[c];
    k.c0 = (c - a.lv_ch0[k.ov]) * kLvChunk;
    k.c1 = k.c0 + kLvChunk < npos_of_ov_len ? k.c0 + kLvChunk : npos_of_ov_len;
    k.pb = a.lv_pbase[k.ov];
    return k;
}
__device__ __forceinline__ uint32_t lv_digit(uint32_t h, int pass) { return pass ? h >> 8 : h & 255u; }

// digit histogram of one chunk (one wave per chunk, 4 per block)
__global__ void __launch_bounds__(256) lv_sort_hist_kernel(LargeArgs a, int pass) {
    __shared__ uint32_t cnt[4][256];
    const uint32_t wib = threadIdx.x / 64, l = (uint32_t)lane_id();
    for (uint64_t c = (uint64_t)blockIdx.x * 4 + wib; c < a.nch; c += (uint64_t)gridDim.x * 4) {
        const uint32_t ov = a.ch_val[c];
        const LvBytes B = lv_bytes(a, ov);
        const LvChunk k = lv_chunk(a, (uint32_t)c, lv_npos(B.len));
        for (uint32_t d = l; d < 256; d += 64) cnt[wib][d] = 0;
        wave_sync();
        for (uint32_t x = k.c0 + l; x < k.c1; x += 64) {
            const uint32_t p = pass ? a.tmp[k.pb + x] : x;
            lds_add(to_lds<uint32_t>(&cnt[wib][lv_digit(lv_hash(B.load4(p)), pass)]), 1u);
        }
        wave_sync();
        for (uint32_t d = l; d < 256; d += 64) a.hist[c * 256 + d] = cnt[wib][d];
        wave_sync();
    }
}

// per value: hist[c][d] -> the chunk's first slot for digit d (digit-major, chunks in order)
__global__ void __launch_bounds__(256) lv_sort_scan_kernel(LargeArgs a) {
    __shared__ uint32_t tot[256];
    const uint32_t d = threadIdx.x;
    for (uint32_t ov = blockIdx.x; ov < a.nv; ov += gridDim.x) {
        const uint32_t c0 = a.lv_ch0[ov], c1 = a.lv_ch0[ov + 1];
        uint32_t run = 0;
        for (uint32_t c = c0; c < c1; c++) {
            const uint32_t h = a.hist[(uint64_t)c * 256 + d];
            a.hist[(uint64_t)c * 256 + d] = run;
            run += h;
        }
        tot[d] = run;
        __syncthreads();
        // exclusive scan of the 256 digit totals (thread 0; 256 adds)
        if (d == 0) {
            uint32_t s = 0;
            for (int k = 0; k < 256; k++) {
                const uint32_t t = tot[k];
                tot[k] = s;
                s += t;
            }
        }
        __syncthreads();
        const uint32_t base = tot[d];
        for (uint32_t c = c0; c < c1; c++) a.hist[(uint64_t)c * 256 + d] += base;
        __syncthreads();
    }
}

// stable scatter: a chunk's entries in order; within 64 of them a lane's rank among the lanes of its
// digit comes from a match mask (one ballot per digit bit), the digit's slot counter from LDS
__global__ void __launch_bounds__(256) lv_sort_scatter_kernel(LargeArgs a, int pass) {
    __shared__ uint32_t cur[4][256];
    const uint32_t wib = threadIdx.x / 64, l = (uint32_t)lane_id();
    const int nbits = pass ? 7 : 8;
    for (uint64_t c = (uint64_t)blockIdx.x * 4 + wib; c < a.nch; c += (uint64_t)gridDim.x * 4) {
        const uint32_t ov = a.ch_val[c];
        const LvBytes B = lv_bytes(a, ov);
        const LvChunk k = lv_chunk(a, (uint32_t)c, lv_npos(B.len));
        for (uint32_t d = l; d < 256; d += 64) cur[wib][d] = a.hist[c * 256 + d];
        wave_sync();
        uint32_t *dst = pass ? a.S : a.tmp;
        for (uint32_t x0 = k.c0; x0 < k.c1; x0 += 64) {
            const uint32_t x = x0 + l;
            const bool in = x < k.c1;
            const uint32_t p = in ? (pass ? a.tmp[k.pb + x] : x) : 0u;
            const uint32_t d = in ? lv_digit(lv_hash(B.load4(p)), pass) : 0u;
            uint64_t m = ballot(in);
            for (int bt = 0; bt < nbits; bt++) {
                const uint64_t bb = ballot(((d >> bt) & 1u) != 0);
                m &= ((d >> bt) & 1u) ? bb : ~bb;
            }
            const uint32_t rank = popc_lt(m), cntd = (uint32_t)__builtin_popcountll(m);
            const uint32_t at = in ? cur[wib][d] : 0u;
            wave_sync();
            if (in) dst[k.pb + at + rank] = p;
            if (in && rank + 1 == cntd) cur[wib][d] = at + cntd; // (the digit's highest lane)
            wave_sync();
        }
    }
}

// R[S[k]] = k and HC[x]: 0 if zlib does not search at x, else x's chain length capped at 255 (the
// same-hash entries before x in S, less NIL position 0, which the stable sort puts first in its run).
// zlib searches at x iff its nearest earlier same-hash position (S[R[x] - 1]) exists, is not NIL and
// lies within MAX_DIST (deflate.c: hash_head != NIL && strstart - hash_head <= MAX_DIST).  The count
// lets the parse's longest_match take the first 255 chain entries without loading their bytes to test
// the hash.  A chunk's wave carries the run start across its 64-entry steps; the run start of the
// chunk's first entry is found by looking back up to 256 entries (a longer run caps the count anyway).
__global__ void __launch_bounds__(256) lv_rank_kernel(LargeArgs a) {
    const uint32_t wib = threadIdx.x / 64, l = (uint32_t)lane_id();
    for (uint64_t c = (uint64_t)blockIdx.x * 4 + wib; c < a.nch; c += (uint64_t)gridDim.x * 4) {
        const uint32_t ov = a.ch_val[c];
        const LvBytes B = lv_bytes(a, ov);
        const LvChunk k = lv_chunk(a, (uint32_t)c, lv_npos(B.len));
        // run start of entry c0 - 1 (the carry into the first step), or c0 when c0 starts the value
        uint32_t prs = k.c0, ph = 0xffffffffu;
        if (k.c0 > 0) {
            ph = lv_hash(B.load4(a.S[k.pb + k.c0 - 1]));
            prs = k.c0 >= 257 ? k.c0 - 257 : 0u; // (a run of more than 256 before c0: count >= 255)
            for (uint32_t b = 0; b < 256 && b < k.c0; b += 64) {
                const uint32_t y = k.c0 - 1 - b - l; // (entries c0 - 1, c0 - 2, ...)
                const bool in = b + l < k.c0;
                const uint64_t m = ballot(in && lv_hash(B.load4(a.S[k.pb + y])) != ph);
                if (m) {
                    prs = k.c0 - b - (uint32_t)__builtin_ctzll(m); // (the first entry after the change)
                    break;
                }
                if (b + 64 >= k.c0) prs = 0;
            }
        }
        for (uint32_t x0 = k.c0; x0 < k.c1; x0 += 64) {
            const uint32_t x = x0 + l;
            const bool in = x < k.c1;
            const uint32_t p = in ? a.S[k.pb + x] : 0u;
            const uint32_t h = in ? lv_hash(B.load4(p)) : 0xfffffffeu;
            uint32_t hp = (uint32_t)__shfl_up((int)h, 1), qp = (uint32_t)__shfl_up((int)p, 1);
            if (l == 0) {
                hp = ph;
                qp = x > 0 ? a.S[k.pb + x - 1] : 0u;
            }
            uint32_t rs = wave_incl_max_dpp(in && h != hp ? x : 0u);
            rs = rs > prs ? rs : prs;
            if (in) {
                a.R[k.pb + p] = x;
                uint32_t cnt = x - rs;
                if (cnt && a.S[k.pb + rs] == 0) cnt--; // (NIL heads its run)
                const bool search = x > 0 && h == hp && qp != 0 && p - qp <= kLvMaxDist;
                a.HC[k.pb + p] = (uint8_t)(search ? (cnt < 255 ? cnt : 255) : 0);
            }
            ph = readlane(h, 63);
            prs = readlane(rs, 63);
        }
    }
}

// ---- 2. parse -------------------------------------------------------------------------------------
struct LvParse {
    LvBytes B;
    const uint32_t *S, *R;
    const uint8_t *HC;
    uint32_t *tok;
    uint64_t pb;
    uint32_t len, npos;

    // leading equal bytes of i and q (LCP), capped at cap: 16 bytes per step
    __device__ uint32_t lcp(uint32_t i, uint32_t q, uint32_t cap) const {
        uint32_t o = 0;
        for (;;) {
            uint64_t a0, a1, b0, b1;
            B.load16(i + o, a0, a1);
            B.load16(q + o, b0, b1);
            const uint64_t y0 = a0 ^ b0, y1 = a1 ^ b1;
            const uint32_t e0 = y0 ? (uint32_t)__builtin_ctzll(y0) >> 3 : 8u;
            const uint32_t e = e0 < 8 ? e0 : 8u + (y1 ? (uint32_t)__builtin_ctzll(y1) >> 3 : 8u);
            o += e;
            if (e < 16 || o >= cap) break;
        }
        return o < cap ? o : cap;
    }
    // longest_match(i) with prev_length b0 (deflate.c): the nearest of the longest among the first C
    // chain candidates (C = 4096, 1024 once prev_length >= good_length 32; the first at distance <=
    // MAX_DIST, later ones < MAX_DIST), if longer than b0; 64 candidates per wave step
    // (r = R[i], cnt = HC[i]: the chain length, 255 = at least 255 (lv_rank_kernel); the parse reads both
    // from its window of 64 positions)
    // (q0: lane l's first-step candidate S[r - 1 - l], 0 before the value's first sorted entry)
    __device__ uint32_t first_cand(int r) const {
        const int k = r - 1 - (int)lane_id();
        return k >= 0 ? S[pb + (uint32_t)k] : 0u;
    }
    __device__ uint32_t search(uint32_t i, uint32_t b0, int r, uint32_t cnt, uint32_t q0, uint32_t *q_out) const {
        const uint32_t l = (uint32_t)lane_id();
        const uint32_t C = b0 >= 32 ? 1024u : 4096u;
        const uint32_t nice = (len - i) < 258 ? (len - i) : 258;
        uint32_t hi = 0;
        if (cnt == 255) hi = lv_hash(B.load4(i));
        uint32_t best = 0, bestq = 0, examined = 0;
        // chain entries one step ahead: the next step's S load is issued with this step's, so its round
        // trip hides behind this step's byte loads (loads return in order)
        uint32_t qn = q0;
        for (int kb = r - 1;; kb -= 64) {
            const int k = kb - (int)l;
            const uint32_t ord = examined + l;
            const uint32_t q = qn;
            qn = k - 64 >= 0 ? S[pb + (uint32_t)(k - 64)] : 0u;
            const uint32_t d = i - q;
            // chain membership from the count; past 255 entries by the hash (the run's end)
            const bool member = ord < cnt || (cnt == 255 && k >= 0 && q != 0 && lv_hash(B.load4(q)) == hi);
            const bool valid = member && (ord == 0 ? d <= kLvMaxDist : d < kLvMaxDist) && ord < C;
            const uint64_t m = ballot(valid);
            const uint32_t npre = ~m == 0 ? 64u : (uint32_t)__builtin_ctzll(~m);
            if (npre == 0) break;
            const uint32_t cl = l < npre ? lcp(i, q, nice) : 0u;
            const uint32_t thr = best > b0 ? best : b0;
            const uint32_t key = cl > thr ? (cl << 16) | (0xffffu - ord) : 0u;
            const uint32_t mx = wave_max_dpp(key);
            if (mx) {
                best = mx >> 16;
                bestq = readlane(q, (int)(0xffffu - (mx & 0xffffu) - examined));
            }
            examined += npre;
            if (best >= nice || npre < 64 || examined >= C) break;
        }
        *q_out = bestq;
        return best > b0 ? best : 0u;
    }
    // the first position >= i (< end) where zlib searches, else end
    __device__ uint32_t next_hc(uint32_t i, uint32_t end) const {
        const uint32_t l = (uint32_t)lane_id();
        const uint32_t lim = end < npos ? end : npos;
        for (uint32_t x0 = i; x0 < lim; x0 += 64) {
            const uint32_t x = x0 + l;
            const uint64_t m = ballot(x < lim && HC[pb + x] != 0);
            if (m) return x0 + (uint32_t)__builtin_ctzll(m);
        }
        return end;
    }
};

__device__ __forceinline__ void lv_state(uint32_t *spec, uint32_t *cont, uint32_t s, uint32_t e, bool last, uint32_t p,
                                         uint32_t code, uint32_t ntok) {
    const uint32_t w = code << 30 | ntok;
    if (p - s < kLvOverlap) spec[p - s] = w;
    if (!last && p >= e && p - e < kLvOverlap) cont[p - e] = w;
}

__global__ void __launch_bounds__(256, 8) lv_parse_kernel(LargeArgs a) {
    const uint32_t l = (uint32_t)lane_id();
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t sg = wave; sg < a.nseg; sg += nwaves) {
        const uint32_t ov = a.seg_val[sg];
        LvParse P;
        P.B = lv_bytes(a, ov);
        P.S = a.S;
        P.R = a.R;
        P.HC = a.HC;
        P.pb = a.lv_pbase[ov];
        P.len = P.B.len;
        P.npos = lv_npos(P.len);
        const uint32_t g0 = a.lv_seg0[ov], g1 = a.lv_seg0[ov + 1];
        const bool last = sg + 1 == g1;
        const uint32_t s = (uint32_t)(sg - g0) * kLvSeg;
        const uint32_t e = last ? P.len : s + kLvSeg;
        const uint32_t eo = last ? P.len : (e + kLvOverlap < P.len ? e + kLvOverlap : P.len);
        uint32_t *spec = a.map + sg * 2 * kLvOverlap, *cont = spec + kLvOverlap;
        // (not unrolled: unrolled, the compiler hoists all 64 store addresses out of the segment loop into
        // 128 VGPRs, which held this kernel at 168 VGPRs / 3 waves per SIMD until round 5)
#pragma unroll 1
        for (uint32_t k = l; k < 2 * kLvOverlap; k += 64) spec[k] = 0;
        P.tok = a.tok + a.seg_tok0[sg];
        wave_sync_global();
        // R and HC of 64 positions from w0, one per lane: one coalesced load each instead of two
        // dependent round trips at the head of every search
        uint32_t w0 = 0x80000000u, wR = 0, wH = 0; // (p - w0 >= 64 for every p < 2^31: no window yet)
        auto window = [&](uint32_t p) {
            if (p - w0 >= 64u) {
                w0 = p;
                const uint32_t x = p + l;
                wR = x < P.npos ? P.R[P.pb + x] : 0u;
                wH = x < P.npos ? (uint32_t)P.HC[P.pb + x] : 0u;
            }
        };
        auto hc_at = [&](uint32_t p) -> uint32_t {
            if (p >= P.npos) return 0u;
            window(p);
            return readlane(wH, (int)(p - w0));
        };
        // deflate_slow (deflate.c) from a fresh state at s; the state is wave-uniform
        uint32_t i = s, ml = 2, ms = 0, avail = 0, ntok = 0;
        while (i < eo) {
            if (ml == 2) {
                // a run of positions without a search: literal steps only
                uint32_t j = i;
                if (!hc_at(i)) j = P.next_hc(i, eo);
                if (j > i) {
                    const uint32_t lo = i - avail, n = j - 1 - lo; // literals b[lo .. j - 2]
                    for (uint32_t k = l; k < n; k += 64) P.tok[ntok + k] = P.B.byte(lo + k);
                    for (uint32_t p = i + l; p < j; p += 64) // loop-top states in the recorded regions
                        if (p - s < kLvOverlap || (!last && p >= e && p - e < kLvOverlap))
                            lv_state(spec, cont, s, e, last, p, p == i && !avail ? 1u : 2u,
                                     ntok + (p - i) - (avail ? 0u : (p > i ? 1u : 0u)));
                    ntok += n;
                    avail = 1;
                    i = j;
                    if (i >= eo) break;
                }
                if (l == 0) lv_state(spec, cont, s, e, last, i, avail ? 2u : 1u, ntok);
            }
            const uint32_t pl = ml, pm = ms;
            ml = 2;
            const uint32_t cnt = i + 3 <= P.len && pl < 258 ? hc_at(i) : 0u;
            if (cnt) {
                uint32_t q = 0;
                const int r = (int)readlane(wR, (int)(i - w0));
                const uint32_t q0 = P.first_cand(r);
                const uint32_t m = P.search(i, pl, r, cnt, q0, &q);
                if (m) {
                    ml = m;
                    ms = q;
                    if (m == 3 && i - q > kLvTooFar) ml = 2;
                }
            }
            if (pl >= 3 && ml <= pl) {
                if (l == 0) P.tok[ntok] = (i - 1 - pm) << 16 | (pl - 3);
                ntok++;
                i += pl - 1;
                avail = 0;
                ml = 2;
            } else if (avail) {
                if (l == 0) P.tok[ntok] = P.B.byte(i - 1);
                ntok++;
                i++;
            } else {
                avail = 1;
                i++;
            }
        }
        if (last && avail) { // (deflate_slow's trailing literal)
            if (l == 0) P.tok[ntok] = P.B.byte(i - 1);
            ntok++;
        }
        if (l == 0) a.seg_tok[sg * 4] = ntok;
    }
}

// ---- 0. select: the batch's values of lo < len <= hi, as (index, length) pairs after a count ----------
__global__ void lv_select_kernel(const uint32_t *src_len, uint64_t n, uint64_t lo, uint64_t hi, uint32_t *out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t len = src_len[i];
        if (len > lo && len <= hi) {
            const uint32_t k = atomicAdd(out, 1u);
            out[2 + 2 * (uint64_t)k] = (uint32_t)i;
            out[3 + 2 * (uint64_t)k] = len;
        }
    }
}

// ---- 3. stitch ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) lv_stitch_kernel(LargeArgs a) {
    const uint32_t l = (uint32_t)lane_id();
    for (uint32_t ov = blockIdx.x; ov < a.nv; ov += gridDim.x) {
        const uint32_t g0 = a.lv_seg0[ov], g1 = a.lv_seg0[ov + 1];
        int32_t bad = 0;
        if (l == 0) a.seg_tok[(uint64_t)g0 * 4 + 1] = 0;
        for (uint32_t g = g0; g + 1 < g1; g++) {
            const uint32_t *cont = a.map + (uint64_t)g * 2 * kLvOverlap + kLvOverlap;
            const uint32_t *spec = a.map + (uint64_t)(g + 1) * 2 * kLvOverlap;
            uint32_t found = 0xffffffffu;
            for (uint32_t p0 = 0; p0 < kLvOverlap && found == 0xffffffffu; p0 += 64) {
                const uint32_t x = cont[p0 + l], y = spec[p0 + l];
                const uint64_t m = ballot((x >> 30) != 0 && (x >> 30) == (y >> 30));
                if (m) found = p0 + (uint32_t)__builtin_ctzll(m);
            }
            if (found == 0xffffffffu) {
                bad = 1;
                break;
            }
            if (l == 0) {
                a.seg_tok[(uint64_t)g * 4 + 2] = cont[found] & 0x3fffffffu;
                a.seg_tok[(uint64_t)(g + 1) * 4 + 1] = spec[found] & 0x3fffffffu;
            }
        }
        if (l == 0) {
            a.seg_tok[(uint64_t)(g1 - 1) * 4 + 2] = a.seg_tok[(uint64_t)(g1 - 1) * 4];
            a.fail[ov] = bad;
        }
    }
}

} // namespace pmc
