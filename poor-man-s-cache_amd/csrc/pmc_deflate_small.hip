// pmc_deflate_small.hip -- gzip level-9 compression of values up to 16382 bytes (always a
// single DEFLATE block: zlib flushes at 16383 symbols), the hot path of the cache
// (BASELINE configs 2-4: 256 B .. 4 KiB values).  Same output bytes as pmc_deflate.hip /
// zlib 1.2.11 (reference: /root/reference/src/compressor/gzip_compressor.cpp:3-50); this
// variant is organised for gfx950 latency and LDS capacity:
//
//  * working set ~9n + 3.5 KiB per wave (u16 sorted positions + u16 ranks; the candidate
//    hash is recomputed from the value bytes; sort scratch aliases the Huffman/output
//    region), so 12+ waves share a CU at 1 KiB values.
//  * longest_match: 64 chain candidates per step, LCP by aligned-dword compares; the
//    winner is taken with one ballot + readlane when at most one lane beats the current
//    best (the common case) and a DPP row reduction + 4 readlanes otherwise -- no LDS
//    shuffles on the serial path.  Symbol histograms are built after the parse, in parallel.
//  * Huffman (zlib trees.c build_tree): the binary heap lives in five VGPRs, lane-distributed
//    (entry k in lane k%64 of register k/64), driven by scalar code through v_readlane /
//    v_writelane, so each pqdownheap level costs a few cycles instead of LDS round trips.
//    Entries pack (freq<<5 | depth)<<10 | node, so zlib's `smaller` is one compare.
//    Everything around the heap is wave-parallel: leaf compaction (ballot), code lengths
//    (pointer jumping over the father links), canonical codes (ballot ranks), scan_tree /
//    send_tree (each maximal run of equal lengths has a fixed code sequence given its
//    value and length, so runs are encoded independently).  A length-limit overflow (rare)
//    re-plans the block with the serial zlib restatement (pmc_trees.hpp) on a per-wave
//    HBM scratch Trees.
#include <hip/hip_runtime.h>

#include "pmc_device.hpp"
#include "pmc_kernels.hpp"

namespace pmc {

constexpr uint32_t kSmallMax = 16382;

// Per-wave LDS image (offsets from the wave's base).  Phases reuse dead regions:
//   sort : bytes | S | R (hash keys until the ranks are written) | T, cnt
//   parse: bytes | S | R | M (per-position match_all results)
//   flush: bytes | out image, code tables, tree scratch, histograms (over S, R, M)
struct SmallLayout {
    uint64_t bytes, S, R, X, total;
    uint64_t out, lcode, dcode, blcode, dad, dep, runs, freq; // flush view
    uint64_t out_words;
    uint64_t T, cnt; // sort view
    uint64_t M, masks, masks_p; // parse view
    uint64_t front_total, back_total; // split pipeline: front (stage..parse..histogram), back (emit)
};

// on-demand parse scratch from some offset o: CN u8[n] | HC u64[nw] | EV u32[64] + u8[64]
// (320 B: at 1 KiB one more byte per wave costs a block of 4 waves per CU)
__host__ __device__ inline uint64_t cn_hc_offset(uint64_t n) { return (n + 15) & ~(uint64_t)15; }
__host__ __device__ inline uint64_t cn_ev_offset(uint64_t n) {
    return cn_hc_offset(n) + ((((n + 63) / 64) * 8 + 15) & ~(uint64_t)15);
}
__host__ __device__ inline uint64_t cn_region_bytes(uint64_t n) { return cn_ev_offset(n) + 320; }
__host__ __device__ inline SmallLayout small_layout(uint64_t n) {
    auto a = [](uint64_t x) { return (x + 15) & ~(uint64_t)15; };
    SmallLayout L;
    uint64_t o = 0;
    L.bytes = o;
    o += a(n + 32);
    L.S = o;
    o += a(2 * n + 2);
    L.R = o;
    o += a(2 * n + 2);
    L.X = o;
    // flush view, from S on
    uint64_t f = L.S;
    L.out = f;
    L.out_words = a(gzip_bound(n) + 16) / 4;
    f += L.out_words * 4;
    L.lcode = f;
    f += 288 * 4;
    L.dcode = f;
    f += 32 * 4;
    L.blcode = f;
    f += 32 * 4;
    L.dad = f;
    f += 576 * 2;
    L.dep = f;
    f += 576;
    L.runs = f; // run lengths at run starts: lit/len [0,288), dist [288,320)
    f += 320 * 2;
    L.freq = f; // lfreq u32[288], dfreq u32[32], blfreq u32[32]
    f += 352 * 4;
    // sort view
    uint64_t s = L.X;
    L.T = s;
    s += a(2 * n + 2);
    L.cnt = s;
    s += 16 * 64 * 2;
    // parse view: per-position match_all results, then the segment-walk bit masks
    L.M = L.X;
    L.masks = L.M + a(4 * n);
    L.masks_p = L.masks + a(((n + 63) / 64) * 8);
    uint64_t m = L.masks_p + a(((n + 63) / 64) * 8);
    const uint64_t mc = L.M + cn_region_bytes(n); // on-demand parse view (CN | HC | EV)
    m = m > mc ? m : mc;
    uint64_t t = f > s ? f : s;
    t = t > m ? t : m;
    L.total = a(t);
    L.front_total = a(t);
    L.back_total = a(f);
    return L;
}
uint64_t deflate_small_wave_bytes(uint64_t n) { return small_layout(n).total; }
// Chain counts packed into the top bits of R (ranks use ceil(log2 n) bits): 6 bits for n <= 1024,
// 4 bits for 3072 < n <= 4096 (0 = not packed: a separate u8 CN array).  A count field holds the exact
// count below its maximum; the maximum means "at least that many".  4 bits saturate below the eval's
// 32 lanes per position (more cut walks), which pays only where dropping the n-byte CN array buys a
// wave per SIMD: same-box A/B, 4 KiB front 256 -> 244 ms (7 waves/CU instead of 6); at 2 KiB, 5 bits
// made the front 4 % slower.
// Values above 16382 bytes (the large pass, up to deflate_big_limit()) keep no counts at all (-1):
// the has-candidate bits HC stand in, every such position gets kPreCand validated lanes and is cut.
__host__ __device__ inline int front_pkb(uint64_t n) {
    return n <= 1024 ? 6 : (n > 3072 && n <= 4096) ? 4 : n > kSmallMax ? -1 : 0;
}
// split-pipeline front: bytes | S | R | X (sort table, then the parse's HC bits); the symbol
// histograms overlay S and R after the parse
struct FrontLayout {
    uint64_t bytes, S, R, X, freq, total;
    int pkb;             // chain-count bits packed into R's top (front_pkb), 0: CN array, -1: HC only
    uint64_t cn, hc, ev; // parse scratch in X (cn unused when pk); the sort's 512-B table at X
};
// PMC_FRONT_S12: at 3-4 KiB (pkb 4, positions < 4096) the sorted positions are packed as 12-bit fields
// (8 per 3 dwords, 4 spare bytes for the read of the last field's next dword): the front's LDS per wave
// drops from 21.4 to 19.3 KB, so a CU holds 8 waves instead of 7 (round 2 measured 6 -> 7 waves as
// 256 -> 244 ms at 4 KiB).
#ifndef PMC_FRONT_S12
#define PMC_FRONT_S12 1
#endif
__host__ __device__ inline bool front_s12(uint64_t n) { return PMC_FRONT_S12 && front_pkb(n) == 4; }
__host__ __device__ inline FrontLayout front_layout(uint64_t n) {
    auto a = [](uint64_t x) { return (x + 15) & ~(uint64_t)15; };
    FrontLayout F;
    F.bytes = 0;
    F.S = a(n + 32);
    // (the packed S keeps >= 256 B: the sort parks its 128 high-digit counters there)
    const uint64_t s_bytes = front_s12(n) ? ((n * 12 + 31) / 32) * 4 + 4 : 2 * n + 2;
    F.R = F.S + a(s_bytes > 256 ? s_bytes : 256);
    F.X = F.R + a(2 * n + 2);
    F.pkb = front_pkb(n);
    F.cn = F.X;
    F.hc = F.pkb ? F.X : F.X + a(n);
    F.ev = F.hc + a(((n + 63) / 64) * 8);
    const uint64_t xe = F.ev + 320 > F.X + 512 ? F.ev + 320 : F.X + 512;
    F.freq = F.S;
    const uint64_t t2 = F.freq + 352 * 4;
    F.total = a(xe > t2 ? xe : t2);
    return F;
}
uint64_t deflate_front_wave_bytes(uint64_t n) { return front_layout(n).total; }
// split-pipeline back (emission only): bytes | out | lcode | dcode | blcode | runs | lengths
struct BackLayout {
    uint64_t bytes, out, out_words, lcode, dcode, blcode, runs, ls, blfreq, perm, total;
};
__host__ __device__ inline BackLayout back_layout(uint64_t n) {
    auto a = [](uint64_t x) { return (x + 15) & ~(uint64_t)15; };
    BackLayout B;
    B.bytes = 0;
    B.out = a(n + 32);
    B.out_words = a(gzip_bound(n) + 16) / 4;
    B.lcode = B.out + B.out_words * 4;
    B.dcode = B.lcode + 288 * 4;
    B.blcode = B.dcode + 32 * 4;
    B.runs = B.blcode + 32 * 4;
    B.ls = B.runs + 320 * 2;
    B.blfreq = a(B.ls + kSplitRows); // scan_runs' bit-length counts (unused by the back)
    B.perm = B.blfreq + 32 * 4;      // the code-rank guard's symbols in canonical order (u16 per symbol)
    B.total = a(B.perm + kSplitRows * 2);
    return B;
}
uint64_t deflate_back_wave_bytes(uint64_t n) { return back_layout(n).total; }

__device__ __forceinline__ uint32_t hash3(uint32_t w) {
    return ((w & 0xff) << 10 ^ ((w >> 8) & 0xff) << 5 ^ ((w >> 16) & 0xff)) & 0x7fffu;
}

// ---- register-resident binary heap ---------------------------------------------------
struct RegHeap {
    uint32_t h0, h1, h2, h3, h4; // entry k: lane k&63 of h[k>>6]
    __device__ uint32_t reg(int r) const {
        return r == 0 ? h0 : r == 1 ? h1 : r == 2 ? h2 : r == 3 ? h3 : h4;
    }
    __device__ uint32_t get(int k) const { return readlane(reg(k >> 6), k & 63); }
    __device__ void set(int k, uint32_t v) {
        const int r = k >> 6, ln = k & 63;
        if (r == 0) h0 = writelane(h0, v, ln);
        else if (r == 1) h1 = writelane(h1, v, ln);
        else if (r == 2) h2 = writelane(h2, v, ln);
        else if (r == 3) h3 = writelane(h3, v, ln);
        else h4 = writelane(h4, v, ln);
    }
    // pqdownheap (trees.c) with smaller(n,m) == key(n) <= key(m), key = e >> 10
    __device__ void down(int k, int heap_len) {
        uint32_t v = get(k);
        int j = k << 1;
        while (j <= heap_len) {
            uint32_t x = get(j);
            if (j < heap_len) {
                uint32_t y = get(j + 1);
                if ((y >> 10) <= (x >> 10)) {
                    j++;
                    x = y;
                }
            }
            if ((v >> 10) <= (x >> 10)) break;
            set(k, x);
            k = j;
            j <<= 1;
        }
        set(k, v);
    }
};

// Small heaps (the common case), written so every level of pqdownheap is straight-line
// scalar code (two v_readlane, a select, one masked v_cndmask) with no dynamic register
// indexing.  RegHeap1: entries 1..63, entry k in lane k.  RegHeap2: entries 1..127
// interleaved, entry k in lane k>>1 of (k odd ? h1 : h0), so the children 2k, 2k+1 of node
// k sit in lane k of h0 and h1.
// (a <= b) ? t : f on the scalar unit (uniform operands), kept out of lane-mask form
__device__ __forceinline__ uint32_t s_sel_le(uint32_t a, uint32_t b, uint32_t t, uint32_t f) {
    uint32_t r;
    asm("s_cmp_le_u32 %1, %2\n\ts_cselect_b32 %0, %3, %4" : "=s"(r) : "s"(a), "s"(b), "s"(t), "s"(f) : "scc");
    return r;
}
// Both small heaps keep every slot past heap_len (and slot 0) at ~0: a missing right child
// then never wins the smaller() test, so no j < heap_len check is needed.
// pqdownheap in three steps: (1) every parent lane computes its smaller child at once (zlib's
// smaller(): the right child wins ties), packed key << 8 | child index; (2) the scalar walk
// follows those links from k with one v_readlane + compare per level, collecting the path
// (the smaller children along a sift path are not changed by the sift, so this is exact);
// (3) every path entry takes its smaller child's value in one parallel select.
struct RegHeap1 {
    uint32_t h;
    __device__ uint32_t get(int k) const { return readlane(h, k); }
    __device__ void set(int k, uint32_t v) { h = writelane(h, v, k); }
    __device__ void down(int k, int n) {
        const int l = lane_id();
        const uint32_t v = readlane(h, k), kv = v >> 10;
        const uint32_t a = (uint32_t)__shfl((int)h, (2 * l) & 63), b = (uint32_t)__shfl((int)h, (2 * l + 1) & 63);
        const bool right = (b >> 10) <= (a >> 10);
        const uint32_t mv = right ? b : a;
        const uint32_t pk = (mv >> 10) << 8 | (uint32_t)(2 * l + (right ? 1 : 0));
        uint64_t path = 0;
        int cur = k;
        while (2 * cur <= n) {
            const uint32_t e = readlane(pk, cur);
            if (kv <= (e >> 8)) break;
            path |= 1ull << cur;
            cur = (int)(e & 0xff);
        }
        h = ((path >> l) & 1) ? mv : h;
        h = writelane(h, v, cur);
    }
};
struct RegHeap2 {
    uint32_t h0, h1;
    __device__ uint32_t get(int k) const {
        const uint32_t a = readlane(h0, k >> 1), b = readlane(h1, k >> 1);
        return (k & 1) ? b : a;
    }
    __device__ void set(int k, uint32_t v) {
        const bool hit = lane_id() == (k >> 1);
        const bool odd = (k & 1) != 0;
        h0 = (hit & !odd) ? v : h0;
        h1 = (hit & odd) ? v : h1;
    }
    __device__ void down(int k, int n) {
        const int l = lane_id();
        const uint32_t v = get(k), kv = v >> 10;
        // lane p holds the children 2p (h0) and 2p+1 (h1) of entry p
        const bool right = (h1 >> 10) <= (h0 >> 10);
        const uint32_t mv = right ? h1 : h0;
        const uint32_t pk = (mv >> 10) << 8 | (uint32_t)(2 * l + (right ? 1 : 0));
        uint64_t p0 = 0, p1 = 0; // path entries 2L (bit L of p0) and 2L+1 (bit L of p1)
        int cur = k;
        while (2 * cur <= n) {
            const uint32_t e = readlane(pk, cur);
            if (kv <= (e >> 8)) break;
            if (cur & 1) p1 |= 1ull << (cur >> 1);
            else p0 |= 1ull << (cur >> 1);
            cur = (int)(e & 0xff);
        }
        if (p0 | p1) { // entry p (lane p>>1 of h[p&1]) takes mv of lane p
            const uint32_t s0 = (uint32_t)__shfl((int)mv, (2 * l) & 63);
            const uint32_t s1 = (uint32_t)__shfl((int)mv, (2 * l + 1) & 63);
            h0 = ((p0 >> l) & 1) ? s0 : h0;
            h1 = ((p1 >> l) & 1) ? s1 : h1;
        }
        set(cur, v);
    }
};

struct TreeOut {
    int max_code;
    int64_t opt, stat;
    bool overflow;
    int dummy[2]; // symbols whose freq build_tree set to 1 (zlib's "at least 2 codes"), or -1
};

// chain candidates evaluated per position by the on-demand parse's wave step (the rest, when
// needed, by search()); at most 32 (5-bit field in the eval key)
constexpr uint32_t kPreCandLanes = 32;
// PMC_EVAL_BPERM: each eval offset fetches its position's maximum from the position's last lane by
// ds_bpermute instead of an LDS store by that lane and a read back
#ifndef PMC_EVAL_BPERM
#define PMC_EVAL_BPERM 1
#endif
// PMC_HC_FROM_R: with chain counts in R (PK > 0) the walk's has-candidate words are ballots of those
// counts, so build_cn sets no HC bits (no same-word LDS atomics)
#ifndef PMC_HC_FROM_R
#define PMC_HC_FROM_R 1
#endif
// PMC_EVAL_CN1DPP: the eval's count of position x + 1 by a DPP move from lane l + 1
#ifndef PMC_EVAL_CN1DPP
#define PMC_EVAL_CN1DPP 1
#endif
// PMC_EVAL_PRED (values <= 1 KiB, PK 6): build_cn stores each position's match length with its nearest
// candidate (capped at 32) in the spare top bits of its S entry; an eval runs deflate_slow's lazy walk over
// those lengths for up to kPredHops fresh starts and gives lanes only to the positions that walk visits,
// instead of to every position of the window in order (a round-6 simulation of 1 KiB JSON slices: 38.8 ->
// 24.7 evals per value; the stamps build measured 37.5 -> 23.8).  The walk itself stays exact: a needed position the prediction left out is a
// stop, and the next eval starts there.
#ifndef PMC_EVAL_PRED
#define PMC_EVAL_PRED 1
#endif
// (same box, 10M x 1 KiB: front 175.3 -> 173.5 ms at 3 hops, 173.9 at 4; lengths capped at 16 instead of
// 32: 177.4 -- more misses; the hops as a scalar loop over the masks instead of per-lane precomputed
// targets: 196 ms, the scalar unit saturated)
constexpr uint32_t kPredHops = 3, kPredCap = 32;
// (the fault build runs the u32-counter sort's first scatter from the loop below, whose lanes it reverses)
#ifdef PMC_FAULT_LANE_ORDER
#define PMC_FAULT_PASS0 0
#else
#define PMC_FAULT_PASS0 1
#endif
// A uniform 0/1 integer the compiler may not turn back into a bool: branching on it is one
// s_cmp + s_cbranch_scc.  (Bools merged across blocks become 64-bit lane masks -- s_cselect_b64,
// s_and_b64 with exec, s_cbranch_vcc -- on the scalar unit, which the parse saturates.)
__device__ __forceinline__ uint32_t sflag(uint32_t x) {
    x = __builtin_amdgcn_readfirstlane(x);
    asm volatile("" : "+s"(x));
    return x;
}

struct SmallWave {
    // every working array is LDS-typed (ds_* with 32-bit addresses)
    PMC_LDS uint8_t *b;
    PMC_LDS uint32_t *bw;
    PMC_LDS uint16_t *S, *R;
    uint32_t s12 = 0; // front at 3-4 KiB (front_s12): S packed as 12-bit fields (sget<4>)
    PMC_LDS uint32_t *lfreq, *dfreq, *blfreq;
    PMC_LDS uint32_t *outw;
    PMC_LDS uint8_t *outb;
    uint32_t out_words;
    PMC_LDS uint32_t *lcode, *dcode, *blcode;
    PMC_LDS uint16_t *dad;
    PMC_LDS uint8_t *dep;
    PMC_LDS uint16_t *runs;
    PMC_LDS uint16_t *T, *H, *cnt;
    PMC_LDS uint32_t *M;    // per-position match_all results (aliases the sort scratch)
    PMC_LDS uint64_t *HC;   // on-demand parse: bit x = position x has a chain candidate (aliases M)
    PMC_LDS uint8_t *CN;    // on-demand parse: chain candidates of position x (capped at 255)
    PMC_LDS uint32_t *EV;   // on-demand parse: eval scratch (64 best keys, 64 u8 owner marks)
    int cnp;                // chain-count bits in R's top (front_pkb: 6 / 5 / 4), 0: counts in CN
    PMC_LDS uint64_t *ML;   // segment walk: positions that start a match (or are unresolved)
    PMC_LDS uint64_t *MP;   // segment walk: positions where a lazy-improvement run ends
    PMC_GLB uint32_t *tok;
    PMC_GLB const uint32_t *hdr = nullptr; // split back: this value's tree header from the trees kernel
    PMC_GLB const uint8_t *gsrc = nullptr; // split back (PMC_BACK_NOSTAGE): the source bytes in HBM, not staged
    Trees *fb; // HBM scratch for the serial fallback
    PMC_LDS const uint32_t *crc_tab;
    PMC_LDS uint16_t *perm; // split back: the code-rank guard's canonical order (BackLayout::perm)
#ifdef PMC_FAULT_LANE_ORDER
    uint32_t fault_rev = 0; // this value's sort takes its lanes in reverse (diagnostic build)
#endif
    static constexpr uint64_t kBitsGuard = ~0ull; // emit_planned: the code-rank guard fired
    uint64_t st[16];
    uint64_t t_last;
    int stop; // PMC_STAMPS: end the value after phase `stop` (instruction-count attribution)

    __device__ void stamp(int k) {
#ifdef PMC_STAMPS
        uint64_t t = __builtin_amdgcn_s_memtime();
        st[k] += t - t_last;
        t_last = t;
#endif
    }
    __device__ void count(int k) {
#ifdef PMC_STAMPS
        st[k]++;
#endif
    }
#if defined(PMC_STAMPS) || defined(PMC_PHASE_STOP)
#define PMC_STOP(k, ret)                                                                                               \
    if (stop == (k)) return ret;
#else
#define PMC_STOP(k, ret)
#endif

    // sorted position k: u16, or (PK 4 with PMC_FRONT_S12) bits 12 k .. 12 k + 11 of the packed words
    template <int PK>
    __device__ __forceinline__ uint32_t sget(uint32_t k) const {
        if constexpr (PK == 4 && PMC_FRONT_S12) {
            PMC_LDS const uint32_t *S32 = (PMC_LDS const uint32_t *)S;
            const uint32_t bit = 12u * k, w = bit >> 5;
            return __builtin_amdgcn_alignbit(S32[w + 1], S32[w], bit & 31u) & 0xfffu;
        } else if constexpr (PK == 6 && PMC_EVAL_PRED) {
            return S[k] & 0x3ffu; // (bits 15:10: the nearest candidate's match length, PMC_EVAL_PRED)
        } else {
            return S[k];
        }
    }
    __device__ uint32_t load4(uint32_t p) const {
        uint32_t w0 = bw[p >> 2], w1 = bw[(p >> 2) + 1];
        return __builtin_amdgcn_alignbyte(w1, w0, p & 3);
    }

    // ---- stable LSD radix sort of positions by hash: 4 x 4-bit passes -------------------
    __device__ __noinline__ void sort_positions(uint32_t npos) {
        const int l = lane_id();
        for (uint32_t p = l; p < npos; p += 64) H[p] = (uint16_t)hash3(load4(p));
        const uint32_t c = (npos + 63) / 64;
        const uint32_t beg = (uint32_t)l * c;
        wave_sync();
        for (int pass = 0; pass < 4; pass++) {
            const int sh = 4 * pass;
            PMC_LDS const uint16_t *src = pass == 0 ? nullptr : (pass & 1 ? T : S);
            PMC_LDS uint16_t *dst = pass & 1 ? S : T;
            for (int d = 0; d < 16; d++) cnt[d * 64 + l] = 0;
            wave_sync();
            for (uint32_t j = 0; j < c; j++) {
                uint32_t idx = beg + j;
                if (idx < npos) {
                    uint32_t p = src ? src[idx] : idx;
                    cnt[((H[p] >> sh) & 15) * 64 + l]++;
                }
            }
            wave_sync();
            // exclusive scan of the 1024 counters in (digit, lane) order; lane l owns 16
            uint32_t v[16], s = 0;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                v[k] = cnt[l * 16 + k];
                s += v[k];
            }
            uint32_t base = wave_incl_scan(s) - s;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                cnt[l * 16 + k] = (uint16_t)base;
                base += v[k];
            }
            wave_sync();
            for (uint32_t j = 0; j < c; j++) {
                uint32_t idx = beg + j;
                if (idx < npos) {
                    uint32_t p = src ? src[idx] : idx;
                    uint32_t slot = ((H[p] >> sh) & 15) * 64 + l;
                    uint32_t at = cnt[slot];
                    cnt[slot] = (uint16_t)(at + 1);
                    dst[at] = (uint16_t)p;
                }
            }
            wave_sync();
        }
        for (uint32_t k = l; k < npos; k += 64) R[S[k]] = (uint16_t)k;
        wave_sync();
    }

    // ---- stable 2-pass LSD radix sort of positions by hash (8 + 7 bits) --------------------
    // Keys are recomputed from the bytes in every phase (no key array), T aliases R (ranks are
    // written last) and the only scratch is a 256-counter table, so the sort needs no LDS
    // beyond S, R and 1 KiB.  Within a 64-position chunk a lane's slot comes back from its
    // returning LDS atomic on the digit's counter (lanes of one instruction in lane order), so
    // the scatter is stable without per-lane counters or a ballot per digit bit.
    // Returns the rank of position 0 (the number of positions whose hash is smaller: the sort is
    // stable and 0 is the lowest position); the rank array R itself is written by build_cn.
    __device__ __forceinline__ uint32_t sort_positions2(uint32_t npos_, PMC_LDS uint32_t *tab) {
        SmallWave me = *this; // (see parse_ondemand)
        return me.sort_positions2_body(npos_, tab);
    }
    __device__ __forceinline__ uint32_t sort_positions2_body(uint32_t npos_, PMC_LDS uint32_t *tab) {
        const uint32_t npos = rfl(npos_);
        const uint32_t l = (uint32_t)lane_id();
        const uint32_t h0 = rfl(hash3(load4(0)));
        uint32_t k0 = 0;
        PMC_LDS uint16_t *Tt = R;
        // Both passes' digit counts in one pass over the positions (a histogram does not depend
        // on the order): 256 u16 low-digit counters in tab (512 B), 128 u16 high-digit counters
        // parked in S (untouched until the second scatter) and moved to tab after the first.
        // Counted two per word by u32 LDS atomics.  (S holds the 256 B only from npos >= 128 on;
        // shorter values count per pass.)
        PMC_LDS uint32_t *hiw = (PMC_LDS uint32_t *)S;
        const bool fused = npos >= 128;
        // One u32 counter per digit instead of two u16 per word (digits d and d ^ 1 no longer share an
        // address, so fewer lanes of a returning atomic serialise on one word): the 256 low-digit
        // counters in S (free until the second scatter), the 128 high-digit ones in tab
        // (values of 512 .. 1024 bytes: S then spans at least 1 KiB, the cap's 2 * cap + 2 bytes)
        // (not with a packed S: this path's second scatter writes u16 entries)
        if (npos >= 510 && npos <= 1022 && !s12) {
            PMC_LDS uint32_t *cl = (PMC_LDS uint32_t *)S;
            for (uint32_t k = l; k < 256; k += 64) cl[k] = 0;
            for (uint32_t k = l; k < 128; k += 64) tab[k] = 0;
            wave_sync();
            auto agg_add = [&](PMC_LDS uint32_t *ctr, uint32_t d, bool valid) -> uint32_t {
                return valid ? lds_add(&ctr[d], 1u) : 0u;
            };
            // (the hashes of positions c0 + l stay in registers, two per VGPR, for the first scatter, which
            // visits the same positions in the same lanes: no second load4 of them)
            uint32_t hreg[8];
#pragma unroll
            for (int c = 0; c < 16; c++) {
                const uint32_t c0 = 64u * (uint32_t)c;
                if (c0 >= npos) break;
                const uint32_t x = c0 + l;
                const uint32_t h = hash3(load4(x < npos ? x : 0u));
                hreg[c >> 1] = (c & 1) ? hreg[c >> 1] | h << 16 : h;
                k0 += (uint32_t)__builtin_popcountll(ballot(x < npos && h < h0));
                agg_add(cl, h & 255, x < npos);
                agg_add(tab, (h >> 8) & 127, x < npos);
            }
            wave_sync();
            { // exclusive bases: 4 low counters per lane, 2 high ones per lane
                uint32_t v[4], sum = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) sum += (v[k] = cl[4 * l + k]);
                uint32_t b = wave_incl_scan_dpp(sum) - sum;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    cl[4 * l + k] = b;
                    b += v[k];
                }
                const uint32_t h0c = tab[2 * l], h1c = tab[2 * l + 1], hs = h0c + h1c;
                const uint32_t hb = wave_incl_scan_dpp(hs) - hs;
                tab[2 * l] = hb;
                tab[2 * l + 1] = hb + h0c;
            }
            wave_sync();
#ifndef PMC_FAULT_LANE_ORDER
#pragma unroll
            for (int c = 0; c < 16; c++) { // first scatter, by the low digit, into Tt
                const uint32_t c0 = 64u * (uint32_t)c;
                if (c0 >= npos) break;
                const uint32_t x = c0 + l, h = (hreg[c >> 1] >> (16 * (c & 1))) & 0xffffu;
                const uint32_t slot = agg_add(cl, h & 255, x < npos);
                if (x < npos) Tt[slot] = (uint16_t)x;
            }
            wave_sync();
#endif
            for (int pass = PMC_FAULT_PASS0; pass < 2; pass++) {
                PMC_LDS uint32_t *ctr = pass ? tab : cl;
                PMC_LDS uint16_t *dst = pass ? S : Tt;
                for (uint32_t c0 = 0; c0 < npos; c0 += 64) {
#ifdef PMC_FAULT_LANE_ORDER
                    const uint32_t x = fault_rev ? c0 + 63u - l : c0 + l;
#else
                    const uint32_t x = c0 + l;
#endif
                    const uint32_t p = x < npos ? (pass ? (uint32_t)Tt[x] : x) : 0u;
                    const uint32_t h = hash3(load4(p)), d = pass ? (h >> 8) & 127 : h & 255;
                    const uint32_t slot = agg_add(ctr, d, x < npos);
                    if (x < npos) dst[slot] = (uint16_t)p;
                }
                wave_sync();
            }
            return k0;
        }
        auto scan_tab = [&]() { // 256 counters -> exclusive bases
            const uint32_t t0 = tab[2 * l], t1 = tab[2 * l + 1];
            const uint32_t v0 = t0 & 0xffffu, v1 = t0 >> 16, v2 = t1 & 0xffffu, v3 = t1 >> 16;
            const uint32_t sum = v0 + v1 + v2 + v3;
            const uint32_t b0 = wave_incl_scan_dpp(sum) - sum, b1 = b0 + v0, b2 = b1 + v1, b3 = b2 + v2;
            tab[2 * l] = b0 | b1 << 16;
            tab[2 * l + 1] = b2 | b3 << 16;
        };
        if (fused) {
            for (uint32_t k = l; k < 128; k += 64) tab[k] = 0;
            hiw[l] = 0;
            wave_sync();
            for (uint32_t c0 = 0; c0 < npos; c0 += 64) {
                const uint32_t x = c0 + l;
                const uint32_t h = hash3(load4(x < npos ? x : 0u));
                k0 += (uint32_t)__builtin_popcountll(ballot(x < npos && h < h0));
                if (x < npos) {
                    lds_add(&tab[(h & 255) >> 1], 1u << (16 * (h & 1)));
                    lds_add(&hiw[(h >> 9) & 63], 1u << (16 * ((h >> 8) & 1)));
                }
            }
            wave_sync();
            scan_tab();
            const uint32_t u = hiw[l], u0 = u & 0xffffu, usum = u0 + (u >> 16);
            const uint32_t c0 = wave_incl_scan_dpp(usum) - usum;
            hiw[l] = c0 | (c0 + u0) << 16;
            wave_sync();
        }
        for (int pass = 0; pass < 2; pass++) {
            const uint32_t sh = pass ? 8 : 0;
            PMC_LDS uint16_t *dst = pass ? S : Tt;
            if (fused && pass) { // the high-digit bases move out of S before the scatter writes it
                tab[l] = hiw[l];
                wave_sync();
            } else if (!fused) { // 256 u16 digit counters (512 B) for this pass
                for (uint32_t k = l; k < 128; k += 64) tab[k] = 0;
                wave_sync();
                for (uint32_t c0 = 0; c0 < npos; c0 += 64) {
                    const uint32_t x = c0 + l;
                    const bool valid = x < npos;
                    const uint32_t p = valid ? (pass ? (uint32_t)Tt[x] : x) : 0u;
                    const uint32_t h = hash3(load4(p)), d = (h >> sh) & 255;
                    if (!pass) k0 += (uint32_t)__builtin_popcountll(ballot(valid && h < h0));
                    if (valid) lds_add(&tab[d >> 1], 1u << (16 * (d & 1)));
                }
                wave_sync();
                scan_tab();
                wave_sync();
            }
            if ((uint32_t)pass & s12) { // (packed S: the scatter ORs 12-bit fields into zeroed words)
                for (uint32_t k = l; k < (npos * 12 + 31) / 32 + 1; k += 64) ((PMC_LDS uint32_t *)S)[k] = 0u;
                wave_sync();
            }
            // a lane's slot from one returning LDS atomic on its digit's counter: the lanes of one
            // ds_add_rtn to a word get their old values in lane order (scripts/micro/
            // lds_atomic_order.hip: 16.7M trials of skewed digit mixes, none out of order), so the
            // scatter stays stable without a ballot per digit bit (round 3: front 206 -> 191 ms)
            for (uint32_t c0 = 0; c0 < npos; c0 += 64) {
#ifdef PMC_FAULT_LANE_ORDER // (diagnostic build: a chunk's positions in reverse lane order, which build_cn's guard must catch)
                const uint32_t x = fault_rev ? c0 + 63u - l : c0 + l;
#else
                const uint32_t x = c0 + l;
#endif
                const uint32_t p = x < npos ? (pass ? (uint32_t)Tt[x] : x) : 0u;
                const uint32_t d = (hash3(load4(p)) >> sh) & 255, hs = 16 * (d & 1);
                if (x < npos) {
                    const uint32_t slot = (lds_add(&tab[d >> 1], 1u << hs) >> hs) & 0xffffu;
                    if ((uint32_t)pass & s12) {
                        const uint32_t bit = 12u * slot, w = bit >> 5, bs = bit & 31u;
                        lds_or((PMC_LDS uint32_t *)S + w, p << bs);
                        if (bs > 20u) lds_or((PMC_LDS uint32_t *)S + w + 1, p >> (32u - bs));
                    } else {
                        dst[slot] = (uint16_t)p;
                    }
                }
            }
            wave_sync();
        }
        return k0;
    }

    // 8 bytes at p (dword-aligned LDS reads + alignbyte; the value is zero padded)
    __device__ uint64_t load8(uint32_t p) const {
        const uint32_t w = p >> 2, sh = p & 3;
        const uint32_t w0 = bw[w], w1 = bw[w + 1], w2 = bw[w + 2];
        return (uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32 | __builtin_amdgcn_alignbyte(w1, w0, sh);
    }
    // leading equal bytes of two 8-byte words given their xor y (8 when equal), branch-free
    __device__ static uint32_t eq_bytes8(uint64_t y) {
        return ((uint32_t)__builtin_ctzll(y | (1ull << 63)) >> 3) + (y == 0 ? 1u : 0u);
    }
    // common prefix of positions i and q (first words wi, wq already loaded), capped at nice
    __device__ uint32_t lcp(uint32_t i, uint32_t q, uint32_t wi, uint32_t wq, uint32_t nice) const {
        uint32_t x = wi ^ wq, cl;
        if (x) {
            cl = (uint32_t)__builtin_ctz(x) >> 3;
        } else {
            cl = 4;
            while (cl < nice) {
                const uint64_t y = load8(i + cl) ^ load8(q + cl);
                if (y) {
                    cl += (uint32_t)__builtin_ctzll(y) >> 3;
                    break;
                }
                cl += 8;
            }
        }
        return cl < nice ? cl : nice;
    }
    // Can candidate q beat a match of length thr (>= 4) at i?  Only if the 4 bytes ending
    // at offset thr agree (wthr = load4(i + thr - 3)); zlib's scan_end test, widened.
    __device__ bool may_beat(uint32_t q, uint32_t thr, uint32_t wthr) const {
        return thr < 4 || load4(q + thr - 3) == wthr;
    }

    // ---- longest_match for every position at once (position-parallel) -----------------
    // zlib's longest_match(i) depends on prev_length only through the chain limit (4096 or
    // 1024 candidates) and the final "longer than prev_length" test, so the walk over the
    // first kPreCand chain candidates (nearest first) can run for all positions in
    // parallel before the serial parse.  M[i] = best | bestq << 9 | (walk cut short) << 31
    // with best = max over those candidates of min(LCP, nice), bestq the nearest achieving
    // it.  A cut-short walk is finished by search() if the parse visits i.
    static constexpr uint32_t kPreCand = kPreCandLanes;
    // Work-stealing walk, branch-light: every iteration each lane issues the same loads
    // (one chain entry, 8 bytes at i+off and at c+off, the two prune words) and advances
    // its state with selects -- a candidate is fetched, pruned, or compared 8 bytes further.
    // Lanes whose position is finished store M[i] and claim the next unclaimed position
    // (ballot + popcount), so the iteration count follows the total work.  The only
    // divergent blocks are that store/claim; per-lane control otherwise costs no SALU.
    __device__ __noinline__ void match_all(uint32_t npos, uint32_t len) {
        const uint32_t l = (uint32_t)lane_id();
        uint32_t next = 64; // first unclaimed position (uniform)
        uint32_t i = l, hi = 0, nice = 0, best = 0, bestq = 0, s = 0, c = 0, off = 0;
        int k = -1;
        bool ext = false, act = i < npos;
        if (act) {
            hi = hash3(load4(i));
            nice = (len - i) < 258 ? (len - i) : 258;
            k = (int)R[i] - 1;
        }
        while (ballot(act)) {
            const bool fetch = act && !ext;
            const bool can = fetch && k >= 0 && s < kPreCand;
            const uint32_t qn = S[can ? k : 0];
            c = ext ? c : qn;
            off = ext ? off : 0u;
            const uint32_t ii = act ? i : 0u;
            const uint64_t A = load8(ii + off), B = load8(c + off);
            const uint32_t bt = best >= 4 ? best - 3 : 0u;
            const uint32_t Pi = load4(ii + bt), Pc = load4(c + bt);
            // candidate fetch outcome (position 0 is zlib's NIL, the lowest entry of its run)
            const bool ok = can && qn != 0 && hash3((uint32_t)B) == hi;
            const bool chain_end = fetch && !ok;
            const bool cut = chain_end && s >= kPreCand && best < nice;
            const bool pruned = ok && best >= 4 && Pi != Pc;
            const bool working = ext || (ok && !pruned);
            const uint64_t y = A ^ B;
            const uint32_t m = y ? (uint32_t)__builtin_ctzll(y) >> 3 : 8u;
            const bool fin = working && (y != 0 || off + 8 >= nice);
            uint32_t cl = off + m;
            cl = cl < nice ? cl : nice;
            const bool better = fin && cl > best;
            best = better ? cl : best;
            bestq = better ? c : bestq;
            ext = working && !fin;
            off = off + 8;
            s += ok ? 1u : 0u;
            k -= ok ? 1 : 0;
            const bool done = act && (chain_end || (better && best >= nice));
            const uint64_t dm = ballot(done);
            if (done) {
                M[i] = best | bestq << 9 | (cut ? 1u << 31 : 0u);
                i = next + popc_lt(dm);
                act = i < npos;
                best = bestq = s = 0;
                ext = false;
                if (act) {
                    hi = hash3(load4(i));
                    nice = (len - i) < 258 ? (len - i) : 258;
                    k = (int)R[i] - 1;
                }
            }
            next += (uint32_t)__builtin_popcountll(dm);
        }
        wave_sync();
    }

    // ---- longest_match over the sorted chain -------------------------------------------
    // Resumes a walk cut short by match_all: candidates kPreCand.. of position i, starting
    // from that walk's best / bestq.  Returns the match length (> b0) or 0; *q_out = the
    // nearest candidate achieving it.
    // `start`: candidates the walk that was cut short already compared (nearest first)
    template <int PK>
    __device__ __forceinline__ uint32_t search(uint32_t i, uint32_t b0, uint32_t len, uint32_t best, uint32_t bestq,
                               uint32_t *q_out, uint32_t start = kPreCand) {
        const int l = lane_id();
        const uint32_t C = b0 >= 32 ? 1024u : 4096u;
        const uint32_t nice = (len - i) < 258 ? (len - i) : 258;
        const uint32_t wi = load4(i);
        const uint32_t hi = hash3(wi);
        const int r = (int)(PK > 0 ? R[i] & ((1u << (16 - (PK > 0 ? PK : 0))) - 1u) : (uint32_t)R[i]);
        uint32_t examined = start;
        for (int kb = r - 1 - (int)start;; kb -= 64) {
            const uint32_t thr = best > b0 ? best : b0;
            if (thr >= nice) break; // no candidate can be longer (lengths are capped at nice)
            const uint32_t wthr = thr >= 4 ? load4(i + thr - 3) : 0u;
            const int k = kb - l;
            const uint32_t ord = examined + (uint32_t)l;
            uint32_t q = k >= 0 ? sget<PK>((uint32_t)k) : 0u;
            uint32_t wq = load4(q);
            // position 0 is zlib's NIL (head[] value 0): never a match source; it is the
            // lowest position of its hash run, so valid lanes stay a prefix
            bool valid = k >= 0 && q != 0 && hash3(wq) == hi && ord < C;
            uint64_t m = ballot(valid);
            uint32_t npre = ~m == 0 ? 64u : (uint32_t)__builtin_ctzll(~m);
            if (npre == 0) break;
            const uint32_t cl = (uint32_t)l < npre && may_beat(q, thr, wthr) ? lcp(i, q, wi, wq, nice) : 0u;
            uint64_t mm = ballot(cl > thr);
            if (mm) {
                int src;
                if ((mm & (mm - 1)) == 0) {
                    src = __builtin_ctzll(mm);
                } else {
                    uint32_t key = cl > thr ? (cl << 16) | (0xffffu - ord) : 0u;
                    uint32_t mx = wave_max_dpp(key);
                    src = (int)(0xffffu - (mx & 0xffffu) - examined);
                }
                best = readlane(cl, src);
                bestq = readlane(q, src);
            }
            examined += npre;
            if (best >= nice || npre < 64 || examined >= C) break;
        }
        *q_out = bestq;
        return best > b0 ? best : 0u;
    }

    // ---- deflate_slow as a walk over match segments ----------------------------------------
    // From a fresh state at p (the start, or right after a match) zlib's lazy parse emits the
    // literals [p, t) and then the match at t: j = the first position >= p whose match is
    // usable, t = the end of the run of strict lazy improvements j, j+1, ... (each next
    // position's match longer than the pending one, while it is < 258); the next fresh state
    // is t + best_t.  Two bit masks built in parallel give j and t by find-first-set, so a
    // segment costs a few scalar steps plus one vector store of its literal run.  A segment
    // whose decisions touch a cut walk (M bit 31: longest_match not final) runs the exact
    // step-by-step loop (with search()) up to its match instead.
    __device__ void lit_run(uint32_t ntok, uint32_t p, uint32_t cnt) {
        for (uint32_t k = (uint32_t)lane_id(); k < cnt; k += 64) tok[ntok + k] = p + k;
    }
    __device__ uint32_t ffs_mask(PMC_LDS const uint64_t *m, uint32_t from, uint32_t nw) const {
        uint32_t w = from >> 6;
        if (w >= nw) return 0xffffffffu;
        uint64_t v = rfl64(m[w]) & (~0ull << (from & 63));
        while (!v) {
            if (++w >= nw) return 0xffffffffu;
            v = rfl64(m[w]);
        }
        return w * 64 + (uint32_t)__builtin_ctzll(v);
    }
    __device__ __noinline__ uint32_t parse(uint32_t npos, uint32_t len) {
        const uint32_t l = (uint32_t)lane_id();
        const uint32_t nw = (npos + 63) >> 6;
        for (uint32_t c0 = 0; c0 < npos; c0 += 64) {
            const uint32_t j = c0 + l;
            const uint32_t e = j < npos ? M[j] : 0u, e1 = j + 1 < npos ? M[j + 1] : 0u;
            const uint32_t best = e & 511, q = (e >> 9) & 0x7fffu, best1 = e1 & 511;
            const bool cut = (e >> 31) != 0;
            const bool usable = best >= 4 || (best == 3 && j - q <= 4096); // TOO_FAR
            const bool impr = best < 258 && j + 1 < npos && best1 > best;
            const uint64_t mL = ballot(j < npos && (usable || cut));
            const uint64_t mP = ballot(j < npos && (cut || !impr));
            if (l == 0) {
                ML[c0 >> 6] = mL;
                MP[c0 >> 6] = mP;
            }
        }
        wave_sync();
        uint32_t p = 0, ntok = 0;
        while (p < len) {
            const uint32_t j = ffs_mask(ML, p, nw);
            if (j == 0xffffffffu) { // no match ahead: literals to the end
                lit_run(ntok, p, len - p);
                ntok += len - p;
                break;
            }
            const uint32_t ej = rfl(M[j]);
            if (!(ej >> 31)) {
                const uint32_t t = ffs_mask(MP, j, nw); // exists: bit npos-1 is always set
                const uint32_t et = t == j ? ej : rfl(M[t]), bt = et & 511;
                bool ok = !(et >> 31);
                if (ok && bt < 258 && t + 1 < npos) {
                    const uint32_t e1 = rfl(M[t + 1]);
                    ok = !((e1 >> 31) && (e1 & 511) <= bt);
                }
                if (ok) {
                    lit_run(ntok, p, t - p);
                    ntok += t - p;
                    if (l == 0) tok[ntok] = ((t - ((et >> 9) & 0x7fffu)) << 16) | (bt - 3);
                    ntok++;
                    p = t + bt;
                    continue;
                }
            }
            // exact step-by-step deflate_slow up to the next match.  Positions [p, j) have no
            // usable match (and no cut walk), so the fresh state at p reaches j having emitted
            // the literals [p, j - 1) with b[j - 1] pending (when j > p) and match_length 2.
            stamp(2);
            if (j > p + 1) {
                lit_run(ntok, p, j - 1 - p);
                ntok += j - 1 - p;
            }
            uint32_t i = j, match_length = 2, match_start = 0, prev_length, prev_match;
            bool avail = j > p, matched = false;
            while (i < len) {
                prev_length = match_length;
                prev_match = match_start;
                match_length = 2;
                if (i + 3 <= len && prev_length < 258) {
                    const uint32_t e = rfl(M[i]);
                    uint32_t m = e & 511, q = (e >> 9) & 0x7fffu;
                    if (e >> 31) {
                        m = search<false>(i, prev_length, len, m, q, &q);
                        count(15);
                    }
                    else if (m <= prev_length) m = 0;
                    if (m) {
                        match_length = m;
                        match_start = q;
                        if (m == 3 && i - q > 4096) match_length = 2;
                    }
                }
                if (prev_length >= 3 && match_length <= prev_length) {
                    if (l == 0) tok[ntok] = ((i - 1 - prev_match) << 16) | (prev_length - 3);
                    ntok++;
                    i += prev_length - 1;
                    matched = true;
                    break;
                } else if (avail) {
                    if (l == 0) tok[ntok] = i - 1;
                    ntok++;
                    i++;
                } else {
                    avail = true;
                    i++;
                }
            }
            if (!matched && avail) {
                if (l == 0) tok[ntok] = i - 1;
                ntok++;
            }
            p = i;
            stamp(14);
        }
        wave_sync_global();
        return ntok;
    }

    // ---- deflate_slow with on-demand longest_match ------------------------------------------
    // Only positions the lazy parse visits need longest_match (about 15 % of the positions of
    // a 1 KiB JSON value that have chain candidates at all).  The parse runs serially on the
    // scalar unit; whenever it reaches a position with candidates whose result is not at hand,
    // one wave step evaluates that position and the following ones, each taking as many lanes
    // as it has chain candidates (capped at kPreCand, nearest first) until the 64 lanes are
    // used: each lane compares one (position, candidate) pair and an LDS max per position picks
    // (longest, then nearest).  A chain with more than kPreCand candidates is finished by
    // search() when the parse uses it.  Positions without candidates (CN = 0, HC bit clear)
    // are skipped in bulk as literals.
    // CN[x] = chain candidates of x = entries before x in its run of the hash-sorted order,
    // less position 0 (zlib's NIL: head[] value 0 never starts a match; the sort is stable,
    // so position 0 is the first entry of its run).  HC = CN > 0 as bits.
    // Returns 1 (uniform) when S is not the stable hash order: the sort's scatter slots come from
    // returning LDS atomics whose same-word lanes are assumed to get their old values in lane order
    // (measured on gfx950, not documented).  The guard checks what that order must produce -- (hash,
    // position) strictly increasing along S -- and the caller sends the value to the retry kernel
    // (per-lane counters, no atomic order) instead of parsing chains that may point forward.
    // has-candidate bits of positions 64 w .. 64 w + 63 (uniform): with the counts in R (PK > 0) a ballot of
    // them (one LDS read, as the HC word's), otherwise the HC word build_cn set
    template <int PK>
    __device__ __forceinline__ uint64_t hc_word(uint32_t w, uint32_t npos) const {
        if constexpr (PK > 0 && PMC_HC_FROM_R) {
            const uint32_t x = w * 64u + (uint32_t)lane_id();
            return ballot(x < npos && (uint32_t)R[x < npos ? x : 0u] >> (16 - PK) != 0u);
        } else {
            return rfl64(HC[w]);
        }
    }
    template <int PK>
    __device__ __forceinline__ uint32_t build_cn(uint32_t npos, uint32_t k0, uint32_t len_) {
        constexpr uint32_t RB = 16 - (PK > 0 ? PK : 0), CMAX = PK > 0 ? (1u << PK) - 1 : 255u;
        const uint32_t l = (uint32_t)lane_id();
        // has-candidate bits set by position below (HC as u32 words, LDS atomics): no second
        // pass over the positions.  (PK > 0: the walk takes them from R's counts, hc_word)
        constexpr bool kHc = !(PK > 0 && PMC_HC_FROM_R);
        if (kHc) {
            for (uint32_t k = l; k < (npos + 63) / 64 * 2; k += 64) ((PMC_LDS uint32_t *)HC)[k] = 0u;
            wave_sync();
        }
        uint32_t ph = 0xffffffffu, prs = 0, pq = 0; // previous chunk's last hash, run start, position
        uint32_t bad = 0;
        constexpr bool kPred = PK == 6 && PMC_EVAL_PRED;
        uint32_t pa[8] = {0, 0, 0, 0, 0, 0, 0, 0}; // (kPred) previous chunk's last 32 bytes
        for (uint32_t c0 = 0; c0 < npos; c0 += 64) {
            const uint32_t k = c0 + l;
            const bool valid = k < npos;
            const uint32_t p = valid ? sget<PK>(k) : 0u;
            uint32_t h;
            uint32_t a[8];
            if constexpr (kPred) { // 32 bytes at p; the nearest candidate's are lane l - 1's
                uint64_t A0, A1, A2 = 0, A3 = 0;
                load16(p, A0, A1);
                if (kPredCap > 16) load16(p + 16, A2, A3);
                a[0] = (uint32_t)A0, a[1] = (uint32_t)(A0 >> 32), a[2] = (uint32_t)A1, a[3] = (uint32_t)(A1 >> 32);
                a[4] = (uint32_t)A2, a[5] = (uint32_t)(A2 >> 32), a[6] = (uint32_t)A3, a[7] = (uint32_t)(A3 >> 32);
                h = valid ? hash3(a[0]) : 0xfffffffeu;
            } else {
                h = valid ? hash3(load4(p)) : 0xfffffffeu;
            }
            uint32_t hp = (uint32_t)__shfl_up((int)h, 1), pp = (uint32_t)__shfl_up((int)p, 1);
            hp = l == 0 ? ph : hp;
            pp = l == 0 ? pq : pp;
            if constexpr (kPred) {
                // match length with pp (same hash, not NIL), capped at 32 and at the bytes left
                uint32_t x8[8];
                constexpr int kW = kPredCap / 4;
#pragma unroll
                for (int i = 0; i < kW; i++) {
                    const uint32_t b = (uint32_t)__builtin_amdgcn_update_dpp((int)pa[i], (int)a[i], 0x138, 0xf, 0xf, false);
                    x8[i] = a[i] ^ b; // (wave_shr:1: lane 0 keeps the previous chunk's lane 63)
                    pa[i] = readlane(a[i], 63);
                }
                // leading equal bytes: the first differing dword's lowest set byte (kW * 4 when none)
                uint32_t m = 4u * kW;
#pragma unroll
                for (int i = kW - 1; i >= 0; i--) m = x8[i] ? 4u * i + ((uint32_t)__builtin_ctz(x8[i]) >> 3) : m;
                const uint32_t left = len_ - p;
                m = m < left ? m : left;
                m = valid && k != 0 && h == hp && pp != 0u ? m : 0u;
                if (valid) S[k] = (uint16_t)(p | m << 10);
            }
            // (hash, position) must increase: h > hp, or h == hp and p > pp (k = 0 has no predecessor)
            bad |= (valid && k != 0 && (h < hp || (h == hp && p <= pp))) ? 1u : 0u;
            uint32_t rs = wave_incl_max_dpp(valid && h != hp ? k : 0u);
            rs = rs > prs ? rs : prs;
            const uint32_t cnt = k - rs - (rs == k0 && k > rs ? 1u : 0u);
            if (valid) { // (the rank array R is written here, not by the sort)
                R[p] = (uint16_t)(PK > 0 ? k | (cnt < CMAX ? cnt : CMAX) << RB : k);
                if (PK == 0) CN[p] = (uint8_t)(cnt < 255 ? cnt : 255);
                if (kHc && cnt) lds_or((PMC_LDS uint32_t *)HC + (p >> 5), 1u << (p & 31));
            }
            ph = readlane(h, 63);
            prs = readlane(rs, 63);
            pq = readlane(p, 63);
        }
        wave_sync();
        return ballot(bad != 0u) ? 1u : 0u;
    }
    // results of the current eval: window start p0, evaluated offsets m (uniform) and, in
    // lane j, best | q << 9 | cut << 31 for position p0 + j
    struct Group {
        uint32_t p0;
        uint64_t m;
        uint32_t e;
        uint64_t stop; // offsets where a fresh-state walk stops: usable or cut, or not evaluated
        uint64_t fast; // evaluated, usable, not cut, and position + 1 does not improve on it
        uint64_t impr; // evaluated, usable, not cut, < 258, and position + 1 improves on it
        uint64_t cut;  // evaluated, walk cut short (search() decides)
        // Step records (lane o): the outcome of a fresh-state walk entering the window at offset
        // o, so a walk step is two v_readlane and one scalar branch instead of the mask shifts and
        // find-first-sets of the stop / cut / impr / fast tests on the scalar unit.
        //   w = type << 30 | pos << 24 | b   (FAST / PEND: pos = the match's offset t, whose
        //       length and source the walk reads from e; CUT: pos = the stop; JUMP: b = the
        //       offset to continue from, 0..64)
        uint32_t w;
    };
    static constexpr uint32_t kStepJump = 0, kStepCut = 1, kStepPend = 2, kStepFast = 3;
    static constexpr uint32_t kNoWindow = 0x80000000u; // a p0 no position reaches (i - p0 >= 64)
    // 16 bytes at p as two 8-byte words (5 dword reads + alignbyte)
    __device__ void load16(uint32_t p, uint64_t &lo, uint64_t &hi) const {
        const uint32_t w = p >> 2, sh = p & 3;
        const uint32_t w0 = bw[w], w1 = bw[w + 1], w2 = bw[w + 2], w3 = bw[w + 3], w4 = bw[w + 4];
        lo = (uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32 | __builtin_amdgcn_alignbyte(w1, w0, sh);
        hi = (uint64_t)__builtin_amdgcn_alignbyte(w4, w3, sh) << 32 | __builtin_amdgcn_alignbyte(w3, w2, sh);
    }
    // The eval is a chain of dependent LDS round trips (the wave waits on each), so it is laid
    // out to need few: (1) CN, CN + 1 and R of the window's positions; (2) each evaluated
    // position's first lane receives (offset, position, R) through one store + load, spread to
    // its other lanes by a max-scan; (3) the candidate S[R - d] and 16 bytes at the position;
    // (4) 16 bytes at the candidate; then 16 bytes per step while some lane still matches;
    // (5) an LDS max per position and its read-back.  Lanes outside the evaluated prefix
    // compute on clamped indices and contribute key 0 (no exec-mask branches).
    template <int PK>
    // (pend: the walk's pending match length at p0, 2 = none; it seeds PMC_EVAL_PRED's predicted walk)
    __device__ void eval_group(Group &g, uint32_t p0, uint32_t npos, uint32_t len, uint32_t pend = 2) {
        // SAT: a count field narrower than kPreCand saturates below it; such a position gets
        // kPreCand lanes whose candidates are validated (same hash, inside the array, not NIL) and
        // is marked cut (search() resumes it exactly if the parse needs it)
        constexpr uint32_t RB = 16 - (PK > 0 ? PK : 0), CMAX = PK > 0 ? (1u << PK) - 1 : PK < 0 ? 1u : 255u;
        constexpr bool SAT = CMAX < kPreCand;
        const uint32_t l = (uint32_t)lane_id();
        const uint32_t x = p0 + l;
        const uint32_t xc = x < npos ? x : 0u, x1 = x + 1 < npos ? x + 1 : 0u;
        uint32_t rx = R[xc], cn, cn1;
        if (PK > 0) {
            cn = rx >> RB;
            rx &= (1u << RB) - 1u;
        } else if (PK < 0) { // (no counts: 1 = has candidates, SAT)
            cn = (uint32_t)(HC[xc >> 6] >> (xc & 63)) & 1u;
        } else {
            cn = CN[xc];
        }
        cn = x < npos ? cn : 0u;
#if PMC_EVAL_CN1DPP
        // x + 1's count is lane l + 1's (one DPP move instead of an LDS read).  Lane 63 takes 1 ("x + 1 has
        // candidates"): offset 63 is then never a fast step, and the walk's general step decides it exactly.
        cn1 = (uint32_t)__builtin_amdgcn_update_dpp(1, (int)cn, 0x130, 0xf, 0xf, false); // wave_shl:1
        (void)x1;
#else
        if (PK > 0) cn1 = (uint32_t)R[x1] >> RB;
        else if (PK < 0) cn1 = (uint32_t)(HC[x1 >> 6] >> (x1 & 63)) & 1u;
        else cn1 = CN[x1];
        cn1 = x + 1 < npos ? cn1 : 0u;
#endif
        uint32_t gate = 1; // (PMC_EVAL_PRED: 0 for a position the predicted walk skips)
#if PMC_EVAL_PRED
        if constexpr (PK == 6) {
            // deflate_slow's lazy walk from p0 over the nearest candidates' match lengths (S bits 15:10):
            // from a fresh start s it visits s .. t, t the first position after s that does not improve
            // on its predecessor's length, and starts afresh at t - 1 + that length
            const uint32_t l1 = (uint32_t)S[rx] >> 10;
            const uint32_t ml = cn != 0u && l1 >= 3u ? l1 : 2u;
            const uint32_t mlp = (uint32_t)__builtin_amdgcn_update_dpp((int)pend, (int)ml, 0x138, 0xf, 0xf, false); // lane l - 1's; lane 0: pend
            const uint64_t hcm = ballot(cn != 0u), impm = ballot(ml > mlp);
            // per lane l, as a fresh start: T = the first later offset that does not improve (64: none), the
            // offsets it visits (rm: l .. T, or l alone without a match) and the next fresh start with
            // candidates (jn); the hops then cost two-three readlanes each on the scalar side
            const uint32_t lp1 = l + 1u;
            const uint64_t nim = lp1 < 64u ? ~impm & (~0ull << lp1) : 0ull;
            const uint32_t T = nim ? (uint32_t)__builtin_ctzll(nim) : 64u;
            const uint32_t mlt = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((T - 1u) & 63u) << 2), (int)ml);
            const uint32_t J = ml < 3u ? lp1 : T - 1u + mlt;
            const uint64_t hj = J < 64u ? hcm & (~0ull << J) : 0ull;
            const uint32_t jn = hj ? (uint32_t)__builtin_ctzll(hj) : 64u;
            const uint64_t rm = ml < 3u ? 1ull << l : (T >= 63u ? ~0ull : (2ull << T) - 1ull) & (~0ull << l);
            uint64_t inc = 1; // (offset 0: the position the walk asks for)
            uint32_t sp = 0;
            if (pend >= 3 && !(impm & 1)) { // a pending match that p0 does not improve on: next start p0 + pend - 1
                const uint64_t m = pend - 1u < 64u ? hcm & (~0ull << (pend - 1u)) : 0ull;
                sp = m ? (uint32_t)__builtin_ctzll(m) : 64u;
            }
#pragma unroll
            for (uint32_t h = 0; h < kPredHops; h++) {
                if (sp >= 64u) break;
                inc |= readlane64(rm, (int)sp);
                sp = readlane(jn, (int)sp);
            }
            if (sp < 64u) inc |= ~0ull << sp; // (past the hop limit: the rest of the window in order)
            gate = (uint32_t)(inc >> l) & 1u;
        }
#endif
        const uint32_t w0 = gate == 0u ? 0u : SAT && cn == CMAX ? kPreCand : cn < kPreCand ? cn : kPreCand;
        const uint32_t w = w0; // lanes of this position
        const uint32_t incl = wave_incl_scan_dpp(w), offs = incl - w;
        const bool inc = w != 0 && incl <= 64;
        const uint64_t im = ballot(inc); // evaluated (lane-owning) offsets
        const uint32_t nl = im ? readlane(incl, 63 - __builtin_clzll(im)) : 0u;
#ifdef PMC_STAMPS
        st[7] += nl; // (stamps build: lanes used per eval)
#endif
        // first lane of each evaluated offset j: offs << 26 | (j + 1) << 19 | R (offs grows with j,
        // so a max-scan hands every lane its owner); other lanes store to dummy slots
        PMC_LDS uint32_t *dmy = EV + 64; // (the u8 mark area, 16 words)
        EV[l] = 0;
        (inc ? EV : dmy)[inc ? offs : (l & 15)] = offs << 26 | (l + 1) << 19 | rx;
        wave_sync();
        const uint32_t mk = EV[l];
        // (LDS keeps one wave's accesses in order: the read above sees the marks)
        // Values of <= 4 KiB (PK > 0 always) take each offset's maximum by the segmented max-scan below,
        // which stores every evaluated offset's word: no reset for them (a non-evaluated offset's word is
        // never read: its walk masks come from the counts).  The atomic-max path needs zeros.
        constexpr bool kSegOnly = PK > 0;
        if (!kSegOnly) EV[l] = 0;
        const bool v = l < nl;
        const uint32_t sc = wave_incl_max_dpp(mk);
        const uint32_t own = v ? ((sc >> 19) & 127) - 1 : 0u;
        const uint32_t P = p0 + own, d = l - (sc >> 26) + 1; // the lane's candidate: the d-th nearest
        const uint32_t rxo = sc & 0xffffu;
        uint32_t q = sget<PK>(v && (!SAT || rxo >= d) ? rxo - d : 0u);
        uint64_t A0, A1, B0, B1;
        load16(P, A0, A1);
        q = v ? q : 0u;
        load16(q, B0, B1);
        // (SAT) lanes past the chain: another hash, below the array, or position 0 (NIL)
        const bool vk = v && (!SAT || (rxo >= d && q != 0u && hash3((uint32_t)A0) == hash3((uint32_t)B0)));
        const uint32_t nice = (len - P) < 258 ? (len - P) : 258;
        // (branch-free on the vector ALU: 0/1 integers and products instead of bools and
        // selects, which became exec-mask and lane-mask work on the saturated scalar unit)
        auto eq16 = [](uint64_t z0, uint64_t z1) { // equal leading bytes of 16 (16 when equal)
            const uint32_t c0 = eq_bytes8(z0);
            return c0 + (c0 >> 3) * eq_bytes8(z1);
        };
        auto is0 = [](uint64_t z0, uint64_t z1) { // 1 iff both words are zero
            const uint32_t t = (uint32_t)z0 | (uint32_t)(z0 >> 32) | (uint32_t)z1 | (uint32_t)(z1 >> 32);
            return 1u >> (t < 1u ? t : 1u);
        };
        const uint64_t y0 = A0 ^ B0, y1 = A1 ^ B1;
        uint32_t cl = eq16(y0, y1);
        uint32_t ext = (v ? 1u : 0u) & is0(y0, y1) & ((16u - nice) >> 31);
        asm volatile("" : "+v"(ext));
        uint32_t off = 16;
        while (ballot(ext != 0u)) {
            count(8);
            // (lane masks, not products with ext: a 32-bit multiply is a quarter-rate VALU op)
            const uint32_t xm = 0u - ext;
            uint64_t C0, C1, D0, D1;
            load16((P + off) & xm, C0, C1);
            load16((q + off) & xm, D0, D1);
            const uint64_t z0 = C0 ^ D0, z1 = C1 ^ D1;
            cl = ((off + eq16(z0, z1)) & xm) | (cl & ~xm);
            ext &= is0(z0, z1) & ((off + 16u - nice) >> 31);
            off += 16;
        }
        cl = cl < nice ? cl : nice;
        uint32_t kk; // offset l's result: best << 23 | nearness << 18 | q
        if (kSegOnly || sflag(len <= 4096 ? 1u : 0u)) {
            // An offset's lanes are contiguous and own grows with the lane: an inclusive max-scan of
            // own << 26 | (cl, nearness, q) leaves each offset's maximum in its last lane.
            // No same-address LDS atomics: the lanes of one position used to serialise on its word (round 4:
            // front 194 -> 185 ms at 1 KiB).  Positions < 4096 at these sizes, so q takes 12 bits.
            const uint32_t k2 = own << 26 | (vk ? cl << 17 | (kPreCand - d) << 12 | q : 0u);
            const uint32_t mx = wave_incl_max_dpp(k2);
#if PMC_EVAL_BPERM
            // offset l reads its maximum from its last lane, incl - 1, by one ds_bpermute (no exec-masked
            // store, wave sync and read back); an offset without lanes reads some lane's word, which nothing
            // uses (its walk masks come from the counts)
            const uint32_t m = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((incl - 1u) & 63u) << 2), (int)mx) &
                               0x3ffffffu;
            kk = (m >> 17) << 23 | ((m >> 12) & 31u) << 18 | (m & 4095u);
#else
            const uint32_t onx = (uint32_t)__builtin_amdgcn_update_dpp(64, (int)own, 0x130, 0xf, 0xf, false); // lane l + 1
            if (v && (l + 1 >= nl || onx != own)) {
                const uint32_t m = mx & 0x3ffffffu;
                EV[own] = (m >> 17) << 23 | ((m >> 12) & 31u) << 18 | (m & 4095u);
            }
            wave_sync();
            kk = EV[l];
#endif
        } else {
            __hip_atomic_fetch_max(&EV[own], vk ? cl << 23 | (kPreCand - d) << 18 | q : 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
            wave_sync();
            kk = EV[l];
        }
        const uint32_t best = kk >> 23;
        const uint32_t nx = (len - x) < 258 ? (len - x) : 258;
        auto neg = [](uint32_t d) { return d >> 31; }; // 1 iff d < 0 as int (all values here are small)
        uint32_t cutc = (SAT ? (cn == CMAX ? 1u : 0u) : neg(kPreCand - cn)) & neg(best - nx);
        const uint32_t bq = kk & 0x7fffu, e = best | bq << 9 | cutc << 31; // (positions < 32768)
        g.p0 = p0;
        g.m = im;
        g.e = e;
        // Walk masks (the fast path of deflate_slow, per offset); e of offset l + 1 via DPP.
        // The conditions are 0/1 integers (sign bits of differences of small values), so they
        // combine on the vector ALU: as bools they became lane-mask logic on the scalar unit,
        // which this kernel saturates.
        const uint32_t en = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, 0x130, 0xf, 0xf, false); // wave_shl:1
        const uint64_t imv = im >> l;
        uint32_t ev = (uint32_t)imv & 1u, ev1 = (uint32_t)(imv >> 1) & 1u; // (lane 63: im >> 64 is 0)
        const uint32_t ge4 = neg(3u - best), eq3 = neg((best ^ 3u) - 1u), near = neg(x - bq - 4097u);
        uint32_t usable = ge4 | (eq3 & near);                                // TOO_FAR
        const uint32_t enb = en & 511u, enc = en >> 31, le = neg(best - enb) ^ 1u, ge258 = neg(257u - best);
        const uint32_t cn1z = neg(cn1 - 1u), cnnz = neg(cn - 1u) ^ 1u;
        asm volatile("" : "+v"(ev), "+v"(ev1), "+v"(usable), "+v"(cutc)); // (keep them integers)
        const uint32_t no_impr = ge258 | cn1z | (ev1 & (enc ^ 1u) & le);
        const uint32_t impr = (ge258 ^ 1u) & ev1 & (enc ^ 1u) & (le ^ 1u);
        const uint32_t okfast = ev & usable & (cutc ^ 1u);
        g.stop = ballot(((ev & (usable | cutc)) | ((ev ^ 1u) & cnnz)) != 0u);
        g.fast = ballot((okfast & no_impr) != 0u);
        g.impr = ballot((okfast & impr) != 0u);
        g.cut = ballot((ev & cutc) != 0u);
        // step record of lane l (vector ALU; the masks are uniform): the first stop sj >= l, and
        // from a usable sj the end st of its run of lazy improvements (impr bit 63 is clear)
        const uint64_t sx = g.stop & (~0ull << l);
        const uint32_t sj = sx ? (uint32_t)__builtin_ctzll(sx) : 64u, sjc = sj & 63u;
        const uint32_t st = (uint32_t)__builtin_ctzll(~g.impr & (~0ull << sjc));
        const uint32_t evs = (uint32_t)(g.m >> sjc) & (sj < 64 ? 1u : 0u), cts = (uint32_t)(g.cut >> sjc) & 1u;
        const uint32_t fst = (uint32_t)(g.fast >> st) & 1u;
        const uint32_t ty = evs ? (cts ? kStepCut : fst ? kStepFast : kStepPend) : kStepJump;
        const uint32_t pos = cts ? sjc : st;
        g.w = ty << 30 | pos << 24 | sj;
    }
    // Token sink: tokens collect in one VGPR (lane k holds token 64 * block + k) and leave
    // with one coalesced store per 64 tokens, so emitting costs no exec-masked stores.
    struct TokBuf {
        uint32_t v = 0, n = 0;
    };
    __device__ void tb_flush(TokBuf &t) { tok[t.n - 64 + (uint32_t)lane_id()] = t.v; }
    __device__ void tb_put(TokBuf &t, uint32_t x) {
        t.v = (uint32_t)lane_id() == (t.n & 63) ? x : t.v;
        t.n++;
        if ((t.n & 63) == 0) tb_flush(t);
    }
    // literal tokens for positions p .. p + cnt - 1
    __device__ void tb_run(TokBuf &t, uint32_t p, uint32_t cnt) {
        const uint32_t l = (uint32_t)lane_id();
        while (cnt) {
            count(7);
            const uint32_t o = t.n & 63, take = cnt < 64 - o ? cnt : 64 - o;
            t.v = l - o < take ? p + (l - o) : t.v;
            t.n += take;
            p += take;
            cnt -= take;
            if ((t.n & 63) == 0) tb_flush(t);
        }
    }
    __device__ void tb_finish(TokBuf &t) {
        const uint32_t l = (uint32_t)lane_id();
        if (l < (t.n & 63)) tok[(t.n & ~63u) + l] = t.v;
    }
    // Implied literals: tokens cover the positions in order, so the literals between two matches
    // are the run [lf, s) up to the next match's start s.  The parse only tracks lf; each match
    // stores its run and itself with lane-parallel stores (lane k: token n + k), and the tail run
    // [lf, len) goes out at the end -- no per-literal bookkeeping on the scalar unit.
    __device__ void tb_match(TokBuf &t, uint32_t lf, uint32_t s, uint32_t m) {
        const uint32_t l = (uint32_t)lane_id(), nl = s - lf, cnt = nl + 1;
        // first 64 tokens with every lane storing (no exec mask work on the scalar unit): lanes
        // past the run repeat the match token at its own slot, so no byte past it is written
        {
            const uint32_t k = l < nl ? l : nl;
            tok[t.n + k] = k < nl ? lf + k : m;
        }
        if (cnt > 64) {
            for (uint32_t b = 64; b < cnt; b += 64) {
                const uint32_t k = b + l;
                if (k < cnt) tok[t.n + k] = k < nl ? lf + k : m;
            }
        }
        t.n += cnt;
    }
    __device__ void tb_lits(TokBuf &t, uint32_t lf, uint32_t e) {
        const uint32_t l = (uint32_t)lane_id(), cnt = e - lf;
        for (uint32_t b = 0; b < cnt; b += 64) {
            const uint32_t k = b + l;
            if (k < cnt) tok[t.n + k] = lf + k;
        }
        t.n += cnt;
    }
    // longest_match record of has-candidate position x (evaluating a new window if needed)
    template <int PK>
    __device__ uint32_t group_get(Group &g, uint32_t x, uint32_t npos, uint32_t len, uint32_t pend) {
        const uint32_t off = x - g.p0;
        if (off < 64 && ((g.m >> off) & 1)) return readlane(g.e, (int)off);
        stamp(2);
        eval_group<PK>(g, x, npos, len, pend);
        stamp(10);
        count(13);
        return readlane(g.e, 0);
    }
    // (a noinline member reaches the wave state through `this`, a pointer to scratch: every
    // member pointer would be re-read from memory inside the loop.  A local copy lives in SGPRs.)
    template <int PK>
    // (k0_: the rank of position 0, from sort_positions2; build_cn needs it before R exists)
    __device__ __forceinline__ uint32_t parse_ondemand(uint32_t npos_, uint32_t len_, uint32_t k0_) {
        SmallWave me = *this;
        const uint32_t r = me.parse_ondemand_body<PK>(npos_, len_, k0_);
#ifdef PMC_STAMPS
        for (int k = 0; k < 16; k++) st[k] = me.st[k];
        t_last = me.t_last;
#endif
        return r;
    }
    template <int PK>
    __device__ __forceinline__ uint32_t parse_ondemand_body(uint32_t npos_, uint32_t len_, uint32_t k0_) {
        const uint32_t npos = rfl(npos_), len = rfl(len_); // (arguments arrive in VGPRs)
        const uint32_t nw = (npos + 63) >> 6;
        if (sflag(build_cn<PK>(npos, rfl(k0_), len))) return kNtokRetry; // (the sort's lane-order guard)
        stamp(11);
        PMC_STOP(13, 0)
        Group g;
        g.p0 = kNoWindow;
        g.m = g.stop = g.fast = g.impr = g.cut = 0;
        g.e = 0;
        TokBuf tb;
        uint32_t i = 0, ml = 2, ms = 0, lf = 0; // lf: first position of the pending literal run
        uint32_t hci = 0;              // HC word cached in SGPRs
        uint64_t hcw = hc_word<PK>(0, npos);
#ifdef PMC_STAMPS
        // eval usage (stamps build): st[3] evaluated positions, st[4] those the walk consumed,
        // st[5] evals started inside the previous window's 64-position span
        uint64_t d_used = 0;
        uint32_t d_p0 = kNoWindow;
        auto d_use = [&](uint32_t a, uint32_t b) { // offsets a..b of the current window
            if (a < 64) d_used |= (b >= 63 ? ~0ull : ((2ull << b) - 1)) & (~0ull << a);
        };
        auto d_eval = [&](uint32_t newp0) {
            if (d_p0 != kNoWindow) {
                st[3] += (uint64_t)__builtin_popcountll(g.m);
                st[4] += (uint64_t)__builtin_popcountll(g.m & d_used);
                st[5] += newp0 - d_p0 < 64 ? 1u : 0u;
            }
            d_used = 0;
            d_p0 = newp0;
        };
#define PMC_D_EVAL(x) d_eval(x)
#define PMC_D_USE(a, b) d_use(a, b)
#else
#define PMC_D_EVAL(x)
#define PMC_D_USE(a, b)
#endif
        while (i < len) {
            // (the parse state is wave-uniform: keep it in SGPRs so control stays scalar)
            i = rfl(i);
            ml = rfl(ml);
            ms = rfl(ms);
            lf = rfl(lf);
            tb.n = rfl(tb.n);
            count(14);
            if (ml == 2) {
                // Fresh state.  Inside the current window the step record of offset i - p0 holds
                // the whole step (positions without candidates are never stops, so no HC scan is
                // needed there); otherwise jump to the next position with candidates and
                // evaluate a window there.  Fast steps and jumps stay in this inner loop, whose
                // few loop-carried values keep the scalar latch short; a pending lazy match or a
                // cut walk leaves it for the general step.
                uint32_t W = 0, off = 0;
                for (;;) {
                    off = i - g.p0;
                    if (off >= 64) {
                        uint32_t j = len;
                        uint32_t w = i >> 6;
                        if (w < nw) {
                            if (w != hci) {
                                hci = w;
                                hcw = hc_word<PK>(w, npos);
                            }
                            uint64_t m = hcw & (~0ull << (i & 63));
                            while (!m && ++w < nw) {
                                hci = w;
                                hcw = hc_word<PK>(w, npos);
                                m = hcw;
                            }
                            if (m) j = w * 64 + (uint32_t)__builtin_ctzll(m);
                        }
                        i = j;
                        if (i >= len) break;
                        stamp(2);
                        PMC_D_EVAL(i);
                        eval_group<PK>(g, i, npos, len);
                        stamp(10);
                        count(13);
                        off = 0;
                    }
                    W = readlane(g.w, (int)off);
                    const uint32_t ty = W >> 30;
                    PMC_D_USE(off, ty == kStepJump ? (W & 127u) - 1u : (W >> 24) & 63u);
                    if (ty == kStepJump) { // no decision in this window from here: a new one at p0 + b
                        i = g.p0 + (W & 127u);
                        g.p0 = kNoWindow;
                        continue;
                    }
                    if (ty != kStepFast) break;
                    // literals up to the match at t, then the match
                    const uint32_t st = (W >> 24) & 63u, t = g.p0 + st, e0 = readlane(g.e, (int)st);
                    const uint32_t b0 = e0 & 511u, q0 = (e0 >> 9) & 0x7fffu;
                    tb_match(tb, lf, t, (t - q0) << 16 | (b0 - 3u));
                    i = t + b0;
                    lf = i;
                    if (i >= len) break;
                }
                if (i >= len) break;
                const uint32_t ps = g.p0 + ((W >> 24) & 63u);
                if ((W >> 30) == kStepPend) { // t + 1 may improve on t's match (cut or unevaluated)
                    i = ps + 1;
                    const uint32_t e0 = readlane(g.e, (int)((W >> 24) & 63u));
                    ml = e0 & 511u;
                    ms = (e0 >> 9) & 0x7fffu;
                    continue;
                }
                i = ps; // a cut walk: the general step decides
            }
            count(9);
            const uint32_t pl = ml, pm = ms;
            ml = 2;
            if (sflag((i < npos ? 1u : 0u) & (pl < 258 ? 1u : 0u))) {
                if ((i >> 6) != hci) {
                    hci = i >> 6;
                    hcw = hc_word<PK>(hci, npos);
                }
                if (sflag((uint32_t)(hcw >> (i & 63)) & 1u)) {
#ifdef PMC_STAMPS
                    if (!(i - g.p0 < 64 && ((g.m >> (i - g.p0)) & 1))) PMC_D_EVAL(i);
                    PMC_D_USE(i - g.p0, i - g.p0);
#endif
                    const uint32_t e = group_get<PK>(g, i, npos, len, pl);
                    uint32_t m = e & 511, q = (e >> 9) & 0x7fffu;
                    if (e >> 31) {
                        stamp(2);
                        m = search<PK>(i, pl, len, m, q, &q);
                        stamp(12);
                        count(15);
                    } else if (m <= pl) {
                        m = 0;
                    }
                    if (m) {
                        ml = m;
                        ms = q;
                        if (m == 3 && i - q > 4096) ml = 2; // TOO_FAR
                    }
                }
            }
            if (sflag((pl >= 3 ? 1u : 0u) & (ml <= pl ? 1u : 0u))) {
                tb_match(tb, lf, i - 1, ((i - 1 - pm) << 16) | (pl - 3));
                i += pl - 1;
                lf = i;
                ml = 2;
            } else {
                i++;
            }
        }
        tb_lits(tb, lf, len);
        wave_sync_global();
        return rfl(tb.n);
    }

    // build_tree's heapify + merge loop (trees.c) on a register heap; returns the next
    // node id (root = result - 1).  Father links go to dad[] (lane 0 stores).
    template <class Heap>
    __device__ int heap_merge(Heap &hp, int heap_len, int elems, bool &deep) {
        const int l = lane_id();
        for (int n = heap_len / 2; n >= 1; n--) hp.down(n, heap_len);
        int node = elems;
        do {
            const uint32_t n = hp.get(1);
            hp.set(1, hp.get(heap_len));
            hp.set(heap_len, ~0u);
            heap_len--;
            hp.down(1, heap_len);
            const uint32_t m = hp.get(1);
            const uint32_t kn = n >> 10, km = m >> 10;
            const uint32_t dn = kn & 31, dm = km & 31;
            const uint32_t d = (dn >= dm ? dn : dm) + 1;
            deep |= d >= 31;
            const uint32_t key = (((kn >> 5) + (km >> 5)) << 5) | (d & 31);
            dad[n & 1023] = (uint16_t)node; // (all lanes store the same value: no exec change)
            dad[m & 1023] = (uint16_t)node;
            hp.set(1, (key << 10) | (uint32_t)node);
            node++;
            hp.down(1, heap_len);
        } while (heap_len >= 2);
        return node;
    }

    // ---- Huffman: build_tree for one tree -------------------------------------------------
    // freq[0..elems) in LDS (u32).  Writes code_out[s] = bitrev code | len << 16 for
    // s <= max_code (0 for unused), returns zlib's opt_len/static_len contributions.
    __device__ __noinline__ TreeOut build_tree(PMC_LDS uint32_t *freq, int elems, const CtData *stree,
                                               const uint8_t *extra, int extra_base, int max_length,
                                               PMC_LDS uint32_t *code_out) {
        const int l = lane_id();
        TreeOut to{};
        // 1. leaves in symbol order -> staging (code_out reused) at heap index 1..k
        int heap_len = 0, max_code = -1;
        for (int c0 = 0; c0 < elems; c0 += 64) {
            const int s = c0 + l;
            const uint32_t f = s < elems ? freq[s] : 0u;
            const uint64_t nz = ballot(f != 0);
            if (f) code_out[heap_len + 1 + popc_lt(nz)] = ((f << 5) << 10) | (uint32_t)s;
            if (nz) max_code = c0 + 63 - __builtin_clzll(nz);
            heap_len += __builtin_popcountll(nz);
        }
        wave_sync();
        // dummies (build_tree: while (heap_len < 2))
        int64_t opt = 0, stat = 0;
        // (all control values stay wave-uniform -- only the LDS stores are lane-guarded --
        //  so the heap loop below compiles to scalar control flow)
        int d0 = -1, d1 = -1;
        if (heap_len < 2) {
            d0 = max_code < 2 ? ++max_code : 0;
            opt -= 1;
            if (stree) stat -= stree[d0].dl;
            if (heap_len + 1 < 2) {
                d1 = max_code < 2 ? ++max_code : 0;
                opt -= 1;
                if (stree) stat -= stree[d1].dl;
            }
        }
        to.dummy[0] = d0;
        to.dummy[1] = d1;
        if (l == 0) {
            if (d0 >= 0) {
                code_out[heap_len + 1] = ((1u << 5) << 10) | (uint32_t)d0;
                freq[d0] = 1;
            }
            if (d1 >= 0) {
                code_out[heap_len + 2] = ((1u << 5) << 10) | (uint32_t)d1;
                freq[d1] = 1;
            }
        }
        heap_len = rfl(heap_len + (d0 >= 0) + (d1 >= 0));
        max_code = rfl(max_code);
        wave_sync();
        stamp(3);
        // 2. heapify + merge (all uniform scalar control; the heap never leaves VGPRs)
        int node;
        bool deep = false;
        if (heap_len < 64) {
            RegHeap1 hp;
            hp.h = l >= 1 && l <= heap_len ? code_out[l] : ~0u;
            node = heap_merge(hp, heap_len, elems, deep);
        } else if (heap_len < 128) {
            RegHeap2 hp;
            hp.h0 = 2 * l >= 1 && 2 * l <= heap_len ? code_out[2 * l] : ~0u;
            hp.h1 = 2 * l + 1 <= heap_len ? code_out[2 * l + 1] : ~0u;
            node = heap_merge(hp, heap_len, elems, deep);
        } else {
            RegHeap hp;
            hp.h0 = code_out[l];
            hp.h1 = code_out[64 + l];
            hp.h2 = code_out[128 + l];
            hp.h3 = code_out[192 + l];
            hp.h4 = code_out[256 + l < 288 ? 256 + l : 287];
            node = heap_merge(hp, heap_len, elems, deep);
        }
        const int root = node - 1;
        if (l == 0) dad[root] = (uint16_t)root;
        wave_sync();
        stamp(9);
        // 3. depth of every node by pointer jumping over the father links (depth <= 21)
        for (int x = l; x < node; x += 64) {
            bool in_tree = x >= elems || (x <= max_code && freq[x] != 0);
            if (!in_tree) dad[x] = (uint16_t)x;
            dep[x] = (in_tree && x != root) ? 1 : 0;
        }
        wave_sync();
        for (int it = 0; it < 5; it++) {
            uint32_t na[9], nd[9];
#pragma unroll
            for (int j = 0; j < 9; j++) {
                int x = l + 64 * j;
                if (x < node) {
                    uint32_t a = dad[x];
                    na[j] = dad[a];
                    nd[j] = (uint32_t)dep[x] + dep[a];
                }
            }
            wave_sync();
#pragma unroll
            for (int j = 0; j < 9; j++) {
                int x = l + 64 * j;
                if (x < node) {
                    dad[x] = (uint16_t)na[j];
                    dep[x] = (uint8_t)nd[j];
                }
            }
            wave_sync();
        }
        stamp(10);
        // 4. code lengths, overflow check, opt_len / static_len sums
        uint32_t over = 0;
        int64_t po = 0, ps = 0;
        for (int s = l; s <= max_code; s += 64) {
            uint32_t f = freq[s];
            uint32_t len = f ? dep[s] : 0u;
            over |= len > (uint32_t)max_length;
            uint32_t xb = s >= extra_base ? extra[s - extra_base] : 0u;
            po += (int64_t)f * (len + xb);
            if (stree) ps += (int64_t)f * (stree[s].dl + xb);
        }
        over = ballot(over != 0) != 0 || deep;
        to.overflow = over;
        po = (int64_t)wave_sum_u32((uint32_t)po);
        ps = (int64_t)wave_sum_u32((uint32_t)ps);
        to.opt = opt + po;
        to.stat = stat + ps;
        to.max_code = max_code;
        if (over) return to;
        stamp(11);
        // 5. gen_codes: canonical code = next_code[len] + rank among equal lengths
        uint32_t bl_count[16];
#pragma unroll
        for (int L = 0; L < 16; L++) bl_count[L] = 0;
        for (int c0 = 0; c0 <= max_code; c0 += 64) {
            const int s = c0 + l;
            const uint32_t len = (s <= max_code && freq[s]) ? dep[s] : 0u;
#pragma unroll
            for (int L = 1; L <= 15; L++) bl_count[L] += __builtin_popcountll(ballot(len == (uint32_t)L));
        }
        uint32_t next_code[16];
        uint32_t code = 0;
        next_code[0] = 0;
#pragma unroll
        for (int L = 1; L <= 15; L++) {
            code = (code + (L > 1 ? bl_count[L - 1] : 0u)) << 1;
            next_code[L] = code;
        }
        // (every entry below elems is written: the staging area left heap entries there)
        for (int c0 = 0; c0 < elems; c0 += 64) {
            const int s = c0 + l;
            const uint32_t len = (s <= max_code && freq[s]) ? dep[s] : 0u;
            uint32_t mycode = 0;
#pragma unroll
            for (int L = 1; L <= 15; L++) {
                const uint64_t mk = ballot(len == (uint32_t)L);
                if (len == (uint32_t)L) mycode = next_code[L] + popc_lt(mk);
                next_code[L] += __builtin_popcountll(mk);
            }
            if (s < elems)
                code_out[s] = len ? ((__builtin_bitreverse32(mycode) >> (32 - len)) | (len << 16)) : 0u;
        }
        wave_sync();
        stamp(12);
        return to;
    }

    // per maximal run of code lengths (value v, length R): bl-code counts (scan_tree)
    // R / 6 and R / 138 for run lengths R <= 288 by 24-bit multiplies (full-rate VALU ops; the
    // compiler's reciprocal divisions used quarter-rate 32-bit ones): exact for R < 32768 / 527
    __device__ static uint32_t div6(uint32_t x) { return __umul24(x, 10923u) >> 16; }
    __device__ static uint32_t div138(uint32_t x) { return __umul24(x, 475u) >> 16; }
    __device__ static void run_counts(uint32_t v, uint32_t R, PMC_LDS uint32_t *blfreq) {
        if (v) {
            uint32_t c1 = R < 7 ? R : 7, rem = R - c1, full = div6(rem), last = rem - __umul24(full, 6u);
            uint32_t nv = (c1 < 4 ? c1 : 1) + (last < 3 ? last : 0);
            uint32_t n16 = (c1 >= 4 ? 1 : 0) + full + (last >= 3 ? 1 : 0);
            if (nv) lds_add(&blfreq[v], nv);
            if (n16) lds_add(&blfreq[16], n16);
        } else {
            uint32_t full = div138(R), last = R - __umul24(full, 138u);
            uint32_t n18 = full + (last > 10 ? 1 : 0), n17 = (last >= 3 && last <= 10) ? 1 : 0;
            uint32_t n0 = last < 3 ? last : 0;
            if (n0) lds_add(&blfreq[0], n0);
            if (n17) lds_add(&blfreq[17], n17);
            if (n18) lds_add(&blfreq[18], n18);
        }
    }
    // bits of one run (send_tree), closed form of run_bits' count
    __device__ uint32_t run_nbits(uint32_t v, uint32_t R) const {
        const uint32_t Lv = blcode[v] >> 16;
        if (v) {
            const uint32_t L16 = (blcode[16] >> 16) + 2;
            const uint32_t c1 = R < 7 ? R : 7, rem = R - c1, full = div6(rem), last = rem - __umul24(full, 6u);
            uint32_t n = c1 < 4 ? __umul24(c1, Lv) : Lv + L16;
            n += __umul24(full, L16);
            n += last ? (last < 3 ? __umul24(last, Lv) : L16) : 0u;
            return n;
        }
        const uint32_t L17 = (blcode[17] >> 16) + 3, L18 = (blcode[18] >> 16) + 7;
        const uint32_t full = div138(R), last = R - __umul24(full, 138u);
        return __umul24(full, L18) + (last ? (last < 3 ? __umul24(last, Lv) : last <= 10 ? L17 : L18) : 0u);
    }
    // bits of one run (send_tree); emit into the image at pos when write (the run's codes are
    // gathered in a 64-bit register and ORed into the image a register at a time)
    __device__ uint32_t run_bits(uint32_t v, uint32_t R, uint64_t pos, bool write) {
        uint64_t accv = 0;
        uint32_t accn = 0;
        auto put = [&](uint32_t c, uint32_t xv, uint32_t xn, uint32_t &acc) {
            uint32_t cw = blcode[c], cn = cw >> 16;
            if (write) {
                if (accn > 48) { // (one code with extra bits is at most 7 + 7 bits)
                    or_bits_lds(pos + acc - accn, accv, (int)accn);
                    accv = 0;
                    accn = 0;
                }
                accv |= ((uint64_t)(cw & 0xffff) | ((uint64_t)xv << cn)) << accn;
                accn += cn + xn;
            }
            acc += cn + xn;
        };
        uint32_t acc = 0;
        if (v) {
            uint32_t c1 = R < 7 ? R : 7, rem = R - c1, full = div6(rem), last = rem - __umul24(full, 6u);
            if (c1 < 4) {
                for (uint32_t k = 0; k < c1; k++) put(v, 0, 0, acc);
            } else {
                put(v, 0, 0, acc);
                put(16, c1 - 4, 2, acc);
            }
            for (uint32_t k = 0; k < full; k++) put(16, 3, 2, acc);
            if (last) {
                if (last < 3) {
                    for (uint32_t k = 0; k < last; k++) put(v, 0, 0, acc);
                } else {
                    put(16, last - 3, 2, acc);
                }
            }
        } else {
            uint32_t full = div138(R), last = R - __umul24(full, 138u);
            for (uint32_t k = 0; k < full; k++) put(18, 127, 7, acc);
            if (last) {
                if (last < 3) {
                    for (uint32_t k = 0; k < last; k++) put(0, 0, 0, acc);
                } else if (last <= 10) {
                    put(17, last - 3, 3, acc);
                } else {
                    put(18, last - 11, 7, acc);
                }
            }
        }
        if (write && accn) or_bits_lds(pos + acc - accn, accv, (int)accn);
        return acc;
    }
    __device__ void or_bits_lds(uint64_t pos, uint64_t v, int n) {
        if (n == 0) return;
        uint64_t w = pos >> 5;
        int s = (int)(pos & 31);
        uint32_t lo = (uint32_t)(v << s);
        uint32_t mid = (uint32_t)(s ? (v >> (32 - s)) : (v >> 32));
        uint32_t hi = s ? (uint32_t)(v >> (64 - s)) : 0u;
        if (lo) lds_or(&outw[w], lo);
        if (n + s > 32 && mid) lds_or(&outw[w + 1], mid);
        if (n + s > 64 && hi) lds_or(&outw[w + 2], hi);
    }

    // scan_tree for lengths code[0..max_code]: records run lengths at run starts into
    // runR (u16) and adds the bl counts.  Chunks are walked back to front so each run
    // start knows where the next run begins.
    template <bool COUNT = true>
    __device__ void scan_runs(PMC_LDS const uint32_t *code, int max_code, PMC_LDS uint16_t *runR) {
        const int l = lane_id();
        int next_start = max_code + 1;
        for (int c0 = (max_code / 64) * 64; c0 >= 0; c0 -= 64) {
            const int s = c0 + l;
            const bool in = s <= max_code;
            const uint32_t v = in ? code[s] >> 16 : 0xffffu;
            const uint32_t vp = (in && s > 0) ? code[s - 1] >> 16 : 0xfffeu;
            const bool start = in && (s == 0 || v != vp);
            const uint64_t m = ballot(start);
            const uint64_t above = l == 63 ? 0 : (m & (~0ull << (l + 1)));
            const int nxt = above ? c0 + __builtin_ctzll(above) : next_start;
            if (start) {
                runR[s] = (uint16_t)(nxt - s);
                if (COUNT) run_counts(v, (uint32_t)(nxt - s), blfreq);
            }
            if (m) next_start = c0 + __builtin_ctzll(m);
        }
    }
    // send_tree: every run start writes its symbols at its prefix offset; returns bits
    __device__ uint64_t send_runs(PMC_LDS const uint32_t *code, int max_code, PMC_LDS const uint16_t *runR,
                                  uint64_t pos) {
        const int l = lane_id();
        uint64_t base = pos;
        for (int c0 = 0; c0 <= max_code; c0 += 64) {
            const int s = c0 + l;
            const bool in = s <= max_code;
            const uint32_t v = in ? code[s] >> 16 : 0u;
            const uint32_t vp = (in && s > 0) ? code[s - 1] >> 16 : 0xfffeu;
            const bool start = in && (s == 0 || v != vp);
            const uint32_t R = start ? runR[s] : 0u;
            const uint32_t nb = start ? run_nbits(v, R) : 0u;
            const uint32_t incl = wave_incl_scan_dpp(nb);
            if (start) run_bits(v, R, base + incl - nb, true);
            base += readlane(incl, 63);
        }
        return base - pos;
    }

    // scan_tree + send_tree in one go (the split back: the bl tree came from the trees kernel, so
    // no counts): the run starts of all chunks first (one ballot each, kept in SGPRs), then each
    // chunk's runs end at the next start, in the chunk or the first one after it -- no run-length
    // array, no back-to-front pass, no second read of the neighbours.  NC = chunks at most.
    template <int NC>
    __device__ uint64_t send_runs_fused(PMC_LDS const uint32_t *code, int max_code, uint64_t pos) {
        const int l = lane_id();
        const int nch = max_code / 64 + 1;
        uint64_t sm[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) {
            sm[c] = 0;
            if (c < nch) {
                const int s = 64 * c + l;
                const bool in = s <= max_code;
                const uint32_t v = in ? code[s] >> 16 : 0xffffu;
                const uint32_t vp = (in && s > 0) ? code[s - 1] >> 16 : 0xfffeu;
                sm[c] = ballot(in && (s == 0 || v != vp));
            }
        }
        uint32_t after[NC]; // first run start past chunk c (max_code + 1 if none)
        uint32_t nxt = (uint32_t)max_code + 1;
#pragma unroll
        for (int c = NC - 1; c >= 0; c--) {
            after[c] = nxt;
            if (c < nch && sm[c]) nxt = 64u * c + (uint32_t)__builtin_ctzll(sm[c]);
        }
        uint64_t base = pos;
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (c < nch) {
                const int s = 64 * c + l;
                const bool start = (sm[c] >> l) & 1;
                const uint64_t above = l == 63 ? 0 : (sm[c] & (~0ull << (l + 1)));
                const uint32_t e = above ? 64u * c + (uint32_t)__builtin_ctzll(above) : after[c];
                const uint32_t v = start ? code[s] >> 16 : 0u, R = e - (uint32_t)s;
                const uint32_t nb = start ? run_nbits(v, R) : 0u;
                const uint32_t incl = wave_incl_scan_dpp(nb);
                if (start) run_bits(v, R, base + incl - nb, true);
                base += readlane(incl, 63);
            }
        }
        return base - pos;
    }

    // compress_block: every token's bits at its prefix-sum offset
    template <bool G = false> // G: a literal's byte from gsrc (HBM) instead of the staged b
    __device__ uint64_t emit_symbols(uint32_t ntok, uint64_t bitpos) {
        const int l = lane_id();
        const Tables &TT = c_tables;
        for (uint32_t t0 = 0; t0 < ntok; t0 += 64) {
            const uint32_t t = t0 + (uint32_t)l;
            uint32_t nb = 0;
            uint64_t v = 0;
            if (t < ntok) {
                const uint32_t tk = tok[t], dist = tk >> 16;
                const uint32_t lc = dist ? tk & 0xff : G ? (uint32_t)gsrc[tk & 0xffff] : (uint32_t)b[tk & 0xffff];
                if (dist == 0) {
                    const uint32_t c = lcode[lc];
                    v = c & 0xffff;
                    nb = c >> 16;
                } else {
                    const uint32_t code = len_code_cf(lc);
                    uint32_t c = lcode[code + kLiterals + 1];
                    v = c & 0xffff;
                    nb = c >> 16;
                    const uint32_t xl = len_extra_cf(code);
                    v |= (uint64_t)((lc - len_base_cf(code)) & ((1u << xl) - 1)) << nb;
                    nb += xl;
                    const uint32_t dm = dist - 1, dc = dist_code_cf(dm);
                    c = dcode[dc];
                    v |= (uint64_t)(c & 0xffff) << nb;
                    nb += c >> 16;
                    const uint32_t xd = dist_extra_cf(dc);
                    v |= (uint64_t)((dm - dist_base_cf(dc)) & ((1u << xd) - 1)) << nb;
                    nb += xd;
                }
            }
            const uint32_t incl = wave_incl_scan_dpp(nb);
            if (nb) or_bits_lds(bitpos + incl - nb, v, (int)nb);
            bitpos += readlane(incl, 63);
        }
        return bitpos;
    }

    // ---- block flush: trees, block type, emission (single final block) --------------------
    __device__ __noinline__ uint64_t flush(uint32_t ntok, uint32_t len, uint64_t bitpos) {
        const int l = lane_id();
        const Tables &TT = c_tables;
        // histograms from the symbol slab
        for (int s = l; s < 352; s += 64) lfreq[s] = 0; // lfreq, dfreq, blfreq contiguous
        wave_sync();
        for (uint32_t t = l; t < ntok; t += 64) {
            const uint32_t tk = tok[t], dist = tk >> 16, lc = dist ? tk & 0xff : b[tk & 0xffff];
            if (dist == 0) {
                lds_add(&lfreq[lc], 1u);
            } else {
                lds_add(&lfreq[len_code_cf(lc) + kLiterals + 1], 1u);
                lds_add(&dfreq[dist_code_cf(dist - 1)], 1u);
            }
        }
        if (l == 0) lfreq[kEndBlock] = 1;
        wave_sync();
        stamp(6);
        PMC_STOP(5, bitpos)
        TreeOut tl = build_tree(lfreq, kLCodes, TT.static_ltree, TT.extra_lbits, kLiterals + 1, kMaxBits, lcode);
        TreeOut td = build_tree(dfreq, kDCodes, TT.static_dtree, TT.extra_dbits, 0, kMaxBits, dcode);
        stamp(3);
        PMC_STOP(6, bitpos)
        // (not in dad[]: the bit-length tree's build_tree below reuses dad[])
        PMC_LDS uint16_t *runL = runs, *runD = runs + 288;
        TreeOut tb{};
        int mbi = 0;
        bool fallback = tl.overflow || td.overflow;
        if (!fallback) {
            scan_runs(lcode, tl.max_code, runL);
            scan_runs(dcode, td.max_code, runD);
            wave_sync();
            tb = build_tree(blfreq, kBLCodes, nullptr, TT.extra_blbits, 0, kMaxBLBits, blcode);
            fallback = tb.overflow;
        }
        int64_t opt_len = 0, static_len = 0;
        int l_max = tl.max_code, d_max = td.max_code;
        if (!fallback) {
            for (mbi = kBLCodes - 1; mbi >= 3; mbi--)
                if ((blcode[TT.bl_order[mbi]] >> 16) != 0) break;
            opt_len = tl.opt + td.opt + tb.opt + 3 * ((int64_t)mbi + 1) + 5 + 5 + 4;
            static_len = tl.stat + td.stat;
        } else {
            // serial zlib restatement on HBM scratch (length-limit overflow: rare).  It starts
            // from the real frequencies: undo the dummy leaves build_tree added above.
            for (int s = l; s < kLCodes; s += 64) {
                const bool dm = s == tl.dummy[0] || s == tl.dummy[1];
                fb->ltree[s] = CtData{(uint16_t)(dm ? 0u : lfreq[s]), 0};
            }
            if (l < kDCodes) {
                const bool dm = l == td.dummy[0] || l == td.dummy[1];
                fb->dtree[l] = CtData{(uint16_t)(dm ? 0u : dfreq[l]), 0};
            }
            if (l < kBLCodes) fb->bltree[l] = CtData{0, 0};
            wave_sync_global();
            uint32_t ol = 0, sl = 0;
            if (l == 0) {
                BlockPlan p = plan_block(*fb, TT);
                ol = p.opt_lenb;
                sl = p.static_lenb;
                l_max = p.l_max;
                d_max = p.d_max;
                mbi = p.max_blindex;
            }
            wave_sync_global();
            ol = rfl(ol);
            sl = rfl(sl);
            l_max = rfl(l_max);
            d_max = rfl(d_max);
            mbi = rfl(mbi);
            for (int s = l; s < 288; s += 64)
                lcode[s] = s <= l_max ? (uint32_t)fb->ltree[s].fc | ((uint32_t)fb->ltree[s].dl << 16) : 0u;
            if (l < 32) dcode[l] = l <= d_max ? (uint32_t)fb->dtree[l].fc | ((uint32_t)fb->dtree[l].dl << 16) : 0u;
            wave_sync();
            // express the plan's byte sizes as bit totals with the same rounding
            opt_len = (int64_t)ol * 8 - 10;
            static_len = (int64_t)sl * 8 - 10;
        }
        stamp(3);
        PMC_STOP(7, bitpos)
        const uint32_t opt_lenb_raw = (uint32_t)(((uint64_t)opt_len + 3 + 7) >> 3);
        const uint32_t static_lenb = (uint32_t)(((uint64_t)static_len + 3 + 7) >> 3);
        const uint32_t opt_lenb = static_lenb <= opt_lenb_raw ? static_lenb : opt_lenb_raw;
        const uint32_t stored_len = len;
        if (stored_len + 4 <= opt_lenb) {
            // stored block (last): header, align, LEN, NLEN, bytes
            if (l == 0) or_bits_lds(bitpos, 1u, 3);
            bitpos = (bitpos + 3 + 7) & ~(uint64_t)7;
            const uint64_t o = bitpos >> 3;
            wave_sync();
            if (l < 4) {
                uint32_t v = l < 2 ? stored_len : ~stored_len;
                outb[o + l] = (uint8_t)(v >> (8 * (l & 1)));
            }
            for (uint32_t k = l; k < stored_len; k += 64) outb[o + 4 + k] = b[k];
            bitpos += (4 + (uint64_t)stored_len) * 8;
            wave_sync();
            return bitpos;
        }
        const bool fixed = static_lenb == opt_lenb;
        if (fixed) {
            for (int s = l; s < 288; s += 64)
                lcode[s] = s < kLCodes ? (uint32_t)TT.static_ltree[s].fc | ((uint32_t)TT.static_ltree[s].dl << 16) : 0u;
            if (l < 32) dcode[l] = l < kDCodes ? (uint32_t)TT.static_dtree[l].fc | ((uint32_t)TT.static_dtree[l].dl << 16) : 0u;
            if (l == 0) or_bits_lds(bitpos, (1u << 1) | 1u, 3);
            bitpos += 3;
            wave_sync();
        } else {
            const int lcodes = l_max + 1, dcodes = d_max + 1, blcodes = mbi + 1;
            if (fallback) {
                uint64_t hb = 0;
                if (l == 0) {
                    LaneBitsL lb{outw, bitpos};
                    lb.put((2u << 1) | 1u, 3);
                    BlockPlan p{0, 0, l_max, d_max, mbi};
                    send_all_trees(*fb, TT, lb, p);
                    hb = lb.pos;
                }
                bitpos = rfl64(hb);
                wave_sync();
            } else {
                if (l == 0) {
                    or_bits_lds(bitpos, (2u << 1) | 1u, 3);
                    or_bits_lds(bitpos + 3, (uint32_t)(lcodes - 257), 5);
                    or_bits_lds(bitpos + 8, (uint32_t)(dcodes - 1), 5);
                    or_bits_lds(bitpos + 13, (uint32_t)(blcodes - 4), 4);
                }
                if (l < blcodes) or_bits_lds(bitpos + 17 + 3 * l, blcode[TT.bl_order[l]] >> 16, 3);
                bitpos += 17 + 3 * (uint64_t)blcodes;
                wave_sync();
                bitpos += send_runs(lcode, lcodes - 1, runL, bitpos);
                bitpos += send_runs(dcode, dcodes - 1, runD, bitpos);
                wave_sync();
            }
        }
        bitpos = emit_symbols(ntok, bitpos);
        const uint32_t eob = lcode[kEndBlock];
        wave_sync();
        if (l == 0) or_bits_lds(bitpos, eob & 0xffff, (int)(eob >> 16));
        bitpos += eob >> 16;
        bitpos = (bitpos + 7) & ~(uint64_t)7;
        wave_sync();
        return bitpos;
    }


    // ---- split pipeline pieces (pmc_deflate_split.hip) ----------------------------------------
    // histogram of the token slab into lfreq / dfreq (END_BLOCK counted once)
    __device__ void histogram(uint32_t ntok, uint32_t len) {
        const int l = lane_id();
        const Tables &TT = c_tables;
        for (int s = l; s < 352; s += 64) lfreq[s] = 0;
        wave_sync();
        for (uint32_t t = l; t < ntok; t += 64) {
            const uint32_t tk = tok[t], dist = tk >> 16, lc = dist ? tk & 0xff : b[tk & 0xffff];
            if (dist == 0) {
                lds_add(&lfreq[lc], 1u);
            } else {
                lds_add(&lfreq[len_code_cf(lc) + kLiterals + 1], 1u);
                lds_add(&dfreq[dist_code_cf(dist - 1)], 1u);
            }
        }
        if (l == 0) lfreq[kEndBlock] = 1;
        wave_sync();
    }
    // gen_codes (trees.c) for code lengths Ls[0..elems): canonical code = next_code[len] +
    // rank among equal lengths; code_out[s] = bit-reversed code | len << 16 (0: unused)
    __device__ __noinline__ void codes_from_lengths(PMC_LDS const uint8_t *Ls, int elems, PMC_LDS uint32_t *code_out) {
        const int l = lane_id();
        uint32_t bl_count[16];
#pragma unroll
        for (int L = 0; L < 16; L++) bl_count[L] = 0;
        for (int c0 = 0; c0 < elems; c0 += 64) {
            const int s = c0 + l;
            const uint32_t len = s < elems ? Ls[s] : 0u;
#pragma unroll
            for (int L = 1; L <= 15; L++) bl_count[L] += __builtin_popcountll(ballot(len == (uint32_t)L));
        }
        uint32_t next_code[16];
        uint32_t code = 0;
        next_code[0] = 0;
#pragma unroll
        for (int L = 1; L <= 15; L++) {
            code = (code + (L > 1 ? bl_count[L - 1] : 0u)) << 1;
            next_code[L] = code;
        }
        for (int c0 = 0; c0 < elems; c0 += 64) {
            const int s = c0 + l;
            const uint32_t len = s < elems ? Ls[s] : 0u;
            uint32_t mycode = 0;
#pragma unroll
            for (int L = 1; L <= 15; L++) {
                const uint64_t mk = ballot(len == (uint32_t)L);
                if (len == (uint32_t)L) mycode = next_code[L] + popc_lt(mk);
                next_code[L] += __builtin_popcountll(mk);
            }
            if (s < elems) code_out[s] = len ? ((__builtin_bitreverse32(mycode) >> (32 - len)) | (len << 16)) : 0u;
        }
        wave_sync();
    }
    // canonical codes (gen_codes) with same-length groups from 4 ballots per chunk: per length
    // counts, then each symbol's rank in its group plus the length's running next code, both
    // kept in tmp (32 words: counts, next codes)
    __device__ __noinline__ void codes_from_lengths4(PMC_LDS const uint8_t *Ls, int elems, PMC_LDS uint32_t *code_out,
                                                     PMC_LDS uint32_t *tmp) {
        const uint32_t l = (uint32_t)lane_id();
        if (l < 32) tmp[l] = 0;
        wave_sync();
        auto group = [&](uint32_t len, bool in) {
            uint64_t m = ballot(in);
#pragma unroll
            for (int bt = 0; bt < 4; bt++) {
                const uint64_t B = ballot((len >> bt) & 1);
                m &= ((len >> bt) & 1) ? B : ~B;
            }
            return m;
        };
        // pass 1: per-length counts; a group's first lane adds its group's size and gets back the
        // count of the same length in earlier chunks (LDS atomics of one wave apply in order),
        // which the group shares by ds_bpermute.  code_out[s] keeps that count + s's rank in the
        // group until the next codes are known.
        for (int c0 = 0; c0 < elems; c0 += 64) {
            const int s = c0 + (int)l;
            const bool in = s < elems;
            const uint32_t len = in ? Ls[s] : 0u;
            const uint64_t m = group(len, in);
            const uint32_t rank = popc_lt(m);
            uint32_t prior = 0;
            if (in && len && rank == 0) prior = lds_add(&tmp[len], (uint32_t)__builtin_popcountll(m));
            const uint32_t lead = m ? (uint32_t)__builtin_ctzll(m) : l;
            prior = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lead << 2), (int)prior);
            if (in) code_out[s] = prior + rank;
        }
        wave_sync();
        {
            // next_code[L] = (next_code[L-1] + count[L-1]) << 1 unrolled: the sum over k < L of
            // count[k] << (L - k) = (sum over k < L of count[k] << (16 - k)) >> (16 - L), exact
            // since every term is a multiple of 2^(16 - L) -- one in-row DPP scan of lanes 1..15
            // instead of fifteen dependent LDS round trips on one lane (count < 2^9: no overflow)
            const uint32_t L = l & 15u, y = L ? tmp[L] << (16 - L) : 0u;
            uint32_t v = y;
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
            const uint32_t nc = (v - y) >> (16 - L);
            wave_sync();
            if (l >= 1 && l < 16) tmp[16 + l] = nc;
        }
        wave_sync();
        // pass 2: code = next_code[len] + earlier same-length symbols (chunks independent)
        for (int c0 = 0; c0 < elems; c0 += 64) {
            const int s = c0 + (int)l;
            if (s < elems) {
                const uint32_t len = Ls[s], mycode = tmp[16 + len] + code_out[s];
                code_out[s] = len ? ((__builtin_bitreverse32(mycode) >> (32 - len)) | (len << 16)) : 0u;
            }
        }
        wave_sync();
    }
    // codes_from_lengths4 for the three trees at once (the split back's code-length row is
    // contiguous: lit/len 286 | dist 30 | bl 19; the code slots lcode 288 | dcode 32 | blcode 32 are
    // too): a group is (tree, length); counts at tmp[tree * 16 + L], next codes at
    // tmp[48 + tree * 16 + L] from one in-row DPP scan whose rows are the trees (96 words of tmp).
    // One call and one set of passes instead of three.  (round 3: ranks from returning atomics
    // instead of 6 ballots + a ds_bpermute per chunk)
    //
    // Guard (returns 1, uniform, on failure): the ranks rest on the lane order of returning LDS
    // atomics, measured on gfx950 but not documented.  Every symbol also lands at its canonical
    // position -- (tree, shorter codes first, then rank) -- in perm[]; with the assumed order,
    // the symbol one position before it, when it has the same length, is a smaller symbol.  A
    // failure sends the value to the retry kernel instead of emitting codes assigned to the wrong
    // symbols (a member that would only fail its CRC on GET).
    // (PMC_FAULT_LANE_ORDER, a diagnostic build: lanes take the symbols of a chunk in reverse, the
    // order the guard must catch)
    __device__ __noinline__ uint32_t codes_from_lengths_all(PMC_LDS const uint8_t *Ls, PMC_LDS uint32_t *code0,
                                                            PMC_LDS uint32_t *tmp, PMC_LDS uint16_t *perm) {
        constexpr int E = kLCodes + kDCodes + kBLCodes;
        const uint32_t l = (uint32_t)lane_id();
#ifdef PMC_FAULT_LANE_ORDER
        const uint32_t lo = 63u - l;
#else
        const uint32_t lo = l;
#endif
        for (uint32_t k = l; k < 96; k += 64) tmp[k] = 0;
        wave_sync();
        auto tree_of = [](int s) { return s < kLCodes ? 0u : s < kLCodes + kDCodes ? 1u : 2u; };
        for (int c0 = 0; c0 < E; c0 += 64) {
            const int s = c0 + (int)lo;
            const bool in = s < E;
            const uint32_t len = in ? Ls[s] : 0u, t = tree_of(s), key = t << 4 | len;
            // the symbol's rank among the earlier ones of its (tree, length): one returning LDS
            // atomic (the lanes of one instruction get their old counts in lane order, and one
            // wave's atomics apply in order across chunks; scripts/micro/lds_atomic_order.hip),
            // parked in its code slot (slots: s, 288 + s - 286, 320 + s - 316)
            if (in) code0[s + 2 * t] = len ? lds_add(&tmp[key], 1u) : 0u;
        }
        wave_sync();
        {
            const uint32_t L = l & 15u, cnt = (L && l < 48) ? tmp[l] : 0u, y = cnt << (16 - L);
            uint32_t v = y, u = cnt;
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
            u += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x111, 0xf, 0xf, false);
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
            u += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x112, 0xf, 0xf, false);
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
            u += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x114, 0xf, 0xf, false);
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
            u += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x118, 0xf, 0xf, false);
            const uint32_t nc = (v - y) >> (16 - L);
            wave_sync();
            if (l < 48 && L >= 1) {
                tmp[48 + l] = nc;
                tmp[96 + l] = u - cnt; // symbols of this tree with shorter codes
            }
        }
        wave_sync();
        // codes; each symbol's canonical position (its tree's base + the symbols with shorter codes +
        // its rank) gets the symbol in perm
        for (int c0 = 0; c0 < E; c0 += 64) {
            const int s = c0 + (int)lo;
            if (s < E) {
                const uint32_t len = Ls[s], t = tree_of(s), slot = (uint32_t)s + 2 * t, key = t << 4 | len;
                const uint32_t rk = code0[slot], mycode = tmp[48 + key] + rk;
                code0[slot] = len ? ((__builtin_bitreverse32(mycode) >> (32 - len)) | (len << 16)) : 0u;
                if (len)
                    perm[(t == 0 ? 0u : t == 1 ? (uint32_t)kLCodes : (uint32_t)(kLCodes + kDCodes)) + tmp[96 + key] + rk] =
                        (uint16_t)s;
            }
        }
        wave_sync();
        // the guard: a symbol of rank > 0 must follow a smaller symbol of its (tree, length) in perm.  The
        // rank comes back from the code (the canonical code minus the length's first code), so nothing is
        // held in registers across the passes.
        uint32_t bad = 0;
        for (int c0 = 0; c0 < E; c0 += 64) {
            const int s = c0 + (int)lo;
            if (s < E) {
                const uint32_t len = Ls[s], t = tree_of(s), key = t << 4 | len;
                if (len) {
                    const uint32_t code = code0[(uint32_t)s + 2 * t] & 0xffffu;
                    const uint32_t rk = (__builtin_bitreverse32(code) >> (32 - len)) - tmp[48 + key];
                    const uint32_t pj = (t == 0 ? 0u : t == 1 ? (uint32_t)kLCodes : (uint32_t)(kLCodes + kDCodes)) +
                                        tmp[96 + key] + rk;
                    if (rk) bad |= perm[pj - 1] >= (uint32_t)s ? 1u : 0u;
                }
            }
        }
        return ballot(bad != 0u) ? 1u : 0u;
    }
    // the block as planned by deflate_trees_kernel: plan = type | l_max << 2 | d_max << 11 |
    // max_blindex << 16 (type 0 stored, 1 fixed, 2 dynamic); Ls = lit/len, dist, bl lengths
    __device__ uint64_t emit_planned(uint32_t ntok, uint32_t len, uint64_t bitpos, uint32_t plan,
                                     PMC_LDS const uint8_t *Ls) {
        const int l = lane_id();
        const Tables &TT = c_tables;
        const uint32_t type = plan & 3;
        if (type == 0) {
            if (l == 0) or_bits_lds(bitpos, 1u, 3);
            bitpos = (bitpos + 3 + 7) & ~(uint64_t)7;
            const uint64_t o = bitpos >> 3;
            wave_sync();
            if (l < 4) {
                uint32_t v = l < 2 ? len : ~len;
                outb[o + l] = (uint8_t)(v >> (8 * (l & 1)));
            }
            for (uint32_t k = l; k < len; k += 64) outb[o + 4 + k] = gsrc ? gsrc[k] : b[k];
            bitpos += (4 + (uint64_t)len) * 8;
            wave_sync();
            return bitpos;
        }
        if (type == 1) {
            for (int s = l; s < 288; s += 64)
                lcode[s] = s < kLCodes ? (uint32_t)TT.static_ltree[s].fc | ((uint32_t)TT.static_ltree[s].dl << 16) : 0u;
            if (l < 32) dcode[l] = l < kDCodes ? (uint32_t)TT.static_dtree[l].fc | ((uint32_t)TT.static_dtree[l].dl << 16) : 0u;
            if (l == 0) or_bits_lds(bitpos, (1u << 1) | 1u, 3);
            bitpos += 3;
            wave_sync();
        } else {
            const int l_max = (int)((plan >> 2) & 511), d_max = (int)((plan >> 11) & 31), mbi = (int)((plan >> 16) & 31);
            // (lcode | dcode | blcode contiguous; runs is free scratch in the split back)
            if (sflag(codes_from_lengths_all(Ls, lcode, (PMC_LDS uint32_t *)runs, perm))) return kBitsGuard;
            PMC_STOP(23, bitpos)
#if PMC_TREES_HDR
            if (sflag(hdr ? 1u : 0u)) { // the header bits the trees kernel emitted, after the 3-bit block header
                if (l == 0) or_bits_lds(bitpos, (2u << 1) | 1u, 3);
                bitpos += 3;
                const uint32_t hb = rfl(hdr[0]), nw = (hb + 31) / 32, sh = (uint32_t)(bitpos & 31);
                const uint64_t w0 = bitpos >> 5;
                wave_sync();
                for (uint32_t k = (uint32_t)l; k < nw; k += 64) {
                    const uint32_t x = hdr[1 + k];
                    lds_or(&outw[w0 + k], x << sh);
                    if (sh && (x >> (32 - sh))) lds_or(&outw[w0 + k + 1], x >> (32 - sh));
                }
                bitpos += hb;
                wave_sync();
                PMC_STOP(24, bitpos)
                bitpos = sflag(gsrc ? 1u : 0u) ? emit_symbols<true>(ntok, bitpos) : emit_symbols<false>(ntok, bitpos);
                const uint32_t eob = lcode[kEndBlock];
                wave_sync();
                if (l == 0) or_bits_lds(bitpos, eob & 0xffff, (int)(eob >> 16));
                bitpos += eob >> 16;
                bitpos = (bitpos + 7) & ~(uint64_t)7;
                wave_sync();
                return bitpos;
            }
#endif
            const int lcodes = l_max + 1, dcodes = d_max + 1, blcodes = mbi + 1;
            if (l == 0) {
                or_bits_lds(bitpos, (2u << 1) | 1u, 3);
                or_bits_lds(bitpos + 3, (uint32_t)(lcodes - 257), 5);
                or_bits_lds(bitpos + 8, (uint32_t)(dcodes - 1), 5);
                or_bits_lds(bitpos + 13, (uint32_t)(blcodes - 4), 4);
            }
            // (bl_order in closed form: a per-lane index into __constant__ memory is a vector-memory
            // round trip)
            if (l < blcodes) or_bits_lds(bitpos + 17 + 3 * l, blcode[bl_order_cf(l)] >> 16, 3);
            bitpos += 17 + 3 * (uint64_t)blcodes;
            wave_sync();
            bitpos += send_runs_fused<(kLCodes + 63) / 64>(lcode, lcodes - 1, bitpos);
            bitpos += send_runs_fused<1>(dcode, dcodes - 1, bitpos);
            wave_sync();
            PMC_STOP(24, bitpos)
        }
        bitpos = sflag(gsrc ? 1u : 0u) ? emit_symbols<true>(ntok, bitpos) : emit_symbols<false>(ntok, bitpos);
        const uint32_t eob = lcode[kEndBlock];
        wave_sync();
        if (l == 0) or_bits_lds(bitpos, eob & 0xffff, (int)(eob >> 16));
        bitpos += eob >> 16;
        bitpos = (bitpos + 7) & ~(uint64_t)7;
        wave_sync();
        return bitpos;
    }

    // bit sink for the serial fallback's send_all_trees (lane 0)
    struct LaneBitsL {
        PMC_LDS uint32_t *out;
        uint64_t pos;
        __device__ void put(unsigned v, int n) {
            if (n == 0) return;
            uint64_t w = pos >> 5;
            int s = (int)(pos & 31);
            uint64_t x = (uint64_t)(v & ((n >= 32) ? 0xffffffffu : ((1u << n) - 1))) << s;
            out[w] |= (uint32_t)x;
            if ((uint32_t)(x >> 32)) out[w + 1] |= (uint32_t)(x >> 32);
            pos += (uint64_t)n;
        }
    };

    // ---- split pipeline: front half (stage, hash sort, lazy parse, histograms) ------------
    __device__ void stage(const uint8_t *src, uint32_t len) {
        const int l = lane_id();
        const uint32_t padded = (len + 32) & ~3u;
        if ((((uintptr_t)src) & 15) == 0) {
            // 16 bytes per lane per load (one HBM round trip per KiB), then the tail bytes
            PMC_GLB const uint4 *s16 = (PMC_GLB const uint4 *)src;
            const uint32_t full16 = len >> 4;
            const uint32_t nw = padded / 4; // words to write (zero past the value)
            for (uint32_t k = l; 4 * k < nw; k += 64) {
                uint4 x = make_uint4(0, 0, 0, 0);
                if (k < full16) {
                    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                    const v4u y = *(PMC_GLB const v4u *)(s16 + k);
                    x = make_uint4(y.x, y.y, y.z, y.w);
                }
                if (4 * k + 3 < nw) { // (one 16-byte LDS store; the padded tail dword by dword)
                    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                    *(PMC_LDS v4u *)(bw + 4 * k) = v4u{x.x, x.y, x.z, x.w};
                } else {
                    bw[4 * k] = x.x;
                    if (4 * k + 1 < nw) bw[4 * k + 1] = x.y;
                    if (4 * k + 2 < nw) bw[4 * k + 2] = x.z;
                }
            }
            wave_sync();
            for (uint32_t k = full16 * 16 + l; k < len; k += 64) b[k] = src[k];
        } else if ((((uintptr_t)src) & 3) == 0) {
            const uint32_t *s4 = reinterpret_cast<const uint32_t *>(src);
            const uint32_t full = len >> 2;
            for (uint32_t k = l; k < padded / 4; k += 64) bw[k] = k < full ? s4[k] : 0u;
            wave_sync();
            if ((uint32_t)l < (len & 3)) b[full * 4 + l] = src[full * 4 + l];
        } else {
            for (uint32_t k = l; k < padded / 4; k += 64) bw[k] = 0;
            wave_sync();
            for (uint32_t k = l; k < len; k += 64) b[k] = src[k];
        }
        wave_sync();
    }
    // (PMC_STOP 11..14: front-kernel instruction attribution, see scripts/front_cost.sh)
    __device__ uint32_t run_front(const uint8_t *src, uint32_t len) {
        stage(src, len);
        stamp(0);
        PMC_STOP(11, 0)
        const uint32_t npos = len >= 3 ? len - 2 : 0;
        uint32_t ntok;
        if (npos) {
            const uint32_t k0 = sort_positions2(npos, (PMC_LDS uint32_t *)CN);
            stamp(1);
            PMC_STOP(12, 0)
            ntok = cnp == 6   ? parse_ondemand<6>(npos, len, k0)
                   : cnp == 4 ? parse_ondemand<4>(npos, len, k0)
                   : cnp < 0  ? parse_ondemand<-1>(npos, len, k0)
                              : parse_ondemand<0>(npos, len, k0);
            PMC_STOP(14, 0)
            if (sflag(ntok == kNtokRetry ? 1u : 0u)) return kNtokRetry; // (sort guard: no histogram)
        } else {
            lit_run(0, 0, len);
            ntok = len;
        }
        wave_sync_global();
        stamp(2);
        histogram(ntok, len);
        stamp(6);
        return ntok;
    }
    // ---- split pipeline: back half (CRC, codes from the planned lengths, emission) -------
    __device__ int run_back(const uint8_t *src, uint32_t len, uint32_t ntok, uint32_t plan, PMC_LDS const uint8_t *Ls,
                            uint8_t *dst, uint32_t dst_cap, uint32_t *dst_len, uint32_t crc_in, uint32_t nostage) {
        const int l = lane_id();
        uint32_t crc;
        if (sflag(nostage)) { // (PMC_BACK_NOSTAGE: crc_in is the batch CRC pass's)
            gsrc = (PMC_GLB const uint8_t *)src;
            crc = crc_in;
            PMC_STOP(21, 0)
        } else {
            gsrc = nullptr;
            stage(src, len);
            PMC_STOP(21, 0)
            crc = wave_crc32_s8(bw, len, crc_tab); // (crc_tab: the back's slicing-by-8 tables)
        }
        PMC_STOP(22, 0)
        for (uint32_t k = l; k < out_words; k += 64) outw[k] = 0;
        wave_sync();
        if (l < 10) {
            const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 2, 3};
            outb[l] = hdr[l];
        }
        wave_sync();
        stamp(0);
        uint64_t bitpos = emit_planned(ntok, len, 80, plan, Ls);
        if (bitpos == kBitsGuard) return kDeflateRetry; // (the code-rank guard: the HBM kernel redoes it)
        PMC_STOP(23, 0)
        PMC_STOP(24, 0)
        PMC_STOP(25, 0)
        stamp(0); // (the back's times share slot 0: slots 3-5 count the front's eval usage)
        uint32_t nbytes = (uint32_t)(bitpos >> 3); // (< 64 KiB: a small value's member)
        if (l < 8) {
            uint32_t v = l < 4 ? crc : len;
            outb[nbytes + l] = (uint8_t)(v >> (8 * (l & 3)));
        }
        nbytes += 8;
        wave_sync();
        if (nbytes > dst_cap) return PMC_E_CAPACITY_DEV;
        if ((((uintptr_t)dst) & 3) == 0) {
            uint32_t *d4 = reinterpret_cast<uint32_t *>(dst);
            const uint32_t full = nbytes >> 2;
            for (uint32_t k = l; k < full; k += 64) d4[k] = outw[k];
            if ((uint32_t)l < (nbytes & 3)) dst[full * 4 + l] = outb[full * 4 + l];
        } else {
            for (uint32_t k = l; k < nbytes; k += 64) dst[k] = outb[k];
        }
        if (l == 0) *dst_len = (uint32_t)nbytes;
        stamp(0);
        return 0;
    }

    // ---- one value ----------------------------------------------------------------------
    __device__ int run(const uint8_t *src, uint32_t len, uint8_t *dst, uint32_t dst_cap, uint32_t *dst_len) {
        const int l = lane_id();
        const uint32_t padded = (len + 32) & ~3u;
        if ((((uintptr_t)src) & 3) == 0) {
            const uint32_t *s4 = reinterpret_cast<const uint32_t *>(src);
            const uint32_t full = len >> 2;
            for (uint32_t k = l; k < padded / 4; k += 64) bw[k] = k < full ? s4[k] : 0u;
            wave_sync();
            if ((uint32_t)l < (len & 3)) b[full * 4 + l] = src[full * 4 + l];
        } else {
            for (uint32_t k = l; k < padded / 4; k += 64) bw[k] = 0;
            wave_sync();
            for (uint32_t k = l; k < len; k += 64) b[k] = src[k];
        }
        wave_sync();
        const uint32_t crc = wave_crc32(b, len, crc_tab);
        stamp(0);
        PMC_STOP(1, 0)
        const uint32_t npos = len >= 3 ? len - 2 : 0;
        if (npos) {
            sort_positions(npos);
            PMC_STOP(2, 0)
        }
        PMC_STOP(3, 0)
        stamp(1);
        // deflate_slow (single block: len < 16383 symbols).  Tokens: match = (dist << 16) |
        // (len - 3); literal = its position (dist 0), the byte is fetched in flush.
        uint32_t ntok;
        if (npos) {
            ntok = parse_ondemand<false>(npos, len, (uint32_t)R[0]);
            // (sort_positions' per-lane counters are stable by construction, so the guard in
            // build_cn cannot fire here; if it ever did, the HBM kernel redoes the value)
            if (sflag(ntok == kNtokRetry ? 1u : 0u)) return kDeflateRetry;
        } else { // no position with MIN_MATCH lookahead: all literals
            lit_run(0, 0, len);
            ntok = len;
        }
        wave_sync_global();
        stamp(2);
        PMC_STOP(4, 0)
        // flush: the output image aliases the (dead) sort scratch
        for (uint64_t k = l; k < out_words; k += 64) outw[k] = 0;
        wave_sync();
        if (l < 10) {
            const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 2, 3};
            outb[l] = hdr[l];
        }
        wave_sync();
        uint64_t bitpos = flush(ntok, len, 80);
        stamp(4);
        PMC_STOP(5, 0)
        PMC_STOP(6, 0)
        PMC_STOP(7, 0)
        PMC_STOP(8, 0)
        uint64_t nbytes = bitpos >> 3;
        if (l < 8) {
            uint32_t v = l < 4 ? crc : len;
            outb[nbytes + l] = (uint8_t)(v >> (8 * (l & 3)));
        }
        nbytes += 8;
        wave_sync();
        if (nbytes > dst_cap) return PMC_E_CAPACITY_DEV;
        if ((((uintptr_t)dst) & 3) == 0) {
            uint32_t *d4 = reinterpret_cast<uint32_t *>(dst);
            const uint64_t full = nbytes >> 2;
            for (uint64_t k = l; k < full; k += 64) d4[k] = outw[k];
            if ((uint64_t)l < (nbytes & 3)) dst[full * 4 + l] = outb[full * 4 + l];
        } else {
            for (uint64_t k = l; k < nbytes; k += 64) dst[k] = outb[k];
        }
        if (l == 0) *dst_len = (uint32_t)nbytes;
        stamp(5);
        return 0;
    }
};

__device__ inline void small_wave_init(SmallWave &w, uint8_t *base, const SmallLayout &L, const DeflateArgs &a,
                                       uint32_t *crc_tab) {
    w.b = to_lds<uint8_t>(base + L.bytes);
    w.bw = to_lds<uint32_t>(base + L.bytes);
    w.S = to_lds<uint16_t>(base + L.S);
    w.R = to_lds<uint16_t>(base + L.R);
    w.lfreq = to_lds<uint32_t>(base + L.freq);
    w.dfreq = w.lfreq + 288;
    w.blfreq = w.dfreq + 32;
    w.outw = to_lds<uint32_t>(base + L.out);
    w.outb = to_lds<uint8_t>(base + L.out);
    w.out_words = (uint32_t)L.out_words;
    w.lcode = to_lds<uint32_t>(base + L.lcode);
    w.dcode = to_lds<uint32_t>(base + L.dcode);
    w.blcode = to_lds<uint32_t>(base + L.blcode);
    w.dad = to_lds<uint16_t>(base + L.dad);
    w.dep = to_lds<uint8_t>(base + L.dep);
    w.runs = to_lds<uint16_t>(base + L.runs);
    w.T = to_lds<uint16_t>(base + L.T);
    w.H = w.R; // hash keys live in R until the ranks overwrite them
    w.cnt = to_lds<uint16_t>(base + L.cnt);
    w.M = to_lds<uint32_t>(base + L.M);
    w.CN = to_lds<uint8_t>(base + L.M);
    w.cnp = 0;
    w.HC = to_lds<uint64_t>(base + L.M + cn_hc_offset(a.cap_len));
    w.EV = to_lds<uint32_t>(base + L.M + cn_ev_offset(a.cap_len));
    w.crc_tab = to_lds<const uint32_t>((void *)crc_tab);
    for (int k = 0; k < 16; k++) w.st[k] = 0;
    w.stop = a.stop_after;
#ifdef PMC_STAMPS
    w.t_last = __builtin_amdgcn_s_memtime();
#endif
}

__device__ inline void small_wave_stamps_out(const SmallWave &w, const DeflateArgs &a) {
#ifdef PMC_STAMPS
    if (lane_id() == 0 && a.dbg)
        for (int k = 0; k < 16; k++) atomicAdd((unsigned long long *)&a.dbg[k], (unsigned long long)w.st[k]);
#endif
}

__global__ void __launch_bounds__(256, 4) deflate_small_kernel(DeflateArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint32_t *crc_tab = reinterpret_cast<uint32_t *>(lds);
    for (int k = threadIdx.x; k < 256; k += blockDim.x) crc_tab[k] = c_crc_table[k];
    __syncthreads();
    const int wpb = blockDim.x / 64, wib = threadIdx.x / 64, l = lane_id();
    const uint64_t wave = (uint64_t)blockIdx.x * wpb + wib;
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
    uint8_t *base = lds + 1024 + (uint64_t)wib * a.wave_bytes;
    const SmallLayout L = small_layout(a.cap_len);
    SmallWave w;
    w.b = to_lds<uint8_t>(base + L.bytes);
    w.bw = to_lds<uint32_t>(base + L.bytes);
    w.S = to_lds<uint16_t>(base + L.S);
    w.R = to_lds<uint16_t>(base + L.R);
    w.lfreq = to_lds<uint32_t>(base + L.freq);
    w.dfreq = w.lfreq + 288;
    w.blfreq = w.dfreq + 32;
    w.outw = to_lds<uint32_t>(base + L.out);
    w.outb = to_lds<uint8_t>(base + L.out);
    w.out_words = (uint32_t)L.out_words;
    w.lcode = to_lds<uint32_t>(base + L.lcode);
    w.dcode = to_lds<uint32_t>(base + L.dcode);
    w.blcode = to_lds<uint32_t>(base + L.blcode);
    w.dad = to_lds<uint16_t>(base + L.dad);
    w.dep = to_lds<uint8_t>(base + L.dep);
    w.runs = to_lds<uint16_t>(base + L.runs);
    w.T = to_lds<uint16_t>(base + L.T);
    w.H = w.R; // hash keys live in R until the ranks overwrite them
    w.cnt = to_lds<uint16_t>(base + L.cnt);
    w.M = to_lds<uint32_t>(base + L.M);
    w.CN = to_lds<uint8_t>(base + L.M);
    w.cnp = 0;
    w.HC = to_lds<uint64_t>(base + L.M + cn_hc_offset(a.cap_len));
    w.EV = to_lds<uint32_t>(base + L.M + cn_ev_offset(a.cap_len));
    w.ML = to_lds<uint64_t>(base + L.masks);
    w.MP = to_lds<uint64_t>(base + L.masks_p);
    w.tok = (PMC_GLB uint32_t *)(a.tokens + wave * kSlabSyms);
    w.fb = reinterpret_cast<Trees *>(a.scratch + wave * sizeof(Trees));
    w.crc_tab = to_lds<const uint32_t>(crc_tab);
    for (int k = 0; k < 16; k++) w.st[k] = 0;
    w.stop = a.stop_after;
#ifdef PMC_STAMPS
    w.t_last = __builtin_amdgcn_s_memtime();
#endif
    // groups of G consecutive values per wave (G = 64 once the batch fills every wave 64 times; a batch
    // of few values, the latency path's, gets one value per wave instead of all on wave 0 -- 16 x 4 KiB
    // measured 8.7 ms serialised against 0.54 ms for one)
    const uint64_t G = min((uint64_t)64, (a.n + nwaves - 1) / nwaves);
    for (uint64_t g = wave * G; g < a.n; g += nwaves * G) {
        const uint64_t vl = g + (uint64_t)l;
        const bool in = (uint64_t)l < G && vl < a.n;
        const uint32_t myl = in ? a.src_len[vl] : 0u;
        uint64_t todo = ballot(in && myl <= a.lds_max_len);
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint64_t v = g + (uint64_t)j;
            const uint32_t len = readlane(myl, j);
            if (len == 0) {
                if (l == 0) {
                    a.rc[v] = PMC_INVALID_INPUT_DEV;
                    a.dst_len[v] = 0;
                }
                continue;
            }
#ifdef PMC_FAULT_LANE_ORDER // (diagnostic build: this kernel's sort and code ranks need no lane order, so it
                            // declines every odd value itself, as a guard would: the retry routes get exercised)
            int rc = (v & 1) ? kDeflateRetry
                             : w.run(a.src + a.src_off[v], len, a.dst + a.dst_off[v], a.dst_cap[v], a.dst_len + v);
#else
            int rc = w.run(a.src + a.src_off[v], len, a.dst + a.dst_off[v], a.dst_cap[v], a.dst_len + v);
#endif
            if (l == 0) {
                a.rc[v] = rc;
                if (rc) a.dst_len[v] = 0;
                if (rc == kDeflateRetry) {
                    atomicAdd(a.guard, 1u);
                    retry_push(a, v);
                }
            }
        }
    }
#ifdef PMC_STAMPS
    if (l == 0 && a.dbg)
        for (int k = 0; k < 16; k++) atomicAdd((unsigned long long *)&a.dbg[k], (unsigned long long)w.st[k]);
#endif
}

} // namespace pmc
