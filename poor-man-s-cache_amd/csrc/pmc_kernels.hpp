// pmc_kernels.hpp -- launch-argument structs and sizing shared by the kernels and the
// host side of the C-ABI (pmc_capi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pmc {

constexpr int PMC_INVALID_INPUT_DEV = -999;
constexpr int PMC_Z_DATA_ERROR_DEV = -3;
constexpr int PMC_Z_BUF_ERROR_DEV = -5;
constexpr int PMC_E_CAPACITY_DEV = -101;
constexpr int PMC_E_ARG_DEV = -102;

constexpr uint32_t kSlabSyms = 16384; // per-wave symbol slab (>= 16383 symbols per block)

// Worst case gzip member size (same formula as oracle_gzip_bound): stored fallback adds
// 5 B per 16383-symbol block; after a window slide fixed/dynamic blocks stay <= 9/8 len.
__host__ __device__ inline uint64_t gzip_bound(uint64_t len) {
    return len + (len >> 3) + 6 * (len / 16383 + 1) + 32;
}

struct DeflateArgs {
    const uint8_t *src;
    const uint64_t *src_off;
    const uint32_t *src_len;
    uint8_t *dst;
    const uint64_t *dst_off;
    const uint32_t *dst_cap;
    uint32_t *dst_len;
    int32_t *rc;
    uint64_t n;
    uint64_t cap_len;     // working-set capacity (max value length handled)
    uint64_t lds_max_len; // values <= this go to the LDS kernel, larger to the HBM kernel
    uint64_t wave_bytes;  // per-wave working set bytes
    uint32_t *tokens;     // per-wave symbol slabs (kSlabSyms each)
    uint8_t *scratch;     // per-wave HBM working sets (HBM variant)
    uint64_t *dbg;        // PMC_STAMPS builds: per-phase cycle sums (else unused)
    int32_t stop_after;   // PMC_STAMPS builds: end each value after phase k (cost attribution)
    // split small-value pipeline (pmc_deflate_split.hip), one chunk of values at a time:
    // value first + v (v < count) owns slot v of the per-value arrays and column v & 63 of
    // block v >> 6 of the interleaved ones
    uint64_t first, count;
    uint32_t *cT;  // LZ77 tokens, stride cap_len
    uint32_t *cN;  // token count per value
    uint16_t *cH;  // symbol histograms, [value][kSplitRows]
    uint8_t *cL;   // code lengths lit/len | dist | bit-length, [value][kSplitRows]
    uint32_t *cB;  // dynamic-block tree headers from the trees kernel, [value][kHdrWords] (PMC_TREES_HDR)
    uint32_t *cC;  // CRC-32 of each value of the chunk, from crc32_batch_kernel (PMC_BACK_NOSTAGE)
    uint32_t back_nostage; // this pass's back reads cC and the source in HBM instead of staging (PMC_BACK_NOSTAGE)
    uint32_t *cP;  // block plan per value
    uint32_t *cG;  // trees kernel merge lists, interleaved [block][kMergeRows][64]
    uint32_t *cD;  // values deferred to the large-heap trees pass; their number at cD[count]
    uint32_t *cZ;  // used literal/length symbols per value (front -> visit order of the trees)
    uint32_t *cO;  // trees kernel visit order (values grouped by cZ), or null
    uint32_t *cQ;  // work counters of the front [0] and back [1] kernels (zeroed per chunk)
    // split pipeline passes: a pass takes the values with min_len < len <= lds_max_len (the large
    // pass: 16382 < len <= deflate_big_limit()); HBM kernel: retry != 0 also takes every value
    // whose rc is kDeflateRetry (a large-pass value of >= 16383 symbols: several DEFLATE blocks)
    uint64_t min_len;
    int32_t retry;
    uint32_t front_batch; // split front: values per work-counter grab (>= 1)
    // lane-order guard counters (context-lifetime, device): [0] values whose hash sort failed the
    // (hash, position) order check, [1] values whose canonical-code ranks failed theirs.  Such a
    // value is redone by the HBM kernel (retry), which the host launches gated: with `gate` set
    // it returns at once while both counters are 0.
    uint32_t *guard;
    int32_t gate;
    // per-call retry list: [0] count, [1 + k] the batch index of the k-th value a path declined
    // (kDeflateRetry); zeroed at the start of every compress call.  The gated HBM pass visits only
    // these values and returns at once when there are none (a lifetime counter kept the
    // pass scanning every later batch of the context).
    uint32_t *rlist;
};

// A path declines value v (rc = kDeflateRetry): the gated HBM pass of this call redoes it.
__device__ inline void retry_push(const DeflateArgs &a, uint64_t v) {
    if (a.rlist) a.rlist[1 + atomicAdd(a.rlist, 1u)] = (uint32_t)v;
}

// ---- large values (pmc_deflate_large.hip): values above the split pipeline's large pass ---------------
// Each value's positions are sorted stably by hash in HBM (S, and the rank array R), then cut into
// segments of kLvSeg positions that one wave each parses speculatively from a fresh deflate_slow state
// (on through kLvOverlap positions of the next segment); a parse is exact from the first loop-top
// position where its state equals the exact parse of the segment before it (stitching), and one wave
// per value then emits the stitched token stream block by block (deflate_lv_emit_kernel).
constexpr uint32_t kLvSeg = 16384, kLvOverlap = 2048, kLvChunk = 4096;
struct LargeArgs {
    const uint8_t *src;
    const uint64_t *src_off;
    const uint32_t *src_len;
    // round tables (host-planned, device copies)
    const uint32_t *lv_val;   // [nv] batch index of large value ov
    const uint64_t *lv_pbase; // [nv] base of its positions in S / R / HC / tmp
    const uint32_t *lv_seg0;  // [nv + 1] first segment of each value
    const uint32_t *lv_ch0;   // [nv + 1] first sort chunk of each value
    const uint32_t *seg_val;  // [nseg] value ordinal
    const uint64_t *seg_tok0; // [nseg] base of the segment's token buffer in tok
    const uint32_t *ch_val;   // [nch] value ordinal of sort chunk c (chunk c - lv_ch0[ov] of the value)
    uint32_t nv, nseg, nch;
    uint32_t *tmp, *S, *R;    // position-indexed (lv_pbase): sort scratch, sorted positions, ranks
    uint8_t *HC;              // position-indexed: the nearest chain candidate exists (zlib's search runs)
    uint32_t *hist;           // [nch][256] digit counts -> scatter bases
    uint32_t *tok;            // segment token buffers (literal = byte, match = dist << 16 | len - 3)
    uint32_t *map;            // [nseg][2][kLvOverlap]: loop-top states of the start / continuation regions
    uint32_t *seg_tok;        // [nseg][4]: tokens parsed, stitched begin, stitched end, (unused)
    int32_t *fail;            // [nv] no convergence at some boundary: the HBM kernel redoes the value
};
__global__ void lv_select_kernel(const uint32_t *src_len, uint64_t n, uint64_t lo, uint64_t hi, uint32_t *out);
__global__ void lv_sort_hist_kernel(LargeArgs a, int pass);
__global__ void lv_sort_scan_kernel(LargeArgs a);
__global__ void lv_sort_scatter_kernel(LargeArgs a, int pass);
__global__ void lv_rank_kernel(LargeArgs a);
__global__ void lv_parse_kernel(LargeArgs a);
__global__ void lv_stitch_kernel(LargeArgs a);

constexpr int32_t kDeflateRetry = -7778;     // internal rc: the split pipeline declined the value
constexpr uint32_t kNtokMultiBlock = 0xffffffffu; // cN marker: >= 16383 symbols
constexpr uint32_t kNtokRetry = 0xfffffffeu;      // cN marker: the sort's lane-order guard fired (retry)

constexpr uint32_t kBackTabBytes = 8 * 256 * 4; // the back kernel's slicing-by-8 CRC tables (LDS per block)
constexpr uint32_t kSplitRows = 336;  // 286 lit/len + 30 dist + 19 bit-length (+1)
constexpr uint32_t kMergeRows = 572;  // 2 heap entries per merge, <= 285 merges
// a dynamic block's tree header (HLIT..send_tree, at most 14 + 19 * 3 + 316 * 7 = 2283 bits): word 0 the
// bit count, then the bits LSB-first (76 words: 16-byte rows)
constexpr uint32_t kHdrWords = 76;
// PMC_TREES_HDR: for values of more than kHdrMinLen bytes the trees kernel (one lane per value) emits the
// header bits and sets kPlanHdr in the plan; the back copies them.  (Same box, 10M x 1 KiB: trees 20.6 ->
// 27.8 ms, back 36.7 -> 26.3; 1M x 4 KiB: -1.2 ms; at 256 B the trees' cost exceeded the back's saving,
// +6.8 / -5.4 ms, so smaller values keep the back's wave-wide headers.)
#ifndef PMC_TREES_HDR
#define PMC_TREES_HDR 1
#endif
constexpr uint32_t kHdrMinLen = 512, kPlanHdr = 1u << 21;
// PMC_BACK_NOSTAGE: for passes of values of <= kNostageMaxLen bytes the back stages no source bytes: their
// CRC-32 comes from a batch CRC pass before it (the verify kernel's method) and a literal token's byte is
// read from the source in HBM (L2: the back's prefetch has touched its lines).  Same box: 10M x 256 B back
// 23.35 -> 21.5 ms (CRC pass included); at 1 KiB 26.3 -> 27.65 and 4 KiB 11.4 -> 14.15, so larger values
// keep the staged bytes and the back's own CRC.
#ifndef PMC_BACK_NOSTAGE
#define PMC_BACK_NOSTAGE 1
#endif
constexpr uint32_t kNostageMaxLen = 512;
constexpr uint32_t kPlanDeferred = 0xffffffffu;
#ifndef PMC_TREES_CAP
#define PMC_TREES_CAP 84
#endif
constexpr int kTreesCap = PMC_TREES_CAP; // lane heap capacity of the first trees pass
// (chunks of values <= 1 KiB: 79, the smallest heap that holds the staged 320-byte lengths row -- 8 waves per
// CU; 1 KiB JSON slices use 60 lit/len symbols on average, 79 at the 99th percentile)
#ifndef PMC_TREES_CAP1K
#define PMC_TREES_CAP1K 79
#endif
constexpr int kTreesCap1K = PMC_TREES_CAP1K;

// bytes of chunk scratch per value of the split pipeline
__host__ __device__ inline uint64_t split_value_bytes(uint64_t cap) {
    return cap * 4 + 4 + kSplitRows * 2 + kSplitRows + 4 + kMergeRows * 4 + 4 + 8;
}

struct InflateArgs {
    const uint8_t *src;
    const uint64_t *src_off;
    const uint32_t *src_len;
    uint8_t *dst;
    const uint64_t *dst_off;
    const uint32_t *dst_cap;
    uint32_t *dst_len;
    int32_t *rc;
    uint64_t n;
    uint64_t lds_max_out; // values whose output fits the LDS image go to the LDS kernel
    uint64_t lds_max_in;
    uint64_t wave_bytes;
    uint8_t *scratch;
    uint64_t *dbg; // PMC_STAMPS builds: per-phase cycle sums (slots 0..7 deflate-independent)
    uint32_t *crc_expect; // lane kernel -> verify kernel: the member's CRC-32 trailer
    int32_t retry_only;   // wave kernels: only members the lane kernel marked kInflateRetry
    const uint32_t *order; // lane kernel: member visit order (by compressed length), or null
    uint32_t *rec_scratch; // record kernel: per-lane record rows (gridDim * 64 rows of rec_stride words)
    uint32_t rec_stride;   // records per row (<= kRecMax)
    int32_t big_only;      // lane kernel: only members the record kernel marked kInflateBig
    int32_t stop_after;    // PMC_STAMPS / PMC_PHASE_STOP builds: record kernel ends after phase k
    uint32_t *rec_work;    // record kernel: work counter (64-member batches handed out), zeroed per launch
    uint32_t rec_max_out;  // record kernel: members of more output go to the lane kernel (<= kRecOutMax)
    int32_t multi_pass;    // lane kernel: the multi-block pass runs (mark such members kInflateMulti)
    uint32_t *retried;     // wave kernels in retry_only mode: members they decode are counted here (or null)
    uint32_t rec_group;    // record kernel: members per grab (a power of two <= 64; 0 = 64)
    uint32_t verify_group; // verify kernel: members per wave (a power of two <= 64; 0 = 64)
    uint32_t *big_list;    // record kernel appends the members it leaves to the lane kernel (kInflateBig) here,
    uint32_t *big_count;   // counted here; the lane passes after it then visit that list only (or null: all n)
};

// lane-inflate visit order: member indices grouped by compressed length, so a wave's 64
// lanes decode members of similar length and finish their decode loops together
constexpr uint32_t kOrderBins = 2048;
__global__ void order_hist_kernel(const uint32_t *src_len, uint64_t n, uint32_t *hist);
__global__ void order_scan_kernel(uint32_t *hist);
__global__ void order_scatter_kernel(const uint32_t *src_len, uint64_t n, uint32_t *cursor, uint32_t *order);

constexpr int32_t kInflateRetry = -7777; // internal rc: lane fast path declined the member
constexpr int32_t kInflateBig = -7779;   // internal rc: output beyond the record kernel's image
constexpr int32_t kInflateWide = -7781;  // internal rc: lit/len code longer than the lane kernel's lists
constexpr int32_t kInflateMulti = -7783; // internal rc: a member of several blocks (the multi-block lane pass)
constexpr uint32_t kRecOutMax = 4096;    // record kernel: output image bytes per member
constexpr uint32_t kRecMax = 2048;       // record kernel: records per member (scratch row)

uint64_t deflate_wave_bytes(bool hbm, uint64_t n);
uint64_t deflate_small_wave_bytes(uint64_t n);
uint64_t inflate_wave_bytes(bool hbm, uint64_t max_out, uint64_t max_in);

template <bool kHbm>
__global__ void deflate_kernel(DeflateArgs a);
__global__ void deflate_lv_emit_kernel(DeflateArgs a, LargeArgs L);
uint64_t deflate_lv_emit_wave_bytes(uint64_t n);
__global__ void deflate_small_kernel(DeflateArgs a);
uint64_t deflate_front_wave_bytes(uint64_t n);
uint64_t deflate_back_wave_bytes(uint64_t n);
template <uint32_t CAPC>
__global__ void deflate_front_kernel(DeflateArgs a);
// the front instance for a pass of cap pcap: 1024 / 4096 (compile-time layout) or 0 (runtime layout)
#ifndef PMC_FRONT_CAPC
#define PMC_FRONT_CAPC 1
#endif
inline uint32_t front_cap_class(uint64_t pcap) {
    if (!PMC_FRONT_CAPC) return 0u;
    return pcap > 512 && pcap <= 1024 ? 1024u : pcap > 3072 && pcap <= 4096 ? 4096u : 0u;
}
template <int CAP>
__global__ void deflate_trees_kernel(DeflateArgs a);
__global__ void deflate_back_kernel(DeflateArgs a);
template <bool kHbm>
__global__ void inflate_kernel(InflateArgs a);
template <int LIT, bool MB>
__global__ void inflate_lane_kernel(InflateArgs a);
template <uint32_t OUT>
__global__ void inflate_rec_kernel(InflateArgs a);
uint32_t rec_lds_bytes(uint32_t out); // dynamic LDS of inflate_rec_kernel<out>
__global__ void inflate_verify_kernel(InflateArgs a);
__global__ void arg_check_kernel(const uint32_t *src_len, uint64_t n, uint64_t max_len, int32_t *rc,
                                 uint32_t *dst_len);
__global__ void lane_order_probe_kernel(uint32_t trials, uint32_t *violations);
__global__ void crc32_batch_kernel(const uint8_t *buf, const uint64_t *off, const uint32_t *len, uint64_t n,
                                   uint32_t *crc);

} // namespace pmc
