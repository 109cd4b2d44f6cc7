// pmc_capi.hip -- host side of the C-ABI declared in include/pmc_codec.h.
//
// Owns per-device state (stream, symbol slabs, HBM working sets, pinned staging) and
// turns a batch into at most two launches per direction: the LDS-resident kernel for
// values whose working set fits a wave's LDS share, and the HBM-resident variant for
// the rest (large values; same device code, working set in a per-wave HBM slab).
#include <hip/hip_runtime.h>

#include <vector>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>

#include <unistd.h>

#include "../../include/pmc_codec.h"
#include "pmc_device.hpp"
#include "pmc_kernels.hpp"

#define PMC_API extern "C" __attribute__((visibility("default")))

namespace pmc {

__constant__ Tables c_tables = make_tables();
__constant__ uint32_t c_crc_table[256];
__constant__ uint32_t c_crc_shift16[kCrcShiftEntries];
__constant__ uint32_t c_crc_shift64k[kCrcShiftEntries];
__constant__ uint32_t c_crc_slice8[8 * 256];
__constant__ uint32_t c_crc_zpiece[4 * 4 * 256];
__constant__ uint32_t c_crc_ones[kCrcQuarterMax + 1];

static thread_local std::string g_err;
static void set_err(const char *what, hipError_t e) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, e == hipSuccess ? "" : hipGetErrorString(e));
    g_err = buf;
}
#define HIP_TRY(x)                    \
    do {                              \
        hipError_t e_ = (x);          \
        if (e_ != hipSuccess) {       \
            set_err(#x, e_);          \
            return PMC_E_NO_DEVICE;   \
        }                             \
    } while (0)

// ---- CRC-32 constants (zlib crc32.c / 1.2.12 crc32_combine_gen) -------------------------
static uint32_t h_multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = b & 1 ? (b >> 1) ^ kCrcPoly : b >> 1;
    }
    return p;
}
static uint32_t h_x2nmodp(uint64_t n, unsigned k) { // x^(n * 2^k) mod P
    uint32_t x2n[64];
    uint32_t p = 1u << 30; // x^1
    x2n[0] = p;
    for (int i = 1; i < 64; i++) x2n[i] = p = h_multmodp(p, p);
    p = 1u << 31; // x^0
    while (n) {
        if (n & 1) p = h_multmodp(x2n[k & 63], p);
        n >>= 1;
        k++;
    }
    return p;
}

static int upload_constants() {
    uint32_t tab[256];
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = c & 1 ? kCrcPoly ^ (c >> 1) : c >> 1;
        tab[n] = c;
    }
    static uint32_t s16[kCrcShiftEntries], s64k[kCrcShiftEntries];
    // x^(8*16*d) = x^(d * 2^7);  x^(8*65536*d) = x^(d * 2^19)
    for (int d = 0; d < kCrcShiftEntries; d++) {
        s16[d] = h_x2nmodp((uint64_t)d, 7);
        s64k[d] = h_x2nmodp((uint64_t)d, 19);
    }
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_table), tab, sizeof tab));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_shift16), s16, sizeof s16));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_shift64k), s64k, sizeof s64k));
    static uint32_t s8[8 * 256], zp[4 * 4 * 256], ones[kCrcQuarterMax + 1];
    for (int b = 0; b < 256; b++) {
        s8[b] = tab[b];
        for (int k = 1; k < 8; k++) s8[k * 256 + b] = (s8[(k - 1) * 256 + b] >> 8) ^ tab[s8[(k - 1) * 256 + b] & 0xff];
    }
    for (int k = 0; k < 4; k++) {
        const uint32_t m = h_x2nmodp(1, 9 + k); // x^(8 * 64 * 2^k)
        for (int j = 0; j < 4; j++)
            for (int b = 0; b < 256; b++) zp[(k * 4 + j) * 256 + b] = h_multmodp(m, (uint32_t)b << (8 * j));
    }
    for (uint32_t len = 0; len <= kCrcQuarterMax; len++) ones[len] = h_multmodp(h_x2nmodp(len, 3), 0xFFFFFFFFu);
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_slice8), s8, sizeof s8));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_zpiece), zp, sizeof zp));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_ones), ones, sizeof ones));
    return PMC_OK;
}

constexpr uint64_t kLdsPerCu = 160 * 1024;
constexpr uint64_t kCrcTabBytes = 1024;

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return PMC_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max(n, (size_t)4096);
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            set_err("hipMalloc", e);
            return PMC_Z_MEM_ERROR;
        }
        cap = want;
        return PMC_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};
struct HostBuf {
    void *p = nullptr;
    size_t cap = 0;
    unsigned flags = hipHostMallocDefault;
    int ensure(size_t n) {
        if (n <= cap) return PMC_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max(n, (size_t)4096);
        hipError_t e = hipHostMalloc(&p, want, flags);
        if (e != hipSuccess) {
            set_err("hipHostMalloc", e);
            return PMC_Z_MEM_ERROR;
        }
        cap = want;
        return PMC_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

} // namespace pmc

using namespace pmc;

struct pmc_ctx {
    int device = 0;
    int cus = 0;
    hipStream_t stream = nullptr;
    DevBuf tokens, dscratch;     // deflate symbol slabs / HBM working sets
    DevBuf fbscratch;            // per-wave Trees for the small kernel's serial fallback
    DevBuf split;                // chunk arrays of the split small-value pipeline
    DevBuf crcx;                 // inflate: CRC-32 trailers from the lane kernel
    DevBuf order;                // inflate: lane visit order (bins | member indices)
    DevBuf recs;                 // inflate: the record kernel's per-lane record rows
    DevBuf bigl;                 // inflate: count + list of the members the record kernel leaves to the lane kernel
    // lane-order guards (DeflateArgs::guard): u32 [0] sort, [1] code ranks, [2] the create-time probe's
    // violations, [3] values sent to the HBM kernel's retry pass by the other paths, [4] members the
    // decompress fast paths handed to the wave kernels; lane_order_ok = the probe passed (else compress takes the kernels that do not need it)
    DevBuf guard;
    DevBuf rlist;                // compress: the per-call retry list (DeflateArgs::rlist)
    bool lane_order_ok = true;
    // host-call routing (pmc_ctx_path_counts): [0] / [1] compress / decompress calls on the latency
    // path, [2] / [3] on the throughput pipeline
    uint64_t path_calls[4] = {0, 0, 0, 0};
    uint64_t latency_redone = 0; // latency-path compress calls whose declined values a pipeline call redid
    // large values (pmc_deflate_large.hip): selection list, round tables, round scratch, emit scratch
    DevBuf lvsel, lvtab, lvbuf, lvemit;
    HostBuf lvpin;
    // per direction (0 compress, 1 decompress): the event recorded after the last batch call and its
    // stream; a call on another stream waits for it, since both use the direction's scratch
    hipEvent_t dir_ev[2] = {};
    hipStream_t dir_st[2] = {};
    bool dir_used[2] = {false, false};
    bool prof = false;           // pmc_ctx_profile: bracket every launch with events
    struct KRec {
        int kind;
        hipEvent_t a, b;
    };
    std::vector<KRec> krecs;
    std::mutex host_mu;          // host-API calls (host_batch, pinned_batch) of this context, one at a time
    // per direction: the scratch buffers above (DevBuf::ensure may free and reallocate them) and
    // dir_ev / dir_st / dir_used are touched by one enqueueing thread at a time, whichever API
    // (device batch, host batch, pinned, store, slab) it came through; a compress and a decompress
    // still enqueue concurrently.  Recursive: the slab and store calls hold it around their own
    // dir_enter / dir_leave and call the batch entry points inside.
    std::recursive_mutex dir_mu[2];
    DevBuf staging;              // device side of host-API calls
    uint64_t *dbg = nullptr;     // diagnostic stamp sums (PMC_STAMPS builds)
    HostBuf pinned;              // host side of host-API calls
    HostBuf zc;                  // latency path: coherent host memory the kernel reads and writes in place
    void *zc_dev = nullptr;      // its device address
    // pmc_gzip_*_batch_pinned: chunk c's H2D (stream h2d), kernels (stream) and D2H (stream d2h)
    // overlap those of chunks c +- 1; slot c & 1 of `pipe` holds chunk c's arrays and bytes.
    struct Pipe {
        hipStream_t h2d = nullptr, d2h = nullptr;
        hipEvent_t in[2] = {}, out[2] = {}, done[2] = {};
        DevBuf slot[2];
        HostBuf total;           // compacted chunks: each slot's chunk total, read by the host
        HostBuf bounce[2];       // slot mode, compacted chunk: outputs on their way to dst_off
        bool busy[2] = {false, false};
    } pipe;
};

namespace {

// Runs `launch` (which enqueues one kernel on st); with profiling on, brackets it with events.
template <class F>
void klaunch(pmc_ctx *ctx, int kind, hipStream_t st, F launch) {
    if (!ctx->prof) {
        launch();
        return;
    }
    pmc_ctx::KRec r{kind, nullptr, nullptr};
    if (hipEventCreate(&r.a) != hipSuccess || hipEventCreate(&r.b) != hipSuccess) {
        launch();
        return;
    }
    (void)hipEventRecord(r.a, st);
    launch();
    (void)hipEventRecord(r.b, st);
    ctx->krecs.push_back(r);
}

// Same-direction batch calls of one context share its scratch: a call issued on a different stream
// than the previous one of its direction first waits (on the device) for that call to finish.
int dir_enter(pmc_ctx *ctx, int dir, hipStream_t st) {
    if (ctx->dir_used[dir] && ctx->dir_st[dir] != st)
        if (hipStreamWaitEvent(st, ctx->dir_ev[dir], 0) != hipSuccess) return PMC_E_NO_DEVICE;
    return PMC_OK;
}
int dir_leave(pmc_ctx *ctx, int dir, hipStream_t st) {
    if (hipEventRecord(ctx->dir_ev[dir], st) != hipSuccess) return PMC_E_NO_DEVICE;
    ctx->dir_st[dir] = st;
    ctx->dir_used[dir] = true;
    return PMC_OK;
}

struct Launch {
    int wpb;        // waves per block
    int blocks;     // grid size
    uint64_t wave_bytes;
    size_t lds;     // dynamic LDS per block
};

int occupancy_blocks(const void *kernel, int threads, size_t lds) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, threads, lds) != hipSuccess || nb < 1) nb = 1;
    return nb;
}

// values with len <= this go through the LDS deflate kernel (one wave needs the whole
// working set: value, sorted keys, ranks, output image, Huffman trees)
uint64_t deflate_lds_limit() {
    uint64_t lo = 64, hi = 65535;
    while (lo < hi) {
        uint64_t mid = (lo + hi + 1) / 2;
        if (deflate_wave_bytes(false, mid) + kCrcTabBytes <= kLdsPerCu) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// values up to this length take the single-block small kernel (pmc_deflate_small.hip)
uint64_t deflate_small_limit() {
    uint64_t lo = 64, hi = 16382;
    while (lo < hi) {
        uint64_t mid = (lo + hi + 1) / 2;
        if (deflate_small_wave_bytes(mid) + kCrcTabBytes <= kLdsPerCu) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// `extra` = dynamic LDS per block besides the waves' working sets (the CRC table; 0 for the front).
// values up to this length take the split pipeline's large pass: the front's working set (no chain
// counts) and the back's must fit a CU's LDS, and every match distance must stay <= MAX_DIST
// (32506; longer values would need zlib's window limit in the candidate walk)
uint64_t deflate_big_limit() {
    uint64_t lo = kSmallMax, hi = 32506;
    while (lo < hi) {
        uint64_t mid = (lo + hi + 1) / 2;
        if (deflate_front_wave_bytes(mid) <= kLdsPerCu && deflate_back_wave_bytes(mid) + kBackTabBytes <= kLdsPerCu)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

Launch plan_lds(pmc_ctx *ctx, const void *kernel, uint64_t wave_bytes, uint64_t n_items,
                uint64_t extra = kCrcTabBytes) {
    Launch L;
    L.wave_bytes = wave_bytes;
    uint64_t fit = (kLdsPerCu - extra) / wave_bytes;
    // waves per block: the most resident waves per CU, then the widest block.  At 4 KiB values the
    // front needs 25 KB per wave: 4-wave blocks (102 KB) fit once per CU (4 waves), 2-wave blocks
    // three times (6 waves).
    L.wpb = (int)std::max<uint64_t>(1, std::min<uint64_t>(4, fit));
    int per_cu = occupancy_blocks(kernel, 64 * L.wpb, extra + L.wpb * wave_bytes);
    for (int w = L.wpb - 1; w >= 1; w--) {
        const int pc = occupancy_blocks(kernel, 64 * w, extra + w * wave_bytes);
        if (w * pc > L.wpb * per_cu) {
            L.wpb = w;
            per_cu = pc;
        }
    }
    L.lds = extra + L.wpb * wave_bytes;
    uint64_t need_blocks = (n_items + L.wpb - 1) / L.wpb;
    L.blocks = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)ctx->cus * per_cu, need_blocks));
    return L;
}

} // namespace

// ================================================================== API
PMC_API const char *pmc_last_error(void) { return g_err.c_str(); }
PMC_API const char *pmc_version(void) { return "pmc_codec 0.1 gfx950 (zlib-1.2.11 level-9 gzip, bit-exact)"; }
PMC_API size_t pmc_gzip_bound(size_t len) { return (size_t)gzip_bound(len); }

PMC_API int pmc_ctx_create(int device, pmc_ctx **out) {
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= device) {
        set_err("hipGetDeviceCount", e);
        return PMC_E_NO_DEVICE;
    }
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        g_err = std::string("device is ") + prop.gcnArchName + ", library built for gfx950";
        return PMC_E_NO_DEVICE;
    }
    int rc = upload_constants();
    if (rc) return rc;
    // the LDS-resident kernels may use the whole 160 KiB of a CU
    HIP_TRY(hipFuncSetAttribute((const void *)deflate_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kLdsPerCu));
    HIP_TRY(hipFuncSetAttribute((const void *)deflate_small_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kLdsPerCu));
    for (const void *fk : {(const void *)deflate_front_kernel<0>, (const void *)deflate_front_kernel<1024>,
                           (const void *)deflate_front_kernel<4096>})
        HIP_TRY(hipFuncSetAttribute(fk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPerCu));
    HIP_TRY(hipFuncSetAttribute((const void *)deflate_back_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kLdsPerCu));
    HIP_TRY(hipFuncSetAttribute((const void *)deflate_trees_kernel<kTreesCap1K>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPerCu));
    HIP_TRY(hipFuncSetAttribute((const void *)deflate_trees_kernel<kTreesCap>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPerCu));
    HIP_TRY(hipFuncSetAttribute((const void *)deflate_trees_kernel<kLCodes>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPerCu));
    HIP_TRY(hipFuncSetAttribute((const void *)inflate_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kLdsPerCu));
    HIP_TRY(hipFuncSetAttribute((const void *)inflate_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kLdsPerCu));
    pmc_ctx *c = new pmc_ctx;
    c->device = device;
    c->cus = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->dir_ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->dir_ev[1], hipEventDisableTiming) != hipSuccess) {
        delete c;
        return PMC_E_NO_DEVICE;
    }
    // guard counters, and the lane-order self-test (lane_order_probe_kernel: 4 waves x 512 trials)
    uint32_t probe = 0;
    if (c->guard.ensure(32) || hipMemsetAsync(c->guard.p, 0, 32, c->stream) != hipSuccess) {
        pmc_ctx_destroy(c);
        return PMC_E_NO_DEVICE;
    }
    hipLaunchKernelGGL(lane_order_probe_kernel, dim3(1), dim3(256), 0, c->stream, 512u, (uint32_t *)c->guard.p + 2);
    if (hipMemcpyAsync(&probe, (uint32_t *)c->guard.p + 2, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        set_err("lane_order_probe_kernel", hipGetLastError());
        pmc_ctx_destroy(c);
        return PMC_E_NO_DEVICE;
    }
    c->lane_order_ok = probe == 0;
    *out = c;
    return PMC_OK;
}

PMC_API int pmc_ctx_guard_counts(pmc_ctx *ctx, uint32_t counts[5]) {
    if (!ctx || !counts) return PMC_E_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(counts, ctx->guard.p, 20, hipMemcpyDeviceToHost));
    return PMC_OK;
}

PMC_API int pmc_ctx_path_counts(pmc_ctx *ctx, uint64_t counts[4]) {
    if (!ctx || !counts) return PMC_E_ARG;
    std::lock_guard<std::mutex> lock(ctx->host_mu);
    for (int k = 0; k < 4; k++) counts[k] = ctx->path_calls[k];
    return PMC_OK;
}

PMC_API int pmc_ctx_latency_redone(pmc_ctx *ctx, uint64_t *n) {
    if (!ctx || !n) return PMC_E_ARG;
    std::lock_guard<std::mutex> lock(ctx->host_mu);
    *n = ctx->latency_redone;
    return PMC_OK;
}

PMC_API void pmc_ctx_destroy(pmc_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    c->tokens.release();
    c->dscratch.release();
    c->fbscratch.release();
    c->split.release();
    c->crcx.release();
    c->recs.release();
    c->bigl.release();
    c->guard.release();
    c->rlist.release();
    c->lvsel.release();
    c->lvtab.release();
    c->lvbuf.release();
    c->lvemit.release();
    c->lvpin.release();
    for (auto &r : c->krecs) {
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    c->krecs.clear();
    c->staging.release();
    c->pinned.release();
    c->zc.release();
    if (c->pipe.h2d) {
        (void)hipStreamSynchronize(c->pipe.d2h);
        for (int k = 0; k < 2; k++) {
            (void)hipEventDestroy(c->pipe.in[k]);
            (void)hipEventDestroy(c->pipe.out[k]);
            (void)hipEventDestroy(c->pipe.done[k]);
            c->pipe.slot[k].release();
        }
        c->pipe.total.release();
        c->pipe.bounce[0].release();
        c->pipe.bounce[1].release();
        (void)hipStreamDestroy(c->pipe.h2d);
        (void)hipStreamDestroy(c->pipe.d2h);
    }
    for (int k = 0; k < 2; k++)
        if (c->dir_ev[k]) (void)hipEventDestroy(c->dir_ev[k]);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

PMC_API pmc_ctx *pmc_default_ctx(void) {
    static std::once_flag once;
    static pmc_ctx *ctx = nullptr;
    std::call_once(once, [] {
        if (pmc_ctx_create(0, &ctx) != PMC_OK) ctx = nullptr;
    });
    return ctx;
}

PMC_API uint32_t pmc_gzip_isize(const void *in, size_t in_len) {
    if (!in || in_len < 18) return 0;
    const uint8_t *p = (const uint8_t *)in + in_len - 4;
    return p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Batches of at most this many values, from the host-memory calls (the drop-in's single values, a
// server's small batches), take the latency path: one wave-per-value kernel that does the whole
// value (deflate_small_kernel; inflate_kernel for decompress) instead of the throughput pipeline's
// chain of launches (front, order sort, trees, back; record / lane kernels, CRC verify), which only
// pays once a batch fills the CUs.
constexpr uint32_t kLatencyBatch = 1024;
constexpr uint64_t kLatencyMaxLen = 4096;
// (PMC_LATENCY_MAX_LEN / PMC_LATENCY_BATCH override them; 0 disables the path)
static uint64_t latency_max_len() {
    static const uint64_t v = getenv("PMC_LATENCY_MAX_LEN") ? (uint64_t)atoll(getenv("PMC_LATENCY_MAX_LEN")) : kLatencyMaxLen;
    return v;
}
static uint64_t latency_batch() {
    static const uint64_t v = getenv("PMC_LATENCY_BATCH") ? (uint64_t)atoll(getenv("PMC_LATENCY_BATCH")) : kLatencyBatch;
    return v;
}
static uint64_t inflate_lds_out_limit();
// the decompress side's length limit: the wave-per-member inflate kernel's LDS image (48 KiB)
static uint64_t latency_max_out() {
    return latency_max_len() ? std::max(latency_max_len(), inflate_lds_out_limit()) : 0;
}
// the decompress side's batch limit: 4x the compress side's, with at most 4x the output in all (4,096 x
// 4 KiB members: 0.81 ms device-resident through the wave kernel against 1.69 ms through the pipeline;
// compress at 4,096 x 4 KiB is faster through the pipeline, 2.86 against 3.33 ms -- round 5, same box)
static bool latency_decompress(uint64_t n, uint64_t max_out, uint64_t out_bytes) {
    const uint64_t lb = 4 * latency_batch(), lm = latency_max_len();
    return n <= lb && max_out <= latency_max_out() && (max_out <= lm || out_bytes <= lb * lm);
}

// ---- large values (pmc_deflate_large.hip) ------------------------------------------------------------
// The batch's values of lo < len <= hi.  Their lengths live on the device: one small readback (a count,
// then the (index, length) list) lets the host plan rounds of values whose sort arrays, token buffers
// and state maps fit a scratch budget.  This is the only synchronous step of a device-resident compress
// call, taken only when max_len says such values may be present.
static int large_values(pmc_ctx *ctx, const DeflateArgs &a, uint64_t lo, uint64_t hi, hipStream_t st) {
    const uint64_t n = a.n;
    int r = ctx->lvsel.ensure(8 + 8 * n);
    if (r) return r;
    uint32_t *sel = (uint32_t *)ctx->lvsel.p;
    HIP_TRY(hipMemsetAsync(sel, 0, 8, st));
    hipLaunchKernelGGL(lv_select_kernel, dim3((unsigned)std::min<uint64_t>((n + 255) / 256, 4096)), dim3(256), 0, st,
                       a.src_len, n, lo, hi, sel);
    uint32_t cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, sel, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (!cnt) return PMC_OK;
    std::vector<uint32_t> list(2 * (size_t)cnt);
    HIP_TRY(hipMemcpy(list.data(), sel + 2, 8 * (size_t)cnt, hipMemcpyDeviceToHost));
    std::vector<std::pair<uint32_t, uint32_t>> vals(cnt);
    for (uint32_t k = 0; k < cnt; k++) vals[k] = {list[2 * k], list[2 * k + 1]};
    std::sort(vals.begin(), vals.end());
    auto nseg_of = [](uint64_t len) { return std::max<uint64_t>(1, len / kLvSeg); };
    auto nch_of = [](uint64_t len) { return (len - 2 + kLvChunk - 1) / kLvChunk; };
    auto tok_of = [&](uint64_t len) { // token capacity of the value's segments
        const uint64_t ns = nseg_of(len);
        return (ns - 1) * (kLvSeg + kLvOverlap + 2) + (len - (ns - 1) * kLvSeg) + 2;
    };
    auto bytes_of = [&](uint64_t len) {
        return 13 * (len - 2) + 4 * tok_of(len) + nseg_of(len) * (2 * kLvOverlap * 4 + 16) + nch_of(len) * 1024 + 64;
    };
    auto al = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
    const uint64_t budget = 24ull << 30;
    size_t v0 = 0;
    while (v0 < vals.size()) {
        // one round: values v0 .. v1 - 1
        size_t v1 = v0;
        uint64_t need = 0, P = 0, nseg = 0, nch = 0, maxlen = 0;
        while (v1 < vals.size() && (v1 == v0 || need + bytes_of(vals[v1].second) <= budget)) {
            const uint64_t len = vals[v1].second;
            need += bytes_of(len);
            P += len - 2;
            nseg += nseg_of(len);
            nch += nch_of(len);
            maxlen = std::max(maxlen, len);
            v1++;
        }
        const uint32_t nv = (uint32_t)(v1 - v0);
        // host tables, in the order of the device table buffer
        const uint64_t o_val = 0, o_pb = al(o_val + 4ull * nv), o_seg0 = al(o_pb + 8ull * nv),
                       o_ch0 = al(o_seg0 + 4ull * (nv + 1)), o_sval = al(o_ch0 + 4ull * (nv + 1)),
                       o_stok = al(o_sval + 4 * nseg), o_cval = al(o_stok + 8 * nseg), tab_bytes = al(o_cval + 4 * nch);
        HIP_TRY(hipStreamSynchronize(st)); // (the previous round's kernels read the pinned tables' device copy)
        r = ctx->lvpin.ensure(tab_bytes);
        if (!r) r = ctx->lvtab.ensure(tab_bytes);
        if (r) return r;
        uint8_t *h = (uint8_t *)ctx->lvpin.p;
        uint32_t *t_val = (uint32_t *)(h + o_val), *t_seg0 = (uint32_t *)(h + o_seg0), *t_ch0 = (uint32_t *)(h + o_ch0),
                 *t_sval = (uint32_t *)(h + o_sval), *t_cval = (uint32_t *)(h + o_cval);
        uint64_t *t_pb = (uint64_t *)(h + o_pb), *t_stok = (uint64_t *)(h + o_stok);
        uint64_t pb = 0, tb = 0;
        uint32_t sg = 0, ch = 0;
        for (uint32_t ov = 0; ov < nv; ov++) {
            const uint64_t len = vals[v0 + ov].second, ns = nseg_of(len), nc = nch_of(len);
            t_val[ov] = vals[v0 + ov].first;
            t_pb[ov] = pb;
            t_seg0[ov] = sg;
            t_ch0[ov] = ch;
            for (uint64_t j = 0; j < ns; j++, sg++) {
                t_sval[sg] = ov;
                t_stok[sg] = tb;
                tb += j + 1 < ns ? kLvSeg + kLvOverlap + 2 : len - j * kLvSeg + 2;
            }
            for (uint64_t c = 0; c < nc; c++, ch++) t_cval[ch] = ov;
            pb += len - 2;
        }
        t_seg0[nv] = sg;
        t_ch0[nv] = ch;
        uint8_t *dt = (uint8_t *)ctx->lvtab.p;
        HIP_TRY(hipMemcpyAsync(dt, h, tab_bytes, hipMemcpyHostToDevice, st));
        // round scratch: tmp | S | R | HC | hist | tok | map | seg_tok | fail
        const uint64_t b_tmp = 0, b_S = al(b_tmp + 4 * P), b_R = al(b_S + 4 * P), b_HC = al(b_R + 4 * P),
                       b_hist = al(b_HC + P), b_tok = al(b_hist + 1024 * nch), b_map = al(b_tok + 4 * tb),
                       b_stok = al(b_map + 2ull * kLvOverlap * 4 * nseg), b_fail = al(b_stok + 16 * nseg),
                       scratch = al(b_fail + 4ull * nv);
        r = ctx->lvbuf.ensure(scratch);
        if (r) return r;
        uint8_t *d = (uint8_t *)ctx->lvbuf.p;
        LargeArgs L{};
        L.src = a.src;
        L.src_off = a.src_off;
        L.src_len = a.src_len;
        L.lv_val = (const uint32_t *)(dt + o_val);
        L.lv_pbase = (const uint64_t *)(dt + o_pb);
        L.lv_seg0 = (const uint32_t *)(dt + o_seg0);
        L.lv_ch0 = (const uint32_t *)(dt + o_ch0);
        L.seg_val = (const uint32_t *)(dt + o_sval);
        L.seg_tok0 = (const uint64_t *)(dt + o_stok);
        L.ch_val = (const uint32_t *)(dt + o_cval);
        L.nv = nv;
        L.nseg = (uint32_t)nseg;
        L.nch = (uint32_t)nch;
        L.tmp = (uint32_t *)(d + b_tmp);
        L.S = (uint32_t *)(d + b_S);
        L.R = (uint32_t *)(d + b_R);
        L.HC = d + b_HC;
        L.hist = (uint32_t *)(d + b_hist);
        L.tok = (uint32_t *)(d + b_tok);
        L.map = (uint32_t *)(d + b_map);
        L.seg_tok = (uint32_t *)(d + b_stok);
        L.fail = (int32_t *)(d + b_fail);
        const unsigned cb = (unsigned)std::min<uint64_t>((nch + 3) / 4, (uint64_t)ctx->cus * 8);
        const unsigned sb = (unsigned)std::min<uint64_t>((nseg + 3) / 4, (uint64_t)ctx->cus * 8);
        const unsigned vb = (unsigned)std::min<uint64_t>(nv, (uint64_t)ctx->cus * 4);
        klaunch(ctx, PMC_K_DEFLATE_LARGE, st, [&] {
            for (int pass = 0; pass < 2; pass++) {
                hipLaunchKernelGGL(lv_sort_hist_kernel, dim3(cb), dim3(256), 0, st, L, pass);
                hipLaunchKernelGGL(lv_sort_scan_kernel, dim3(vb), dim3(256), 0, st, L);
                hipLaunchKernelGGL(lv_sort_scatter_kernel, dim3(cb), dim3(256), 0, st, L, pass);
            }
            hipLaunchKernelGGL(lv_rank_kernel, dim3(cb), dim3(256), 0, st, L);
            hipLaunchKernelGGL(lv_parse_kernel, dim3(sb), dim3(256), 0, st, L);
            hipLaunchKernelGGL(lv_stitch_kernel, dim3(vb), dim3(64), 0, st, L);
        });
        // emit: one wave per value
        DeflateArgs e = a;
        e.cap_len = maxlen;
        e.wave_bytes = deflate_lv_emit_wave_bytes(maxlen);
        const uint64_t ew = std::max<uint64_t>(4, std::min<uint64_t>(
            {(uint64_t)(nv + 3) / 4 * 4, (uint64_t)ctx->cus * 4, std::max<uint64_t>(4, (8ull << 30) / e.wave_bytes / 4 * 4)}));
        r = ctx->lvemit.ensure(ew * e.wave_bytes);
        if (r) return r;
        e.scratch = (uint8_t *)ctx->lvemit.p;
        klaunch(ctx, PMC_K_DEFLATE_LARGE_EMIT, st, [&] {
            hipLaunchKernelGGL(deflate_lv_emit_kernel, dim3((unsigned)(ew / 4)), dim3(256), deflate_lv_emit_lds(4), st, e,
                               L);
        });
        hipError_t err = hipGetLastError();
        if (err != hipSuccess) {
            set_err("large-value kernels", err);
            return PMC_E_NO_DEVICE;
        }
        v0 = v1;
    }
    return PMC_OK;
}

static int compress_batch_body(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                               uint32_t n, uint8_t *dst, const uint64_t *dst_off, const uint32_t *dst_cap,
                               uint32_t *dst_len, int32_t *rc, uint32_t max_len, void *stream,
                               bool latency = false, bool small = false) {
    if (!ctx) return PMC_E_ARG;
    if (n == 0) return PMC_OK;
    if (max_len == 0) max_len = 1;
    hipStream_t st = (hipStream_t)stream;
    // src_len[i] > max_len: no variant below claims the value; it gets PMC_E_ARG on the device (the
    // latency path's caller computed max_len from the lengths itself)
    if (!latency)
        hipLaunchKernelGGL(arg_check_kernel, dim3((unsigned)std::min<uint64_t>(((uint64_t)n + 255) / 256, 2048)),
                           dim3(256), 0, st, src_len, (uint64_t)n, (uint64_t)max_len, rc, dst_len);
    DeflateArgs a{src, src_off, src_len, dst, dst_off, dst_cap, dst_len, rc, n, 0, 0, 0, nullptr, nullptr,
                  ctx->dbg, -1};
    a.guard = (uint32_t *)ctx->guard.p;
#if defined(PMC_STAMPS) || defined(PMC_PHASE_STOP)
    if (const char *e = getenv("PMC_STOP_AFTER")) a.stop_after = atoi(e); // diagnostic builds only
#endif
    // Values <= small_lim (16382): the split pipeline's small pass; 16382 < len <= big_lim (~31.9K,
    // the front's 160 KiB LDS; MAX_DIST caps it at 32506): its large pass; the rest -- and
    // large-pass values of >= 16383 symbols, which need several DEFLATE blocks -- the general
    // kernel with its working set in HBM (pmc_deflate.hip).  PMC_DEFLATE_V1=1 routes everything
    // through the general kernels (A/B and safety net); PMC_DEFLATE_MONO=1 the single-kernel path.
    static const bool force_v1 = getenv("PMC_DEFLATE_V1") && atoi(getenv("PMC_DEFLATE_V1"));
    static const bool mono_env = getenv("PMC_DEFLATE_MONO") && atoi(getenv("PMC_DEFLATE_MONO"));
    // (a context whose lane-order probe failed compresses through the single-kernel path, whose
    // sort and codes use per-lane counters and ballots instead of returning-atomic ranks)
    // (small: a device-resident batch within the latency path's limits -- the one-kernel path, as for
    // host calls, but with the argument check and the retry pass of the device-resident API)
    const bool mono = mono_env || latency || small || !ctx->lane_order_ok;
    const bool split = !force_v1 && !mono;
    const uint64_t small_lim = force_v1 ? 0 : deflate_small_limit();
    const uint64_t big_lim = split ? deflate_big_limit() : small_lim;
    const uint64_t v1_lim = deflate_lds_limit();
    const uint64_t lds_cut = force_v1 ? std::min<uint64_t>(v1_lim, std::max<uint64_t>(max_len, 1))
                                      : std::min<uint64_t>(small_lim, std::max<uint64_t>(max_len, 1));
    uint64_t cap = (lds_cut + 63) & ~(uint64_t)63;
    cap = std::min<uint64_t>(cap, force_v1 ? v1_lim : small_lim);
    // large pass: values in (small_lim, big_hi]
    // The split pipeline's large pass (16382 < len <= ~31.8K through the front at one wave per CU, the
    // front's working set filling the CU's LDS) is off since round 5: the large-value pipeline compresses
    // these values 1.8x faster (100K x 30 KB: 1.55 -> 2.84 GiB/s, 500K x 20 KB 1.58 -> 3.07, same box,
    // profiles/r05/large) -- except in small batches: one wave per value of the large pass finishes a
    // lone 30 KB value in ~5 ms, the large-value pipeline's two 16 KiB segment parses (global-memory
    // chains) in ~10 ms, so batches of up to 2 values per CU that hold no value above the large pass's
    // limit keep it (a batch with longer values runs the large-value pipeline anyway and sends all its
    // values above small_lim there).  PMC_BIG_PASS=1 / 0 forces it on / off.
    static const int big_env = getenv("PMC_BIG_PASS") ? atoi(getenv("PMC_BIG_PASS")) : -1;
    const bool big_pick = big_env >= 0 ? big_env != 0 : n <= 2 * (uint64_t)ctx->cus && max_len <= big_lim;
    const bool big_pass = split && big_pick && max_len > small_lim && big_lim > small_lim;
    const uint64_t big_hi = big_pass ? std::min<uint64_t>(big_lim, max_len) : 0;
    const uint64_t big_cap = big_pass ? std::min<uint64_t>((big_hi + 63) & ~(uint64_t)63, big_lim) : 0;
    const uint64_t hbm_cut = big_pass ? big_hi : lds_cut; // the HBM kernel takes lengths above this
    // values above hbm_cut: the large-value path (pmc_deflate_large.hip), except on the V1 A/B path
    const bool lv = !force_v1 && max_len > hbm_cut;
    uint64_t hbm_waves = 0, hbm_wb = deflate_wave_bytes(true, max_len);
    // The HBM kernel takes values by length only on the V1 path.  Otherwise it runs gated, as the retry
    // pass of the values this call's other paths declined (a lane-order guard fired, a large-pass value
    // of several blocks, a large value whose segments did not stitch): it visits the call's retry list
    // (DeflateArgs::rlist) and returns at once when the list is empty.  The latency path launches no
    // retry pass: host_batch reads the verdicts and redoes a declined call through the pipeline.
    const bool gated = !(force_v1 && max_len > hbm_cut);
    if (!gated || !latency) {
        // as many waves as the kernel's 196 VGPRs let a CU hold (2 per SIMD) within a scratch budget
        // (32 GiB for the V1 path's length-routed values; 8 GiB for retries, whose waves exit at once
        // when there are none): at 2 waves per CU (round 1-2) the latency-bound walk left 64 KiB values
        // at 0.52 GiB/s, and a 64-wave retry pass left periodic 1 MiB values and multi-block 24 KB
        // values 32x short of that
        // A batch of single-block values (max_len <= kSmallMax) can have retries only from a lane-order
        // guard, which never fired on gfx950 (and a context whose create-time probe sees the order broken
        // sends every batch to the per-lane-counter kernels instead): 64 waves, and 64 waves' scratch,
        // cover that.  Only batches with longer values (multi-block large-pass values, large values whose
        // segments did not stitch) size the pass for throughput (the scratch a gated pass
        // allocates stays with the context).
        const uint64_t cap_waves = gated && max_len <= kSmallMax ? 64ull : (uint64_t)ctx->cus * 8;
        hbm_waves = std::max<uint64_t>(1, std::min<uint64_t>(cap_waves,
                                                             ((gated ? 8ull : 32ull) << 30) / std::max<uint64_t>(hbm_wb, 1)));
    }
    hbm_waves = std::min<uint64_t>(hbm_waves, n);
    if (gated && hbm_waves) {
        int r = ctx->rlist.ensure(4ull * ((uint64_t)n + 1));
        if (r) return r;
        HIP_TRY(hipMemsetAsync(ctx->rlist.p, 0, 4, st));
        a.rlist = (uint32_t *)ctx->rlist.p;
    }
    if (split) {
        // chunk scratch budget (PMC_SPLIT_CHUNK_MB): 96 GiB of the 288 GiB holds 14M 1-KiB values, so the
        // 10M north-star batch is one front/trees/back launch set (~7 KB of chunk arrays per 1 KiB value,
        // allocated only as large as the batch needs).  Fewer, larger chunks mean fewer kernel tails:
        // 2 / 6 / 9 / 16 / 48 / 96 GiB measured -50 %, -2 %, -1 %, 0, +0.9 %, +1.2 % round trip (same box)
        static const uint64_t budget = (getenv("PMC_SPLIT_CHUNK_MB") ? (uint64_t)atoll(getenv("PMC_SPLIT_CHUNK_MB"))
                                                                     : 98304ull) << 20;
        auto chunk_of = [&](uint64_t c) {
            uint64_t ch = std::min<uint64_t>(n, std::max<uint64_t>(4096, budget / split_value_bytes(c)));
            return (ch + 63) & ~(uint64_t)63;
        };
        auto scratch_of = [&](uint64_t c, uint64_t ch) {
            const uint64_t blocks = ch / 64;
            return ch * c * 4 + ch * 4 + ch * 4 + blocks * 64 * kSplitRows * 3 + blocks * 64 * kMergeRows * 4 +
                   blocks * 64 * kHdrWords * 4 + ch * 4 +
                   (ch + 1) * 4 + ch * 8 + kOrderBins * 4 + 64 + 1024;
        };
        uint64_t need = scratch_of(cap, chunk_of(cap));
        if (big_pass) need = std::max<uint64_t>(need, scratch_of(big_cap, chunk_of(big_cap)));
        int r = ctx->split.ensure(need);
        if (r) return r;
        if (hbm_waves) {
            r = ctx->tokens.ensure(hbm_waves * kSlabSyms * sizeof(uint32_t));
            if (r) return r;
            r = ctx->dscratch.ensure(hbm_waves * hbm_wb);
            if (r) return r;
        }
        static const bool no_order = getenv("PMC_TREES_ORDER") && !atoi(getenv("PMC_TREES_ORDER"));
        // (the front keeps no CRC table in LDS: its grid is sized for the blocks that really fit)
        const size_t tl_small = (size_t)(kTreesCap + 1) * 64 * 4, tl_1k = (size_t)(kTreesCap1K + 1) * 64 * 4;
        const size_t tl_big = (size_t)(kLCodes + 1) * 64 * 4;
        // one pass over the batch for the values with lo < len <= hi, working sets sized for pcap
        auto run_pass = [&](uint64_t lo, uint64_t hi, uint64_t pcap) -> int {
            const uint32_t fcap = front_cap_class(pcap);
            const uint64_t fwb = deflate_front_wave_bytes(fcap ? fcap : pcap), bwb = deflate_back_wave_bytes(pcap);
            const void *fk = fcap == 1024   ? (const void *)deflate_front_kernel<1024>
                             : fcap == 4096 ? (const void *)deflate_front_kernel<4096>
                                            : (const void *)deflate_front_kernel<0>;
            Launch Lf = plan_lds(ctx, fk, fwb, n, 0);
            const size_t front_lds = Lf.lds;
            Launch Lb = plan_lds(ctx, (const void *)deflate_back_kernel, bwb, n, kBackTabBytes);
            const uint64_t chunk = chunk_of(pcap), blocks = chunk / 64;
            uint8_t *p = (uint8_t *)ctx->split.p;
            a.cT = (uint32_t *)p;
            p += chunk * pcap * 4;
            a.cN = (uint32_t *)p;
            p += chunk * 4;
            a.cP = (uint32_t *)p;
            p += chunk * 4;
            a.cG = (uint32_t *)p;
            p += blocks * 64 * kMergeRows * 4;
            a.cH = (uint16_t *)p;
            p += blocks * 64 * kSplitRows * 2;
            a.cL = (uint8_t *)p;
            p += blocks * 64 * kSplitRows;
            a.cB = (uint32_t *)p;
            p += blocks * 64 * kHdrWords * 4;
            a.cC = (uint32_t *)p;
            p += chunk * 4;
            a.cD = (uint32_t *)p;
            p += (chunk + 1) * 4;
            a.cZ = (uint32_t *)p;
            p += chunk * 4;
            uint32_t *ord = (uint32_t *)p;
            p += chunk * 4;
            uint32_t *obins = (uint32_t *)p;
            p += kOrderBins * 4;
            a.cQ = (uint32_t *)p;
            a.min_len = lo;
            a.lds_max_len = hi;
            a.cap_len = pcap;
            // front work grabs: several values per grab for small values, whose parse is shorter than
            // the counter's serialised grabs (10M x 256 B: 1 per grab 114 ms, 4 or 8: 51 ms; 1 KiB: 2 per
            // grab -0.3 %, 4 the same)
            a.front_batch = pcap <= 512 ? 4u : pcap <= 2048 ? 2u : 1u;
            for (uint64_t first = 0; first < n; first += chunk) {
                a.first = first;
                a.count = std::min<uint64_t>(chunk, n - first);
                const unsigned tb = (unsigned)((a.count + 63) / 64);
                a.wave_bytes = fwb;
                if (hipMemsetAsync(a.cQ, 0, 8, st) != hipSuccess) return PMC_E_NO_DEVICE;
                klaunch(ctx, PMC_K_DEFLATE_FRONT, st, [&] {
                    const dim3 fg((unsigned)std::min<uint64_t>(Lf.blocks, (a.count + Lf.wpb - 1) / Lf.wpb));
                    if (fcap == 1024)
                        hipLaunchKernelGGL(deflate_front_kernel<1024>, fg, dim3(64 * Lf.wpb), front_lds, st, a);
                    else if (fcap == 4096)
                        hipLaunchKernelGGL(deflate_front_kernel<4096>, fg, dim3(64 * Lf.wpb), front_lds, st, a);
                    else
                        hipLaunchKernelGGL(deflate_front_kernel<0>, fg, dim3(64 * Lf.wpb), front_lds, st, a);
                });
                if (hipMemsetAsync(a.cD + a.count, 0, 4, st) != hipSuccess) return PMC_E_NO_DEVICE;
                // trees visit order by used literal/length symbols (PMC_TREES_ORDER=0: index order)
                a.cO = nullptr;
                if (!no_order && a.count >= 4096) {
                    if (hipMemsetAsync(obins, 0, kOrderBins * 4, st) != hipSuccess) return PMC_E_NO_DEVICE;
                    const unsigned ob = (unsigned)std::min<uint64_t>((a.count + 1023) / 1024, (uint64_t)ctx->cus * 4);
                    klaunch(ctx, PMC_K_ORDER, st, [&] {
                        hipLaunchKernelGGL(order_hist_kernel, dim3(ob), dim3(256), 0, st, (const uint32_t *)a.cZ,
                                           a.count, obins);
                        hipLaunchKernelGGL(order_scan_kernel, dim3(1), dim3(1024), 0, st, obins);
                        hipLaunchKernelGGL(order_scatter_kernel, dim3(ob), dim3(256), 0, st, (const uint32_t *)a.cZ,
                                           a.count, obins, ord);
                    });
                    a.cO = ord;
                }
                klaunch(ctx, PMC_K_DEFLATE_TREES, st, [&] {
                    if (pcap <= 1024) hipLaunchKernelGGL(deflate_trees_kernel<kTreesCap1K>, dim3(tb), dim3(64), tl_1k, st, a);
                    else hipLaunchKernelGGL(deflate_trees_kernel<kTreesCap>, dim3(tb), dim3(64), tl_small, st, a);
                    // (the overflow list's walker: its 73.5 KB heap column fits two one-wave blocks per CU)
                    hipLaunchKernelGGL(deflate_trees_kernel<kLCodes>, dim3(std::min<unsigned>(tb, 2u * (unsigned)ctx->cus)),
                                       dim3(64), tl_big, st, a);
                });
                a.wave_bytes = bwb;
                a.back_nostage = PMC_BACK_NOSTAGE && pcap <= kNostageMaxLen ? 1u : 0u;
                // the values' CRC-32 for the back (counted with the back: it is the back's work moved out)
                if (a.back_nostage) klaunch(ctx, PMC_K_DEFLATE_BACK, st, [&] {
                    const unsigned cb = (unsigned)std::min<uint64_t>((a.count + 511) / 512, (uint64_t)ctx->cus * 4);
                    hipLaunchKernelGGL(crc32_batch_kernel, dim3(cb), dim3(512), 0, st, (const uint8_t *)a.src,
                                       (const uint64_t *)(a.src_off + a.first), (const uint32_t *)(a.src_len + a.first),
                                       a.count, a.cC);
                });
                klaunch(ctx, PMC_K_DEFLATE_BACK, st, [&] {
                    hipLaunchKernelGGL(deflate_back_kernel,
                                       dim3((unsigned)std::min<uint64_t>(Lb.blocks, (a.count + Lb.wpb - 1) / Lb.wpb)),
                                       dim3(64 * Lb.wpb), Lb.lds, st, a);
                });
            }
            return PMC_OK;
        };
        r = run_pass(0, lds_cut, cap);
        if (!r && big_pass) r = run_pass(small_lim, big_hi, big_cap);
        if (r) return r;
        a.min_len = 0;
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            set_err("deflate split pipeline", e);
            return PMC_E_NO_DEVICE;
        }
    } else {
        const void *lds_kernel = force_v1 ? (const void *)deflate_kernel<false> : (const void *)deflate_small_kernel;
        const uint64_t lds_wb = force_v1 ? deflate_wave_bytes(false, cap) : deflate_small_wave_bytes(cap);
        Launch Ls = plan_lds(ctx, lds_kernel, lds_wb, n);
        const uint64_t small_waves = (uint64_t)Ls.blocks * Ls.wpb;
        // size every per-wave buffer before the first launch (no reallocation under a kernel)
        int r = ctx->tokens.ensure(std::max(small_waves, hbm_waves) * kSlabSyms * sizeof(uint32_t));
        if (r) return r;
        r = ctx->fbscratch.ensure(small_waves * sizeof(Trees));
        if (r) return r;
        if (hbm_waves) {
            r = ctx->dscratch.ensure(hbm_waves * hbm_wb);
            if (r) return r;
        }
        a.tokens = (uint32_t *)ctx->tokens.p;
        a.lds_max_len = lds_cut;
        a.cap_len = cap;
        a.wave_bytes = lds_wb;
        a.scratch = (uint8_t *)ctx->fbscratch.p;
        klaunch(ctx, PMC_K_DEFLATE_MONO, st, [&] {
            if (force_v1) hipLaunchKernelGGL(deflate_kernel<false>, dim3(Ls.blocks), dim3(64 * Ls.wpb), Ls.lds, st, a);
            else hipLaunchKernelGGL(deflate_small_kernel, dim3(Ls.blocks), dim3(64 * Ls.wpb), Ls.lds, st, a);
        });
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            set_err("deflate_kernel<lds>", e);
            return PMC_E_NO_DEVICE;
        }
    }
    a.tokens = (uint32_t *)ctx->tokens.p;
    // ---- large values (> hbm_cut): segment-parallel parse, stitched, emitted per value ----
    if (lv) {
        const int r = large_values(ctx, a, hbm_cut, max_len, st);
        if (r) return r;
    }
    // ---- HBM kernel (V1: values > lds_cut; else gated retries) ----
    if (hbm_waves) {
        a.cap_len = max_len;
        a.lds_max_len = gated ? max_len : hbm_cut;
        a.retry = 1; // (large-pass values of several blocks, and values a lane-order guard declined)
        a.gate = gated ? 1 : 0;
        a.wave_bytes = hbm_wb;
        a.scratch = (uint8_t *)ctx->dscratch.p;
        klaunch(ctx, PMC_K_DEFLATE_HBM, st, [&] {
            hipLaunchKernelGGL(deflate_kernel<true>, dim3((unsigned)hbm_waves), dim3(64), kCrcTabBytes, st, a);
        });
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            set_err("deflate_kernel<hbm>", e);
            return PMC_E_NO_DEVICE;
        }
    }
    return PMC_OK;
}

static uint64_t inflate_lds_out_limit() { return 48 * 1024; }
// the output image decompress_batch_body's LDS wave kernel gets for a call with this max_len
static uint64_t inflate_lds_limit_out(uint64_t max_len) {
    const uint64_t c = std::min<uint64_t>(inflate_lds_out_limit(), std::max<uint64_t>(max_len, 1));
    return (c + 63) & ~(uint64_t)63;
}

static int decompress_batch_body(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                 const uint32_t *src_len, uint32_t n, uint8_t *dst, const uint64_t *dst_off,
                                 const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc, uint32_t max_len,
                                 void *stream, bool latency = false, bool need_hbm = true) {
    if (!ctx) return PMC_E_ARG;
    if (n == 0) return PMC_OK;
    hipStream_t st = (hipStream_t)stream;
    InflateArgs a{src, src_off, src_len, dst, dst_off, dst_cap, dst_len, rc, n, 0, 0, 0, nullptr, ctx->dbg ? ctx->dbg + 16 : nullptr,
                  nullptr, 0};
    // lane-per-member fast path (pmc_inflate_lane.hip), then the CRC check; whatever it
    // declines (rc = kInflateRetry) goes through the wave-per-member kernels below
    // (PMC_INFLATE_WAVE=1: everything through the wave kernels).
    static const bool wave_only = getenv("PMC_INFLATE_WAVE") && atoi(getenv("PMC_INFLATE_WAVE"));
    // (round 4 measured routing batches of <= 2048 members to the wave kernels instead: 256 x 4 KiB took
    // 12.5 ms there against 3.2 ms for 4096 members through the lane / record paths -- not done)
    if (!wave_only && !latency) {
        int r = ctx->crcx.ensure((uint64_t)n * 4);
        if (r) return r;
        a.crc_expect = (uint32_t *)ctx->crcx.p;
        // visit order by compressed length (PMC_INFLATE_ORDER=0: index order)
        static const bool no_order = getenv("PMC_INFLATE_ORDER") && !atoi(getenv("PMC_INFLATE_ORDER"));
        if (!no_order && n >= 4096) {
            r = ctx->order.ensure((uint64_t)kOrderBins * 4 + (uint64_t)n * 4);
            if (r) return r;
            uint32_t *bins = (uint32_t *)ctx->order.p, *ord = bins + kOrderBins;
            HIP_TRY(hipMemsetAsync(bins, 0, kOrderBins * 4, st));
            const unsigned ob = (unsigned)std::min<uint64_t>(((uint64_t)n + 1023) / 1024, (uint64_t)ctx->cus * 4);
            klaunch(ctx, PMC_K_ORDER, st, [&] {
                hipLaunchKernelGGL(order_hist_kernel, dim3(ob), dim3(256), 0, st, src_len, (uint64_t)n, bins);
                hipLaunchKernelGGL(order_scan_kernel, dim3(1), dim3(1024), 0, st, bins);
                hipLaunchKernelGGL(order_scatter_kernel, dim3(ob), dim3(256), 0, st, src_len, (uint64_t)n, bins, ord);
            });
            a.order = ord;
        }
        // members of <= kRecOutMax output bytes: the two-phase record kernel, one block per
        // resident wave (each block owns 64 record rows); larger ones: the lane kernel
        static const bool no_rec = getenv("PMC_INFLATE_REC") && !atoi(getenv("PMC_INFLATE_REC"));
        const unsigned lb = (unsigned)std::min<uint64_t>(((uint64_t)n + 63) / 64, (uint64_t)ctx->cus * 16);
        if (!no_rec) {
            const uint32_t rstride =
                (uint32_t)std::min<uint64_t>(kRecMax, std::max<uint64_t>(64, ((uint64_t)max_len + 63) & ~(uint64_t)63));
            // the 1 KiB image instance when no member may decode to more (max_len: the largest capacity),
            // else the 4 KiB one (PMC_REC_OUT1K=0: always)
#ifndef PMC_REC_OUT1K
#define PMC_REC_OUT1K 1
#endif
            const bool out1k = PMC_REC_OUT1K && max_len <= 1024;
            const void *rk = out1k ? (const void *)inflate_rec_kernel<1024> : (const void *)inflate_rec_kernel<kRecOutMax>;
            const uint32_t rlds = rec_lds_bytes(out1k ? 1024 : kRecOutMax);
            // exactly the resident blocks: a block owns its rows for the whole grid-stride loop,
            // and blocks beyond residency would start only when the first ones have finished
            static int rec_per_cu_k[2] = {0, 0};
            int &rec_per_cu = rec_per_cu_k[out1k ? 1 : 0];
            if (!rec_per_cu) {
                int nb = 0;
                if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rk, 64, rlds) != hipSuccess || nb < 1)
                    nb = (int)(kLdsPerCu / rlds);
                rec_per_cu = nb;
            }
            // members per grab: the smallest power of two whose grabs fit the resident blocks once, so a small
            // batch (a server's few hundred GETs) spreads one or a few members per wave instead of 64 on a few
            // CUs with phase B's member-serial loop exposed
            const uint64_t slots = (uint64_t)ctx->cus * rec_per_cu;
            uint32_t G = 1;
            while (G < 64 && ((uint64_t)n + G - 1) / G > slots) G *= 2;
            a.rec_group = G;
            const unsigned rb = (unsigned)std::min<uint64_t>(((uint64_t)n + G - 1) / G, slots);
            a.rec_max_out = out1k ? 1024u : kRecOutMax;
            r = ctx->recs.ensure((uint64_t)rb * 64 * rstride * 4 + 256);
            if (r) return r;
            a.rec_work = (uint32_t *)ctx->recs.p;
            a.rec_scratch = (uint32_t *)((uint8_t *)ctx->recs.p + 256);
            HIP_TRY(hipMemsetAsync(a.rec_work, 0, 4, st));
            r = ctx->bigl.ensure((uint64_t)n * 4 + 256);
            if (r) return r;
            a.big_count = (uint32_t *)ctx->bigl.p;
            a.big_list = (uint32_t *)((uint8_t *)ctx->bigl.p + 256);
            HIP_TRY(hipMemsetAsync(a.big_count, 0, 4, st));
            a.rec_stride = rstride;
#if defined(PMC_STAMPS) || defined(PMC_PHASE_STOP)
            if (const char *e = getenv("PMC_STOP_AFTER")) a.stop_after = atoi(e); // 31 prepare, 32 phase A
#endif
            klaunch(ctx, PMC_K_INFLATE_REC, st,
                    [&] {
                        if (out1k) hipLaunchKernelGGL(inflate_rec_kernel<1024>, dim3(rb), dim3(64), rlds, st, a);
                        else hipLaunchKernelGGL(inflate_rec_kernel<kRecOutMax>, dim3(rb), dim3(64), rlds, st, a);
                    });
            a.big_only = 1;
        }
        // members of several blocks exist only above 16383 output bytes (zlib flushes every 16383
        // symbols): then a third pass decodes them block after block
        a.multi_pass = max_len > 16383 ? 1 : 0;
        klaunch(ctx, PMC_K_INFLATE_LANE, st, [&] {
            hipLaunchKernelGGL((inflate_lane_kernel<kLaneLitCap, false>), dim3(lb), dim3(64), kLaneLdsBytes, st, a);
            // members whose lit/len code did not fit its lists (a third of 30 KB JSON values): the wide
            // instance (it skips every other member at once)
            hipLaunchKernelGGL((inflate_lane_kernel<kLaneWideLit, false>), dim3(lb), dim3(64), kLaneWideLdsBytes, st, a);
            if (a.multi_pass)
                hipLaunchKernelGGL((inflate_lane_kernel<kLaneWideLit, true>), dim3(lb), dim3(64), kLaneMultiLdsBytes, st,
                                   a);
        });
        a.big_only = 0;
        a.big_list = nullptr;
        a.big_count = nullptr;
        // (members per wave as for the record kernel: a small batch takes one wave per member)
        uint32_t VG = 1;
        while (VG < 64 && ((uint64_t)n + VG - 1) / VG > (uint64_t)ctx->cus * 32) VG *= 2;
        a.verify_group = VG;
        const unsigned vb = (unsigned)std::min<uint64_t>(((uint64_t)n + 8ull * VG - 1) / (8ull * VG), (uint64_t)ctx->cus * 4);
        klaunch(ctx, PMC_K_INFLATE_VERIFY, st,
                [&] { hipLaunchKernelGGL(inflate_verify_kernel, dim3(vb), dim3(512), 0, st, a); });
        a.retry_only = 1;
        a.retried = (uint32_t *)ctx->guard.p + 4; // (pmc_ctx_guard_counts counts[4])
        a.order = nullptr;
    }
    // output image capacity for the LDS kernel; the compressed input of a member whose
    // output fits is at most gzip_bound(out) unless it is not a deflate member at all
    uint64_t out_cap = std::min<uint64_t>(inflate_lds_out_limit(), std::max<uint64_t>(max_len, 1));
    out_cap = (out_cap + 63) & ~(uint64_t)63;
    a.lds_max_out = out_cap;
    a.lds_max_in = gzip_bound(out_cap) + 64;
    {
        uint64_t wb = inflate_wave_bytes(false, a.lds_max_out, a.lds_max_in);
        Launch L = plan_lds(ctx, (const void *)inflate_kernel<false>, wb, n);
        a.wave_bytes = wb;
        klaunch(ctx, PMC_K_INFLATE_LDS, st,
                [&] { hipLaunchKernelGGL(inflate_kernel<false>, dim3(L.blocks), dim3(64 * L.wpb), L.lds, st, a); });
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            set_err("inflate_kernel<lds>", e);
            return PMC_E_NO_DEVICE;
        }
    }
    // members whose output or input exceeds the LDS image (rare: large values, or garbage
    // input longer than its ISIZE suggests) -> HBM variant; always launched because input
    // lengths are device-resident (the kernel skips members the LDS kernel handled) -- unless a
    // host-memory caller, who knows the lengths, says no member needs it
    if (need_hbm) {
        uint64_t wb = inflate_wave_bytes(true, 0, 0);
        uint64_t waves = std::min<uint64_t>((uint64_t)ctx->cus * 4, n);
        a.wave_bytes = wb;
        klaunch(ctx, PMC_K_INFLATE_HBM, st, [&] {
            hipLaunchKernelGGL(inflate_kernel<true>, dim3((unsigned)((waves + 3) / 4)), dim3(256),
                               kCrcTabBytes + 4 * wb, st, a);
        });
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            set_err("inflate_kernel<hbm>", e);
            return PMC_E_NO_DEVICE;
        }
    }
    return PMC_OK;
}

PMC_API int pmc_gzip_compress_batch(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                    const uint32_t *src_len, uint32_t n, uint8_t *dst, const uint64_t *dst_off,
                                    const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc, uint32_t max_len,
                                    void *stream) {
    if (!ctx) return PMC_E_ARG;
    if (n == 0) return PMC_OK;
    hipStream_t st = (hipStream_t)stream;
    std::lock_guard<std::recursive_mutex> dir_lock(ctx->dir_mu[0]);
    int r = dir_enter(ctx, 0, st);
    if (r) return r;
    // a server-sized batch of small values (<= 1,024 of <= 4 KiB: the host calls' latency-path limits)
    // takes the one-kernel path here too (400 x 4 KiB: 2.15 -> ~1 ms, round 5)
    const bool small = n <= latency_batch() && max_len <= latency_max_len();
    r = compress_batch_body(ctx, src, src_off, src_len, n, dst, dst_off, dst_cap, dst_len, rc, max_len, stream, false,
                            small);
    const int r2 = dir_leave(ctx, 0, st);
    return r ? r : r2;
}

PMC_API int pmc_gzip_decompress_batch(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                      const uint32_t *src_len, uint32_t n, uint8_t *dst, const uint64_t *dst_off,
                                      const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc, uint32_t max_len,
                                      void *stream) {
    if (!ctx) return PMC_E_ARG;
    if (n == 0) return PMC_OK;
    hipStream_t st = (hipStream_t)stream;
    std::lock_guard<std::recursive_mutex> dir_lock(ctx->dir_mu[1]);
    int r = dir_enter(ctx, 1, st);
    if (r) return r;
    // a server-sized GET batch (<= 4,096 members, capacities within the wave kernel's LDS image and
    // <= 16 MiB of output in all, the host calls' limits): the wave-per-member kernel alone (whole-wave
    // Huffman decode per member instead of one lane's; 400 x 4 KiB: 1.47 -> ~0.5 ms, round 5), then the
    // HBM variant for anything it declined (the lengths are device-resident)
    // A batch of at most 4 members per CU also takes the wave kernels whatever its sizes: one wave per
    // member beats one lane per member until the lanes' density pays (1000 x 1 MiB: 220 ms against 453 ms
    // through the multi-block lane pass; 40K x 64 KiB: 542 ms against 25 ms -- round 5, same box).
    // (PMC_LATENCY_BATCH=0 turns both clauses off, so A/B runs and fault tests can still reach the lane /
    // record pipeline with small batches -- ADVICE r5)
    const bool small = latency_decompress(n, max_len, (uint64_t)n * max_len) ||
                       (latency_batch() != 0 && (uint64_t)n <= 4ull * ctx->cus);
    r = decompress_batch_body(ctx, src, src_off, src_len, n, dst, dst_off, dst_cap, dst_len, rc, max_len, stream, small,
                              true);
    const int r2 = dir_leave(ctx, 1, st);
    return r ? r : r2;
}

PMC_API int pmc_ctx_profile(pmc_ctx *ctx, int enable) {
    if (!ctx) return PMC_E_ARG;
    ctx->prof = enable != 0;
    return PMC_OK;
}

PMC_API int pmc_ctx_kernel_times(pmc_ctx *ctx, double *ms, uint32_t *launches, int nkinds) {
    if (!ctx || !ms || !launches || nkinds < 0) return PMC_E_ARG;
    int rc = PMC_OK;
    for (auto &r : ctx->krecs) {
        float t = 0;
        if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&t, r.a, r.b) != hipSuccess) rc = PMC_E_NO_DEVICE;
        if (r.kind < nkinds) {
            ms[r.kind] += t;
            launches[r.kind] += 1;
        }
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    ctx->krecs.clear();
    return rc;
}

PMC_API int pmc_crc32_batch(pmc_ctx *ctx, const uint8_t *buf, const uint64_t *off, const uint32_t *len, uint32_t n,
                            uint32_t *crc, void *stream) {
    if (!ctx || (n && (!buf || !off || !len || !crc))) return PMC_E_ARG;
    if (!n) return PMC_OK;
    const unsigned b = (unsigned)std::min<uint64_t>(((uint64_t)n + 511) / 512, (uint64_t)ctx->cus * 4);
    hipLaunchKernelGGL(crc32_batch_kernel, dim3(b), dim3(512), 0, (hipStream_t)stream, buf, off, len, (uint64_t)n, crc);
    return hipGetLastError() == hipSuccess ? PMC_OK : PMC_E_NO_DEVICE;
}

PMC_API int pmc_gzip_isize_batch(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                 const uint32_t *src_len, uint32_t n, uint32_t *isize, void *stream) {
    if (!ctx) return PMC_E_ARG;
    if (!n) return PMC_OK;
    hipLaunchKernelGGL(isize_kernel, dim3(std::min<uint32_t>((n + 255) / 256, 4096)), dim3(256), 0,
                       (hipStream_t)stream, src, src_off, src_len, n, isize);
    return hipGetLastError() == hipSuccess ? PMC_OK : PMC_E_NO_DEVICE;
}

// ---- host-resident batches: pinned staging, H2D -> kernels -> D2H -------------------
namespace {
enum Dir { kCompress, kDecompress };

// A host-API call holds its context's lock (the staging buffers, pinned pipe and default context
// are shared by every thread that calls the drop-in) and leaves the caller's current device as
// it found it.
struct HostCall {
    std::lock_guard<std::mutex> lock;
    int prev = -1;
    explicit HostCall(pmc_ctx *ctx) : lock(ctx->host_mu) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~HostCall() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Per-value copies between the caller's buffers and the staging area: one job per value, spread over a
// small pool of persistent host threads once a call moves enough bytes that one core's memcpy (~10 GB/s)
// would show beside the kernels (a 4,096 x 4 KiB batch is 16 MiB in and 17 MiB of slots out): one part per
// MiB, at most 8 parts (PMC_HOST_THREADS overrides).  Threads spawned per call cost more than they saved
// at 16 parts (unpack 0.43 -> 0.7 ms), so the pool's workers live for the process and wait on a condition.
class CopyPool {
  public:
    static CopyPool &get() {
        static CopyPool *p = new CopyPool(); // (never destroyed: workers may outlive static destructors)
        return *p;
    }
    unsigned parts() const { return nthreads + 1; }
    // runs part(k) for k = 0 .. t - 1 (t <= parts()), part 0 on the calling thread
    template <class F>
    void run(unsigned t, F part) {
        // Inline on the calling thread when: one part; a process forked after the pool started (the child
        // has no workers); or the pool is busy with another context's copies (a server's SET and
        // GET contexts copy at the same time: the second caller does its own copies instead of waiting).
        std::unique_lock<std::mutex> one(run_mu, std::defer_lock);
        if (t <= 1 || getpid() != owner || !one.try_lock()) {
            for (unsigned k = 0; k < t; k++) part(k);
            return;
        }
        std::unique_lock<std::mutex> lk(mu);
        fn = [&part](unsigned k) { part(k); };
        want = t - 1;
        taken = 0;
        left = t - 1;
        gen++;
        cv.notify_all();
        lk.unlock();
        part(0u);
        lk.lock();
        done.wait(lk, [&] { return left == 0; });
        fn = nullptr;
    }

  private:
    CopyPool() : owner(getpid()) {
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        const unsigned cap = getenv("PMC_HOST_THREADS") ? (unsigned)std::max(1, atoi(getenv("PMC_HOST_THREADS")))
                                                        : std::min(8u, hw);
        nthreads = cap - 1;
        for (unsigned k = 0; k < nthreads; k++) std::thread([this] { loop(); }).detach();
    }
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return gen != seen && taken < want; });
            seen = gen;
            const unsigned k = ++taken; // parts 1 .. want
            auto f = fn;
            lk.unlock();
            f(k);
            lk.lock();
            if (--left == 0) done.notify_one();
        }
    }
    const pid_t owner; // the process whose threads these workers are
    std::mutex mu, run_mu;
    std::condition_variable cv, done;
    std::function<void(unsigned)> fn;
    unsigned nthreads = 0, want = 0, taken = 0, left = 0;
    uint64_t gen = 0;
};

template <class F>
void par_values(uint32_t n, uint64_t bytes, F job) {
    CopyPool &P = CopyPool::get();
    const unsigned t = (unsigned)std::min<uint64_t>({(uint64_t)P.parts(), (uint64_t)n, std::max<uint64_t>(1, bytes >> 20)});
    P.run(t, [&](unsigned k) {
        const uint32_t a = (uint32_t)((uint64_t)n * k / t), b = (uint32_t)((uint64_t)n * (k + 1) / t);
        for (uint32_t i = a; i < b; i++) job(i);
    });
}

double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// (the caller holds ctx->host_mu; force_pipeline: the throughput route whatever the batch's size)
int host_batch_locked(pmc_ctx *ctx, Dir dir, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                      uint32_t n, uint8_t *dst, const uint64_t *dst_off, const uint32_t *dst_cap, uint32_t *dst_len,
                      int32_t *rc, bool force_pipeline) {
    if (n == 0) return PMC_OK;
    static const bool trace = getenv("PMC_HOST_TRACE") && atoi(getenv("PMC_HOST_TRACE"));
    double t[8] = {};
    if (trace) t[0] = now_us();
    HIP_TRY(hipSetDevice(ctx->device));
    // packed device layout, in the order of the two copies: [offsets, lengths, caps | source bytes]
    // go down in one H2D, [output lengths, verdicts | output bytes] come back in one D2H
    uint64_t in_bytes = 0, out_bytes = 0, max_len = 0, max_in = 0;
    for (uint32_t i = 0; i < n; i++) {
        in_bytes += src_len[i];
        out_bytes += dst_cap[i];
        uint64_t m = dir == kCompress ? src_len[i] : dst_cap[i];
        max_len = std::max(max_len, m);
        max_in = std::max<uint64_t>(max_in, src_len[i]);
    }
    auto al = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
    const uint64_t down = al(n * 8ull) * 2 + al(n * 4ull) * 2 + al(in_bytes + 16);
    const uint64_t up = al(n * 4ull) * 2 + al(out_bytes + 16);
    // Routing (limits measured with scripts/few_sweep.py).  Compress: up to 1,024 values of <= 4 KiB the
    // one-kernel path (deflate_small_kernel) beats the pipeline; above 4 KiB the wave-per-value kernel would
    // work from HBM, far slower than the split pipeline's large pass.  Decompress: the wave-per-member
    // inflate kernel holds a member's output in LDS up to inflate_lds_out_limit() (48 KiB), so a member up
    // to that size stays on the latency path (a 30 KB member: 0.81 ms there against 3.8 ms through the
    // pipeline); its batch limit is 4,096 members / 16 MiB of output (latency_decompress:
    // round 5 measured the wave kernel still 2x ahead there).
    const uint64_t lat_max = latency_max_len(), lat_batch = latency_batch();
    const bool latency = !force_pipeline && (dir == kCompress ? n <= lat_batch && max_len <= lat_max
                                                              : latency_decompress(n, max_len, out_bytes));
    ctx->path_calls[(latency ? 0 : 2) + (dir == kCompress ? 0 : 1)]++;
    // The latency path's kernel reads its inputs from, and writes its outputs to, coherent host memory in
    // place: no H2D / D2H copies (each a runtime copy kernel of its own) around its one launch.
    const bool zc = latency;
    uint8_t *hp, *dp;
    int r;
    if (zc) {
        ctx->zc.flags = hipHostMallocCoherent;
        const void *old = ctx->zc.p;
        r = ctx->zc.ensure(down + up);
        if (r) return r;
        if (ctx->zc.p != old) ctx->zc_dev = nullptr; // (a new buffer: its device address is looked up below)
        if (!ctx->zc_dev) {
            void *d = nullptr;
            HIP_TRY(hipHostGetDevicePointer(&d, ctx->zc.p, 0));
            ctx->zc_dev = d;
        }
        hp = (uint8_t *)ctx->zc.p;
        dp = (uint8_t *)ctx->zc_dev;
    } else {
        r = ctx->pinned.ensure(down + up);
        if (r) return r;
        r = ctx->staging.ensure(down + up);
        if (r) return r;
        hp = (uint8_t *)ctx->pinned.p;
        dp = (uint8_t *)ctx->staging.p;
    }
    uint64_t o = 0;
    uint64_t *h_soff = (uint64_t *)(hp + o), *d_soff = (uint64_t *)(dp + o);
    o += al(n * 8ull);
    uint64_t *h_doff = (uint64_t *)(hp + o), *d_doff = (uint64_t *)(dp + o);
    o += al(n * 8ull);
    uint32_t *h_slen = (uint32_t *)(hp + o), *d_slen = (uint32_t *)(dp + o);
    o += al(n * 4ull);
    uint32_t *h_dcap = (uint32_t *)(hp + o), *d_dcap = (uint32_t *)(dp + o);
    o += al(n * 4ull);
    uint8_t *h_src = hp + o, *d_src = dp + o;
    o += al(in_bytes + 16);
    uint32_t *h_dlen = (uint32_t *)(hp + o), *d_dlen = (uint32_t *)(dp + o);
    o += al(n * 4ull);
    int32_t *h_rc = (int32_t *)(hp + o), *d_rc = (int32_t *)(dp + o);
    o += al(n * 4ull);
    uint8_t *h_dst = hp + o, *d_dst = dp + o;
    uint64_t so = 0, doff = 0;
    for (uint32_t i = 0; i < n; i++) {
        h_soff[i] = so;
        h_slen[i] = src_len[i];
        so += src_len[i];
        h_doff[i] = doff;
        h_dcap[i] = dst_cap[i];
        doff += dst_cap[i];
    }
    par_values(n, in_bytes, [&](uint32_t i) { memcpy(h_src + h_soff[i], src + src_off[i], src_len[i]); });
    if (trace) t[1] = now_us();
    hipStream_t st = ctx->stream;
    if (!zc) HIP_TRY(hipMemcpyAsync(dp, hp, down, hipMemcpyHostToDevice, st));
    auto run = [&](bool lat) -> int {
        const int d = dir == kCompress ? 0 : 1;
        std::lock_guard<std::recursive_mutex> dir_lock(ctx->dir_mu[d]);
        int e = dir_enter(ctx, d, st);
        if (!e) {
            if (dir == kCompress)
                e = compress_batch_body(ctx, d_src, d_soff, d_slen, n, d_dst, d_doff, d_dcap, d_dlen, d_rc,
                                        (uint32_t)max_len, st, lat);
            else  // the wave kernels' HBM variant only for members the LDS image cannot hold
                e = decompress_batch_body(ctx, d_src, d_soff, d_slen, n, d_dst, d_doff, d_dcap, d_dlen, d_rc,
                                          (uint32_t)max_len, st, lat,
                                          !lat || max_len > inflate_lds_limit_out(max_len) ||
                                              max_in > gzip_bound(inflate_lds_limit_out(max_len)) + 64);
            const int e2 = dir_leave(ctx, d, st);
            if (!e) e = e2;
        }
        return e;
    };
    r = run(latency);
    if (r) {
        // kernels already queued may still read or write the staging (in zero-copy mode the host
        // buffers themselves), which the next call refills: let them drain before returning
        (void)hipStreamSynchronize(st);
        return r;
    }
    if (trace) t[2] = now_us();
    if (!zc) HIP_TRY(hipMemcpyAsync(h_dlen, d_dlen, up, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    // The latency path launches no retry pass: the values its kernel declined (a lane-order guard fired)
    // are redone, alone, by a pipeline call (its gated HBM pass), straight into the caller's buffers.
    std::vector<uint32_t> redo;
    if (zc && dir == kCompress)
        for (uint32_t i = 0; i < n; i++)
            if (h_rc[i] == kDeflateRetry) redo.push_back(i);
    std::vector<uint8_t> redone(redo.empty() ? 0 : n, 0);
    if (!redo.empty()) {
        ctx->latency_redone++;
        const uint32_t m = (uint32_t)redo.size();
        std::vector<uint64_t> r_soff(m), r_doff(m);
        std::vector<uint32_t> r_slen(m), r_cap(m), r_dlen(m);
        std::vector<int32_t> r_rc(m);
        for (uint32_t k = 0; k < m; k++) {
            const uint32_t i = redo[k];
            r_soff[k] = src_off[i];
            r_slen[k] = src_len[i];
            r_cap[k] = dst_cap[i];
            r_doff[k] = dst_off ? dst_off[i] : h_doff[i];
            redone[i] = 1;
        }
        if ((r = host_batch_locked(ctx, dir, src, r_soff.data(), r_slen.data(), m, dst, r_doff.data(), r_cap.data(),
                                   r_dlen.data(), r_rc.data(), true)))
            return r;
        for (uint32_t k = 0; k < m; k++) {
            h_rc[redo[k]] = r_rc[k];
            h_dlen[redo[k]] = r_dlen[k];
        }
    }
    if (trace) t[3] = now_us();
    uint64_t moved = 0;
    for (uint32_t i = 0; i < n; i++) {
        rc[i] = h_rc[i];
        dst_len[i] = h_dlen[i];
        if (h_rc[i] == 0 && (redone.empty() || !redone[i])) moved += h_dlen[i];
    }
    par_values(n, moved, [&](uint32_t i) {
        if (h_rc[i] != 0 || (!redone.empty() && redone[i])) return; // (redone values are in place already)
        uint64_t to = dst_off ? dst_off[i] : h_doff[i];
        memcpy(dst + to, h_dst + h_doff[i], h_dlen[i]);
    });
    if (trace) {
        t[4] = now_us();
        fprintf(stderr,
                "pmc_host_trace %s n=%u in=%llu out=%llu path=%s stage_us=%.1f enqueue_us=%.1f wait_us=%.1f "
                "unpack_us=%.1f total_us=%.1f\n",
                dir == kCompress ? "compress" : "decompress", n, (unsigned long long)in_bytes,
                (unsigned long long)moved, latency ? "latency" : "pipeline", t[1] - t[0], t[2] - t[1], t[3] - t[2],
                t[4] - t[3], t[4] - t[0]);
    }
    return PMC_OK;
}

int host_batch(pmc_ctx *ctx, Dir dir, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
               uint32_t n, uint8_t *dst, const uint64_t *dst_off, const uint32_t *dst_cap, uint32_t *dst_len,
               int32_t *rc) {
    if (!ctx) return PMC_E_ARG;
    if (n == 0) return PMC_OK;
    HostCall guard(ctx);
    return host_batch_locked(ctx, dir, src, src_off, src_len, n, dst, dst_off, dst_cap, dst_len, rc, false);
}

// Rebases one chunk's offsets onto its device copy: src_off -= sb, dst_off -= db (dst_off may be null).
__global__ void rebase_kernel(uint64_t *soff, uint64_t *doff, uint32_t n, uint64_t sb, uint64_t db) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        soff[i] -= sb;
        if (doff) doff[i] -= db;
    }
}

// Exclusive prefix sum of v[i] (0 where rc[i] != 0, if rc is given) into out[]; kScanBlock values per
// block, block totals to bsum[] (scan_blocks_kernel turns them into block bases, bsum[nb] = total).
constexpr uint32_t kScanBlock = 1024;
__global__ __launch_bounds__(kScanBlock) void scan_local_kernel(const uint32_t *v, const int32_t *rc, uint32_t n,
                                                                 uint64_t *out, uint64_t *bsum) {
    __shared__ uint64_t s[kScanBlock];
    const uint32_t t = threadIdx.x, i = blockIdx.x * kScanBlock + t;
    const uint64_t x = i < n && !(rc && rc[i] != 0) ? v[i] : 0;
    s[t] = x;
    __syncthreads();
    for (uint32_t d = 1; d < kScanBlock; d <<= 1) {
        uint64_t y = t >= d ? s[t - d] : 0;
        __syncthreads();
        s[t] += y;
        __syncthreads();
    }
    if (i < n) out[i] = s[t] - x;
    if (t == kScanBlock - 1) bsum[blockIdx.x] = s[t];
}

__global__ __launch_bounds__(kScanBlock) void scan_blocks_kernel(uint64_t *bsum, uint32_t nb) {
    __shared__ uint64_t s[kScanBlock];
    __shared__ uint64_t carry;
    const uint32_t t = threadIdx.x;
    if (t == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nb; base += kScanBlock) {
        const uint64_t x = base + t < nb ? bsum[base + t] : 0;
        s[t] = x;
        __syncthreads();
        for (uint32_t d = 1; d < kScanBlock; d <<= 1) {
            uint64_t y = t >= d ? s[t - d] : 0;
            __syncthreads();
            s[t] += y;
            __syncthreads();
        }
        if (base + t < nb) bsum[base + t] = carry + s[t] - x;
        __syncthreads();
        if (t == kScanBlock - 1) carry += s[t];
        __syncthreads();
    }
    if (t == 0) bsum[nb] = carry;
}

__global__ __launch_bounds__(kScanBlock) void scan_add_kernel(uint64_t *out, uint32_t n, const uint64_t *bsum) {
    const uint32_t i = blockIdx.x * kScanBlock + threadIdx.x;
    if (i < n) out[i] += bsum[blockIdx.x];
}

// One wave per member: slot bytes dst[doff[i] ..+ len[i]) -> packed[poff[i] ..) (rc[i] != 0: none).
__global__ __launch_bounds__(256) void compact_kernel(const uint8_t *dst, const uint64_t *doff, const uint32_t *len,
                                                      const int32_t *rc, const uint64_t *poff, uint32_t n,
                                                      uint8_t *packed) {
    const uint32_t lane = threadIdx.x & 63, waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += waves) {
        if (rc[i] != 0) continue;
        const uint8_t *a = dst + doff[i];
        uint8_t *b = packed + poff[i];
        for (uint32_t k = lane; k < len[i]; k += 64) b[k] = a[k];
    }
}

int scan_u32(const uint32_t *v, const int32_t *rc, uint32_t n, uint64_t *out, uint64_t *bsum, hipStream_t st) {
    const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
    hipLaunchKernelGGL(scan_local_kernel, dim3(nb), dim3(kScanBlock), 0, st, v, rc, n, out, bsum);
    hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(kScanBlock), 0, st, bsum, nb);
    hipLaunchKernelGGL(scan_add_kernel, dim3(nb), dim3(kScanBlock), 0, st, out, n, bsum);
    HIP_TRY(hipGetLastError());
    return PMC_OK;
}

int pipe_init(pmc_ctx *ctx) {
    auto &P = ctx->pipe;
    if (P.h2d) return PMC_OK;
    HIP_TRY(hipStreamCreateWithFlags(&P.h2d, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&P.d2h, hipStreamNonBlocking));
    for (int k = 0; k < 2; k++) {
        HIP_TRY(hipEventCreateWithFlags(&P.in[k], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&P.out[k], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&P.done[k], hipEventDisableTiming));
    }
    return P.total.ensure(64);
}

// Pinned host batch, chunked and software-pipelined over three streams (s = c & 1):
//   h2d:    offsets/lengths/caps of chunk c, then its source byte range  -> event in[s]
//   stream: rebase offsets, the codec kernels                            -> event out[s]
//   d2h:    dst_len, rc, then the chunk's destination bytes              -> event done[s]
// and chunk c + 2 reuses slot s after done[s].  Chunk c's source bytes are the range
// [min src_off, max src_off + src_len) of its values (packed layouts copy exactly their bytes).
// Destinations, three ways:
//   tiled slots (dst_off given, and the chunk's slots tile one range in index order:
//     dst_off[i + 1] == dst_off[i] + dst_cap[i]): the range is copied back whole, straight into dst;
//   any other slot layout (gaps, permuted or interleaved slots): the device compacts the chunk's
//     outputs, they land in a pinned bounce buffer and the host copies each output to its dst_off,
//     so no byte outside [dst_off[i], dst_off[i] + dst_len[i]) of a successful value is written;
//   packed mode (dst_off null): the compacted bytes are appended to dst.
// A compacted chunk's device slots are laid out by a scan of dst_cap, its results compacted by a
// scan of dst_len (rc != 0 -> 0 bytes); the host waits for chunk c's byte total (on the compute
// stream, after its kernels) only once chunk c + 1's kernels are enqueued, so the device never idles.
int pinned_batch_run(pmc_ctx *ctx, Dir dir, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                     uint32_t n, uint8_t *dst, const uint64_t *dst_off, const uint32_t *dst_cap, uint32_t *dst_len,
                     int32_t *rc, uint32_t max_len, uint32_t chunk) {
    if (!ctx || !src || !src_off || !src_len || !dst || !dst_cap || !dst_len || !rc) return PMC_E_ARG;
    if (n == 0) return PMC_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    int r = pipe_init(ctx);
    if (r) return r;
    auto &P = ctx->pipe;
    const bool packed = dst_off == nullptr;
    if (chunk == 0) chunk = std::max<uint32_t>(65536, (n + 15) / 16);
    auto al = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
    const uint32_t nchunks = (uint32_t)((n + (uint64_t)chunk - 1) / chunk);
    volatile uint64_t *h_total = (volatile uint64_t *)P.total.p;  // chunk totals, slot s at [s]
    uint8_t *d_pk[2] = {nullptr, nullptr};
    uint64_t out_pos = 0;
    // slot mode, compacted chunk: its outputs wait in bounce[s] until done[s], then go to dst_off
    struct Pend {
        bool on = false;
        uint32_t a = 0, m = 0;
    } pend[2];
    auto scatter = [&](uint32_t s) -> int {
        if (!pend[s].on) return PMC_OK;
        HIP_TRY(hipEventSynchronize(P.done[s]));
        const uint8_t *b = (const uint8_t *)P.bounce[s].p;
        uint64_t p = 0;
        for (uint32_t i = pend[s].a; i < pend[s].a + pend[s].m; i++)
            if (rc[i] == 0) {
                memcpy(dst + dst_off[i], b + p, dst_len[i]);
                p += dst_len[i];
            }
        pend[s].on = false;
        return PMC_OK;
    };
    // compacted chunk c's bytes go back once its total is known (called after chunk c + 1 is enqueued)
    auto finish = [&](uint32_t c) -> int {
        const uint32_t s = c & 1;
        HIP_TRY(hipEventSynchronize(P.out[s]));
        const uint64_t tot = h_total[s];
        uint8_t *to = dst + out_pos;
        if (!packed) {
            int e = scatter(s);  // chunk c - 2's outputs leave bounce[s] first
            if (e) return e;
            if ((e = P.bounce[s].ensure(tot + 64))) return e;
            to = (uint8_t *)P.bounce[s].p;
            pend[s].on = true;
            pend[s].a = c * chunk;
            pend[s].m = std::min<uint32_t>(chunk, n - c * chunk);
        }
        HIP_TRY(hipStreamWaitEvent(P.d2h, P.out[s], 0));
        if (tot) HIP_TRY(hipMemcpyAsync(to, d_pk[s], tot, hipMemcpyDeviceToHost, P.d2h));
        HIP_TRY(hipEventRecord(P.done[s], P.d2h));
        if (packed) out_pos += tot;
        return PMC_OK;
    };
    int64_t unfinished = -1;  // a compacted chunk whose D2H is not enqueued yet
    for (uint32_t c = 0; c < nchunks; c++) {
        const uint32_t a = c * chunk, m = std::min<uint32_t>(chunk, n - a), s = c & 1;
        uint64_t sb = ~0ull, se = 0, db = ~0ull, de = 0;
        for (uint32_t i = a; i < a + m; i++) {
            sb = std::min(sb, src_off[i]);
            se = std::max(se, src_off[i] + src_len[i]);
        }
        bool compact = packed;
        if (!packed) {
            for (uint32_t i = a; i + 1 < a + m && !compact; i++) compact = dst_off[i + 1] != dst_off[i] + dst_cap[i];
            db = dst_off[a];
            de = dst_off[a + m - 1] + dst_cap[a + m - 1];
        }
        if (compact) {
            db = 0;
            de = 0;
            for (uint32_t i = a; i < a + m; i++) de += dst_cap[i];
        }
        const uint32_t nb = (m + kScanBlock - 1) / kScanBlock;
        const uint64_t meta = al(m * 8ull) * 3 + al(m * 4ull) * 4 + al((nb + 1) * 8ull);
        const uint64_t need = meta + al(se - sb + 16) + al(de - db + 16) * (compact ? 2 : 1);
        if (need > P.slot[s].cap) {
            // the slot's previous chunk must have drained before it is reallocated
            if (P.busy[s]) HIP_TRY(hipEventSynchronize(P.done[s]));
            r = P.slot[s].ensure(need + need / 8);
            if (r) return r;
            P.busy[s] = false;
        }
        uint8_t *dp = (uint8_t *)P.slot[s].p;
        uint64_t *d_soff = (uint64_t *)dp, *d_doff = d_soff + al(m * 8ull) / 8, *d_poff = d_doff + al(m * 8ull) / 8;
        uint32_t *d_slen = (uint32_t *)(d_poff + al(m * 8ull) / 8);
        uint32_t *d_dcap = d_slen + al(m * 4ull) / 4, *d_dlen = d_dcap + al(m * 4ull) / 4;
        int32_t *d_rc = (int32_t *)(d_dlen + al(m * 4ull) / 4);
        uint64_t *d_bsum = (uint64_t *)(d_rc + al(m * 4ull) / 4);
        uint8_t *d_src = dp + meta, *d_dst = d_src + al(se - sb + 16);
        d_pk[s] = d_dst + al(de - db + 16);
        if (P.busy[s]) HIP_TRY(hipStreamWaitEvent(P.h2d, P.done[s], 0));
        HIP_TRY(hipMemcpyAsync(d_soff, src_off + a, m * 8ull, hipMemcpyHostToDevice, P.h2d));
        if (!compact) HIP_TRY(hipMemcpyAsync(d_doff, dst_off + a, m * 8ull, hipMemcpyHostToDevice, P.h2d));
        HIP_TRY(hipMemcpyAsync(d_slen, src_len + a, m * 4ull, hipMemcpyHostToDevice, P.h2d));
        HIP_TRY(hipMemcpyAsync(d_dcap, dst_cap + a, m * 4ull, hipMemcpyHostToDevice, P.h2d));
        HIP_TRY(hipMemcpyAsync(d_src, src + sb, se - sb, hipMemcpyHostToDevice, P.h2d));
        HIP_TRY(hipEventRecord(P.in[s], P.h2d));
        HIP_TRY(hipStreamWaitEvent(ctx->stream, P.in[s], 0));
        hipLaunchKernelGGL(rebase_kernel, dim3(std::min<uint32_t>((m + 255) / 256, 1024)), dim3(256), 0, ctx->stream,
                           d_soff, compact ? nullptr : d_doff, m, sb, db);
        HIP_TRY(hipGetLastError());
        if (compact && (r = scan_u32(d_dcap, nullptr, m, d_doff, d_bsum, ctx->stream))) return r;
        r = dir == kCompress
                ? pmc_gzip_compress_batch(ctx, d_src, d_soff, d_slen, m, d_dst, d_doff, d_dcap, d_dlen, d_rc,
                                          max_len, ctx->stream)
                : pmc_gzip_decompress_batch(ctx, d_src, d_soff, d_slen, m, d_dst, d_doff, d_dcap, d_dlen, d_rc,
                                            max_len, ctx->stream);
        if (r) return r;
        if (compact) {
            if ((r = scan_u32(d_dlen, d_rc, m, d_poff, d_bsum, ctx->stream))) return r;
            hipLaunchKernelGGL(compact_kernel, dim3(std::min<uint32_t>((m + 3) / 4, 8192)), dim3(256), 0,
                               ctx->stream, d_dst, d_doff, d_dlen, d_rc, d_poff, m, d_pk[s]);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipMemcpyAsync(dst_len + a, d_dlen, m * 4ull, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(hipMemcpyAsync(rc + a, d_rc, m * 4ull, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(hipMemcpyAsync((void *)(h_total + s), d_bsum + nb, 8, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(hipEventRecord(P.out[s], ctx->stream));
        } else {
            HIP_TRY(hipEventRecord(P.out[s], ctx->stream));
            HIP_TRY(hipStreamWaitEvent(P.d2h, P.out[s], 0));
            HIP_TRY(hipMemcpyAsync(dst_len + a, d_dlen, m * 4ull, hipMemcpyDeviceToHost, P.d2h));
            HIP_TRY(hipMemcpyAsync(rc + a, d_rc, m * 4ull, hipMemcpyDeviceToHost, P.d2h));
            HIP_TRY(hipMemcpyAsync(dst + db, d_dst, de - db, hipMemcpyDeviceToHost, P.d2h));
            HIP_TRY(hipEventRecord(P.done[s], P.d2h));
        }
        P.busy[s] = true;
        if (unfinished >= 0 && (r = finish((uint32_t)unfinished))) return r;
        unfinished = compact ? (int64_t)c : -1;
    }
    if (unfinished >= 0 && (r = finish((uint32_t)unfinished))) return r;
    // slot mode: the last compacted chunks' outputs to their dst_off, in chunk order
    for (uint32_t k = 0; k < 2; k++) {
        const uint32_t s = nchunks >= 2 ? (nchunks - 2 + k) & 1 : k;
        if ((r = scatter(s))) return r;
    }
    HIP_TRY(hipStreamSynchronize(P.d2h));
    P.busy[0] = P.busy[1] = false;
    return PMC_OK;
}

// On an error part of the batch may still be in flight on the three streams, reading and writing the
// caller's buffers: drain them before returning, so the caller may free those buffers at once.
int pinned_batch(pmc_ctx *ctx, Dir dir, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                 uint32_t n, uint8_t *dst, const uint64_t *dst_off, const uint32_t *dst_cap, uint32_t *dst_len,
                 int32_t *rc, uint32_t max_len, uint32_t chunk) {
    if (!ctx) return PMC_E_ARG;
    HostCall guard(ctx);
    const int r = pinned_batch_run(ctx, dir, src, src_off, src_len, n, dst, dst_off, dst_cap, dst_len, rc, max_len,
                                   chunk);
    if (r && ctx && ctx->pipe.h2d) {
        (void)hipStreamSynchronize(ctx->pipe.h2d);
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamSynchronize(ctx->pipe.d2h);
        ctx->pipe.busy[0] = ctx->pipe.busy[1] = false;
    }
    return r;
}

} // namespace

PMC_API int pmc_gzip_compress_batch_host(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                         const uint32_t *src_len, uint32_t n, uint8_t *dst, const uint64_t *dst_off,
                                         const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc) {
    return host_batch(ctx, kCompress, src, src_off, src_len, n, dst, dst_off, dst_cap, dst_len, rc);
}

PMC_API int pmc_gzip_decompress_batch_host(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                           const uint32_t *src_len, uint32_t n, uint8_t *dst,
                                           const uint64_t *dst_off, const uint32_t *dst_cap, uint32_t *dst_len,
                                           int32_t *rc) {
    return host_batch(ctx, kDecompress, src, src_off, src_len, n, dst, dst_off, dst_cap, dst_len, rc);
}

PMC_API int pmc_gzip_compress_batch_pinned(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                           const uint32_t *src_len, uint32_t n, uint8_t *dst,
                                           const uint64_t *dst_off, const uint32_t *dst_cap, uint32_t *dst_len,
                                           int32_t *rc, uint32_t max_len, uint32_t chunk) {
    return pinned_batch(ctx, kCompress, src, src_off, src_len, n, dst, dst_off, dst_cap, dst_len, rc, max_len,
                        chunk);
}

PMC_API int pmc_gzip_decompress_batch_pinned(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                             const uint32_t *src_len, uint32_t n, uint8_t *dst,
                                             const uint64_t *dst_off, const uint32_t *dst_cap, uint32_t *dst_len,
                                             int32_t *rc, uint32_t max_len, uint32_t chunk) {
    return pinned_batch(ctx, kDecompress, src, src_off, src_len, n, dst, dst_off, dst_cap, dst_len, rc, max_len,
                        chunk);
}

PMC_API int pmc_gzip_compress(pmc_ctx *ctx, const void *in, size_t in_len, void *out, size_t out_cap,
                              size_t *out_len) {
    *out_len = 0;
    if (!in || in_len == 0) return PMC_INVALID_INPUT;
    if (!ctx) ctx = pmc_default_ctx();
    if (!ctx) return PMC_E_NO_DEVICE;
    if (in_len > 0xffffffffull || out_cap < pmc_gzip_bound(in_len)) return PMC_E_CAPACITY;
    uint64_t so = 0;
    uint32_t sl = (uint32_t)in_len, cap = (uint32_t)std::min<size_t>(out_cap, 0xffffffffull), dl = 0;
    int32_t rc = 0;
    int r = host_batch(ctx, kCompress, (const uint8_t *)in, &so, &sl, 1, (uint8_t *)out, &so, &cap, &dl, &rc);
    if (r) return r;
    *out_len = dl;
    return rc;
}

PMC_API int pmc_gzip_decompress(pmc_ctx *ctx, const void *in, size_t in_len, void *out, size_t out_cap,
                                size_t *out_len) {
    *out_len = 0;
    if (!in || in_len == 0) return PMC_INVALID_INPUT;
    if (!ctx) ctx = pmc_default_ctx();
    if (!ctx) return PMC_E_NO_DEVICE;
    uint64_t so = 0;
    uint32_t sl = (uint32_t)in_len, cap = (uint32_t)std::min<size_t>(out_cap, 0xffffffffull), dl = 0;
    int32_t rc = 0;
    int r = host_batch(ctx, kDecompress, (const uint8_t *)in, &so, &sl, 1, (uint8_t *)out, &so, &cap, &dl, &rc);
    if (r) return r;
    *out_len = dl;
    return rc;
}

// ---- helpers -------------------------------------------------------------------------
static dim3 grid_for(uint64_t items, int per_thread = 1) {
    uint64_t b = (items / per_thread + 255) / 256;
    return dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(b, 1u << 16)));
}

PMC_API int pmc_gen_values(const uint8_t *corpus, uint32_t corpus_len, uint64_t seed, int kind, uint64_t first,
                           const uint64_t *index, uint32_t n, uint32_t vlen, uint8_t *dst, void *stream) {
    if (!n || !vlen || (kind == 0 && vlen > corpus_len)) return PMC_E_ARG;
    hipLaunchKernelGGL(gen_values_kernel, grid_for((uint64_t)n * ((vlen + 7) / 8)), dim3(256), 0,
                       (hipStream_t)stream, corpus, corpus_len, seed, kind, first, index, n, vlen, dst);
    return hipGetLastError() == hipSuccess ? PMC_OK : PMC_E_NO_DEVICE;
}

PMC_API int pmc_fill_layout(uint64_t *off, uint32_t *len, uint32_t *cap, uint32_t n, uint64_t stride, uint32_t vlen,
                            uint32_t capv, void *stream) {
    if (!n) return PMC_OK;
    hipLaunchKernelGGL(fill_layout_kernel, grid_for(n), dim3(256), 0, (hipStream_t)stream, off, len, cap, n, stride,
                       vlen, capv);
    return hipGetLastError() == hipSuccess ? PMC_OK : PMC_E_NO_DEVICE;
}

PMC_API int pmc_compare_values(const uint8_t *a, const uint64_t *a_off, const uint8_t *b, const uint64_t *b_off,
                               const uint32_t *len, const uint32_t *len_b, uint32_t n, uint32_t *mismatches,
                               void *stream) {
    if (!n) return PMC_OK;
    hipLaunchKernelGGL(compare_values_kernel, dim3(std::min<uint32_t>((n + 3) / 4, 8192)), dim3(256), 0,
                       (hipStream_t)stream, a, a_off, b, b_off, len, len_b, n, mismatches);
    return hipGetLastError() == hipSuccess ? PMC_OK : PMC_E_NO_DEVICE;
}

PMC_API int pmc_route_keys(uint64_t first, uint32_t n, uint32_t num_shards, uint32_t n_gpus, uint8_t *gpu,
                           void *stream) {
    if (!n || !num_shards || !n_gpus) return PMC_E_ARG;
    hipLaunchKernelGGL(route_kernel, grid_for(n), dim3(256), 0, (hipStream_t)stream, first, n, num_shards, n_gpus,
                       gpu);
    return hipGetLastError() == hipSuccess ? PMC_OK : PMC_E_NO_DEVICE;
}

// Diagnostics: device buffer of 32 uint64 that PMC_STAMPS builds add per-phase cycles into.
PMC_API int pmc_debug_stamps(pmc_ctx *ctx, uint64_t *dev_buf) {
    if (!ctx) return PMC_E_ARG;
    ctx->dbg = dev_buf;
    return PMC_OK;
}
