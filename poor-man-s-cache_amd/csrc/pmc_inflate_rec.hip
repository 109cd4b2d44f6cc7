// pmc_inflate_rec.hip -- two-phase lane inflate for members whose output fits a 4 KiB image.
//
// inflate_lane_kernel decodes one member per lane and copies every match byte by byte
// through a per-lane ring: a wave iterates once per symbol AND once per 8 match bytes, reads
// far matches back from dst (a global load that also waits for the ring's earlier stores:
// gfx9 loads and stores share vmcnt) and holds 40 KB of LDS (4 waves per CU).  Here the
// work is split by what parallelises (reference: /root/reference/src/compressor/
// gzip_compressor.cpp:52-111, zlib 1.2.11 inflate_fast):
//   phase A (lane per member): Huffman-decode the member into RECORDS, one per loop step:
//     a group of 1-3 literals (bits 31:30 = count, bytes in 23:0) or a match
//     (bits 31:30 = 0, length - 3 in 7:0, distance - 1 in 22:8).  No byte is produced, so a
//     step never reads dst; records are staged in LDS and flushed to a per-lane scratch row.
//     The input window is refilled from registers loaded one half ahead, so its global loads
//     have a window's worth of steps to land.
//   phase B (wave per member, the wave's 64 decoded members in turn): a DPP scan of the
//     records' lengths gives every record its output position; a start bitmap + popcount maps
//     each output position to its record; a literal position holds its byte, a match
//     position points distance bytes back; pointer jumping (src[p] = src[src[p]]) resolves
//     every position to the literal it copies, in log(depth) rounds over LDS; the image goes
//     to dst with coalesced dword stores.
// Members of more than kRecOutMax output bytes (by their ISIZE trailer) are left to
// inflate_lane_kernel (rc = kInflateBig); everything phase A cannot decode exactly is marked
// kInflateRetry for the wave kernels, as in the lane kernel.  The CRC-32 is checked by
// inflate_verify_kernel.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "pmc_device.hpp"
#include "pmc_kernels.hpp"

namespace pmc {

#ifndef PMC_REC_STAGE
#define PMC_REC_STAGE 4 // (8 until round 5: 4 frees 1 KB of LDS per wave)
#endif
// input window per lane (dwords, refilled by halves with the next half prefetched into registers):
// (8 fits a 10th wave per CU at the 1 KiB image but measured no faster than 16: round 5, same box)
#ifndef PMC_REC_WIN
#define PMC_REC_WIN 16
#endif
constexpr uint32_t kRecWinDw = PMC_REC_WIN, kRecWinHalf = kRecWinDw / 2;
static_assert(kRecWinDw == 8 || kRecWinDw == 16, "window halves of one or two uint4");
constexpr uint32_t kRecStage = PMC_REC_STAGE;         // staged records per lane (LDS column)
constexpr uint32_t kRecFlushAt = 4;                   // a lane with a whole group makes the wave flush
// (a flush leaves < 4 records pending, one step adds one: the ring never holds more than kRecFlushAt)
static_assert(kRecFlushAt >= 4 && kRecFlushAt <= kRecStage && kRecStage % 4 == 0, "record stage ring");
// lists of the record kernel: members of <= 4096 output bytes use distance codes 0..23 only (members
// whose lists do not fit go to the lane kernel).  (88 lit/len entries and a 4-record stage fit 7
// blocks per CU by bytes, but measured no faster than 6: LDS allocation granularity)
#ifndef PMC_REC_LIT
#define PMC_REC_LIT 96
#endif
// PMC_REC8: the symbol lists as bytes (u16 before round 5): a literal/length symbol is its low 8 bits
// plus the rule that in each code length's run of the (length, symbol)-sorted list the literals come
// first, so one byte per length (the run's first entry >= 256: "split") restores the ninth bit.  The
// columns shrink from 300 to 195 B per lane: 25.3 -> 18.6 KB of LDS per wave, 6 -> 8 waves per CU for
// the 1 KiB image (the kernel waits on LDS and memory latency; round 2 measured 5 -> 6 waves as
// 82 -> 70 ms).
#ifndef PMC_REC8
#define PMC_REC8 1
#endif
// PMC_REC_OUT1K: a batch whose outputs are all <= 1 KiB (dst_cap) runs the instance whose phase B
// image holds 1 KiB (phase B's LDS then fits inside phase A's); others the 4 KiB image.
// PMC_REC_DPOS: phase B keeps each record's match distance at the record's start position (in the
// position array itself) instead of a per-record array indexed through a popcount of the start bitmap:
// two 16-byte LDS reads per lane per 1,024 positions instead of sixteen u16 reads
#ifndef PMC_REC_DPOS
#define PMC_REC_DPOS 1
#endif
#ifndef PMC_REC_OUT1K
#define PMC_REC_OUT1K 1
#endif
typedef LaneCols<PMC_REC_LIT, 24> RecCols;
// byte-column layout per lane: lit/len and distance bases (int16 columns, entry i of lane l at u16 word
// i * 64 + l), then byte columns (entry i at byte i * 64 + l): lit/len symbols' low bytes, the splits
// (lengths 1..15), distance symbols
struct RecCols8 {
    static constexpr int kLit = PMC_REC_LIT, kDist = 24;
    static constexpr int kColBaseL = 0, kColBaseD = 15;
    static constexpr uint32_t kSymL = 30 * 128, kSplit = kSymL + kLit * 64, kSymD = kSplit + 15 * 64;
    static constexpr uint32_t kBytes = kSymD + kDist * 64;
    static constexpr int kColWords = (int)((kBytes + 127) / 128); // (u16 words per lane, for the layout below)
    // lane_lengths' pass 1: the symbol's low byte to entry `at`; reaching 256 (end of block, the first
    // symbol >= 256, always of nonzero length) the current offsets per length are the splits
    __device__ static __forceinline__ void place(PMC_LDS uint16_t *col, bool lit, uint32_t at, uint32_t sym,
                                                 uint32_t len, PMC_LDS const uint8_t *bcol) {
        const uint32_t l = (uint32_t)lane_id();
        PMC_LDS uint8_t *b = (PMC_LDS uint8_t *)(col - l) + l;
        if (lit && sym == 256) {
#pragma unroll
            for (uint32_t L = 1; L <= 15; L++)
                b[kSplit + (L - 1) * 64] = L == len ? (uint8_t)at : bcol[(kBColCntL + L) * 64];
        }
        b[(lit ? kSymL : kSymD) + at * 64] = (uint8_t)sym;
    }
};
typedef std::conditional<PMC_REC8 != 0, RecCols8, RecCols>::type RecColsK;
static_assert((kRecStage & (kRecStage - 1)) == 0, "stage ring: a power of two");
// phase A: code columns | input windows | record stage (the build columns live from the window on,
// which starts only after the tables are built)
constexpr uint32_t kRecWinOff = PMC_REC8 ? RecCols8::kBytes : (uint32_t)RecCols::kColWords * 64 * 2;
static_assert(kRecWinOff % 16 == 0, "window dwords aligned");
constexpr uint32_t kRecStageOff = kRecWinOff + kRecWinDw * 64 * 4;
constexpr uint32_t kRecBColBytes = (kBColCl + 19) * 64;
constexpr uint32_t kRecALds = kRecWinOff + ((kRecWinDw + kRecStage) * 64 * 4 > kRecBColBytes
                                                ? (kRecWinDw + kRecStage) * 64 * 4 : kRecBColBytes);
// phase B: two output images (16 B of head room so dword -1 reads) | src u16 | start bitmap |
// per record: its match distance, or 0 for literals (whose bytes go straight to the image)
template <uint32_t OUT>
struct RecB {
    static constexpr uint32_t kOut0 = 16;
    static constexpr uint32_t kOut1 = kOut0 + OUT + 32;
    static constexpr uint32_t kSrc = kOut1 + OUT + 32;
    static constexpr uint32_t kBits = kSrc + 2 * OUT;
#if PMC_REC_DPOS
    // (a record's distance sits at its start position in the src array, written before the position round
    // overwrites that position: no per-record array)
    static constexpr uint32_t kEnd = kBits + OUT / 8;
#else
    static constexpr uint32_t kRecD = kBits + OUT / 8;
    static constexpr uint32_t kEnd = kRecD + 2 * (OUT < kRecMax ? OUT : kRecMax); // (records <= output bytes)
#endif
    static constexpr uint32_t kLds = kEnd > kRecALds ? kEnd : kRecALds;          // phase B reuses phase A's LDS
    static_assert(OUT % 1024 == 0, "positions resolve 1024 at a time");
};
uint32_t rec_lds_bytes(uint32_t out) { return out == 1024 ? RecB<1024>::kLds : RecB<kRecOutMax>::kLds; }

// LaneWinP with the next half loaded into registers one advance ahead
struct LaneWinP {
    static constexpr uint32_t kQ = kRecWinHalf / 4; // uint4 per half
    PMC_LDS uint32_t *w;
    PMC_GLB const uint4 *blk;
    uint32_t nblk, head, wlo, nd;
    uint64_t buf;
    uint32_t n;
    uint4 pf[kQ]; // dwords wlo + kRecWinDw .. + kRecWinHalf - 1
    __device__ uint4 block(uint32_t k) const { return k < nblk ? gload16(blk + k) : make_uint4(0, 0, 0, 0); }
    __device__ void put_half(uint32_t d0, const uint4 *x) {
        const uint32_t s0 = d0 & (kRecWinDw - 1);
#pragma unroll
        for (uint32_t q = 0; q < kQ; q++) {
            w[(s0 + 4 * q + 0) * 64] = x[q].x;
            w[(s0 + 4 * q + 1) * 64] = x[q].y;
            w[(s0 + 4 * q + 2) * 64] = x[q].z;
            w[(s0 + 4 * q + 3) * 64] = x[q].w;
        }
    }
    __device__ void start(const LaneIn &in, uint64_t bp, bool live) {
        blk = in.blk;
        head = (uint32_t)(((uintptr_t)in.p & 15) * 8);
        nblk = live ? (uint32_t)((((uintptr_t)in.p & 15) + in.len + 15) / 16) : 0u;
        const uint64_t a = bp + head;
        nd = (uint32_t)(a >> 5);
        wlo = nd & ~(kRecWinHalf - 1);
        uint4 x[kQ], y[kQ];
#pragma unroll
        for (uint32_t q = 0; q < kQ; q++) {
            x[q] = block(wlo / 4 + q);
            y[q] = block(wlo / 4 + kQ + q);
            pf[q] = block(wlo / 4 + 2 * kQ + q);
        }
        put_half(wlo, x);
        put_half(wlo + kRecWinHalf, y);
        buf = 0;
        n = 0;
        refill();
        drop((uint32_t)(a & 31));
    }
    __device__ void refill() { // branch-free: the dword is read either way (its slot always exists)
        const uint32_t x = w[(nd & (kRecWinDw - 1)) * 64];
        const uint32_t r = n <= 32 ? 1u : 0u;
        buf |= r ? (uint64_t)x << n : 0ull;
        n += 32 * r;
        nd += r;
    }
    __device__ bool needs() const { return nd + 4 > wlo + kRecWinDw; }
    __device__ void advance() { // retire the consumed older half: the prefetched half takes its slots
        if (nd >= wlo + kRecWinHalf) {
            put_half(wlo + kRecWinDw, pf);
            wlo += kRecWinHalf;
#pragma unroll
            for (uint32_t q = 0; q < kQ; q++) pf[q] = block((wlo + kRecWinDw) / 4 + q);
        }
    }
    __device__ uint32_t peek(uint32_t k) const { return (uint32_t)buf & ((1u << k) - 1); }
    __device__ void drop(uint32_t k) {
        buf >>= k;
        n -= k;
    }
    __device__ uint32_t bits(uint32_t k) {
        refill();
        const uint32_t v = peek(k);
        drop(k);
        return v;
    }
    __device__ uint64_t bitpos() const { return (uint64_t)nd * 32 - n - head; }
};

typedef uint32_t rec_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t rec_olen(uint32_t w) { return (w >> 30) ? (w >> 30) : (w & 0xff) + 3; }

// the lit/len code over byte lists (RecCols8): the split of the code length restores bit 8
struct LaneCode8 : LaneCode<15, int16_t, uint8_t> {
    PMC_LDS uint8_t *split;
    template <class R>
    __device__ __forceinline__ uint32_t sym_at(const R &in, uint32_t &len) const {
        const uint32_t x = __builtin_bitreverse32(in.peek(15)) >> 17;
        const uint32_t L = code_len(x);
        const int idx = (int)base[(L - 1) * 64] + (int)(x >> (15 - L));
        const uint32_t sp = split[(L - 1) * 64];
        len = L;
        return (uint32_t)sym[idx * 64] + ((uint32_t)idx >= sp ? 256u : 0u);
    }
    template <class R>
    __device__ __forceinline__ uint32_t peek_sym(const R &in, uint32_t &len) const { return sym_at(in, len); }
    template <class R>
    __device__ __forceinline__ uint32_t decode(R &in) const {
        uint32_t L;
        const uint32_t s = sym_at(in, L);
        in.drop(L);
        return s;
    }
};

template <uint32_t OUT>
__global__ void __launch_bounds__(64) inflate_rec_kernel(InflateArgs a) {
    typedef RecB<OUT> B;
    constexpr uint32_t kRecOutMax = OUT; // (this instance's image; members of more output: the lane kernel)
    extern __shared__ __attribute__((aligned(16))) uint16_t lcol[];
    uint8_t *lds = (uint8_t *)lcol;
    const uint32_t lane = threadIdx.x;
    PMC_LDS uint16_t *col = to_lds<uint16_t>(lcol + lane);
    PMC_LDS uint32_t *winw = to_lds<uint32_t>((uint32_t *)(lds + kRecWinOff) + lane);
    PMC_LDS uint32_t *stg = to_lds<uint32_t>((uint32_t *)(lds + kRecStageOff) + lane);
    PMC_LDS uint8_t *bcol = to_lds<uint8_t>(lds + kRecWinOff + lane);
    PMC_LDS uint8_t *ob0 = to_lds<uint8_t>(lds + B::kOut0), *ob1 = to_lds<uint8_t>(lds + B::kOut1);
    PMC_LDS uint16_t *srcv = to_lds<uint16_t>((uint16_t *)(lds + B::kSrc));
    PMC_LDS uint32_t *bits = to_lds<uint32_t>((uint32_t *)(lds + B::kBits));
#if !PMC_REC_DPOS
    PMC_LDS uint16_t *recd = to_lds<uint16_t>((uint16_t *)(lds + B::kRecD));
#endif
    const uint32_t rstride = a.rec_stride;
    PMC_GLB uint32_t *const rows = (PMC_GLB uint32_t *)a.rec_scratch + (uint64_t)blockIdx.x * 64 * rstride;
    PMC_GLB uint32_t *const row = rows + (uint64_t)lane * rstride;
    // 64-member batches from a work counter, the next grab in flight while a batch runs (a block
    // that becomes resident late finds less work instead of adding a tail)
    // A batch too small to fill the CUs at 64 members per wave grabs fewer (a.rec_group): phase A then
    // runs on that many lanes and phase B's member-serial loop is that short.
    const uint32_t G = a.rec_group ? a.rec_group : 64u;
    uint32_t nx = lane == 0 ? atomicAdd(a.rec_work, 1u) : 0u;
    for (;;) {
        const uint64_t vb = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)nx, 0) * G;
        if (vb >= a.n) break;
        nx = lane == 0 ? atomicAdd(a.rec_work, 1u) : 0u;
        const uint64_t vi = lane < G ? vb + lane : a.n; // (lanes past the group: no member)
        // (longest members first: batches are handed out in order, so the kernel's last ones are short)
        const uint64_t v = a.order && vi < a.n ? (uint64_t)a.order[a.n - 1 - vi] : vi;
        const uint32_t in_len = v < a.n ? a.src_len[v] : 0u;
        // st: 0 decoding, 1 end of block reached, 2 declined, 3 no member / empty input,
        // 4 output larger than the image (inflate_lane_kernel's)
        uint32_t st = v < a.n ? 0u : 3u;
        if (st == 0 && in_len == 0) {
            a.rc[v] = PMC_INVALID_INPUT_DEV;
            a.dst_len[v] = 0;
            st = 3;
        }
        LaneIn in;
        in.p = st == 0 ? a.src + a.src_off[v] : a.src;
        in.len = st == 0 ? in_len : 0u;
        in.blk = (PMC_GLB const uint4 *)((uintptr_t)in.p & ~(uintptr_t)15);
        const uint32_t cap = st == 0 ? a.dst_cap[v] : 0u;
        const uint64_t dptr = st == 0 ? (uint64_t)(uintptr_t)(a.dst + a.dst_off[v]) : 0u;
        if (st == 0) {
            if (in_len < 18) {
                st = 2;
            } else {
                const uint32_t isz = in.byte_at(in_len - 4) | in.byte_at(in_len - 3) << 8 |
                                     in.byte_at(in_len - 2) << 16 | in.byte_at(in_len - 1) << 24;
                if (isz > cap) st = 2;
                else if (isz > a.rec_max_out) st = 4;
            }
        }
#if PMC_REC8
        LaneCode8 lit;
        LaneCode<15, int16_t, uint8_t> dist;
        {
            PMC_LDS uint8_t *b8 = (PMC_LDS uint8_t *)(col - lane) + lane;
            lit.base = (PMC_LDS int16_t *)(col + RecCols8::kColBaseL * 64);
            lit.sym = b8 + RecCols8::kSymL;
            lit.split = b8 + RecCols8::kSplit;
            dist.base = (PMC_LDS int16_t *)(col + RecCols8::kColBaseD * 64);
            dist.sym = b8 + RecCols8::kSymD;
        }
#else
        LaneCode<15> lit, dist;
        lit.base = (PMC_LDS int16_t *)(col + RecCols::kColBaseL * 64);
        lit.sym = col + RecCols::kColLit * 64;
        dist.base = (PMC_LDS int16_t *)(col + RecCols::kColBaseD * 64);
        dist.sym = col + RecCols::kColDist * 64;
#endif
        bool fixed = false;
#ifdef PMC_STAMPS
        uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
        bool over = false;
        if (st == 0 && !lane_prepare<RecColsK>(in, col, bcol, lit, dist, fixed, &over, kLaneWideLit, kLaneDistCap))
            st = over ? 4u : 2u; // (lists the lane kernels hold: theirs)
#ifdef PMC_STAMPS
        uint64_t t1 = __builtin_amdgcn_s_memtime();
        uint64_t n_it = 0, n_act = 0;
#endif
#if defined(PMC_STAMPS) || defined(PMC_PHASE_STOP)
        if (a.stop_after == 31 && st == 0) st = 3;
#endif
        LaneWinP win;
        win.w = winw;
        win.start(in, st == 0 ? in.bitpos() : 0, st == 0);
        const uint32_t ocap = cap < kRecOutMax ? cap : kRecOutMax;
        uint32_t pos = 0, nrec = 0, nfl = 0;
        // ---- phase A: one record per step (a wave without fixed-code members runs the loop
        // without the fixed-code paths) ----
        auto phase_a = [&](auto fxc) {
            constexpr bool FX = decltype(fxc)::value;
            while (ballot(st == 0)) {
    #ifdef PMC_STAMPS
                n_it++;
                n_act += __builtin_popcountll(ballot(st == 0));
    #endif
                if (ballot(st == 0 && win.needs()))
                    if (st == 0) win.advance();
                if (st == 0) {
                    win.refill();
                    const uint32_t sy = FX && fixed ? fixed_lit(win) : lit.decode(win);
                    uint32_t rec = 0, olen = 0;
                    if (sy < 256) {
                        // literals are most of the steps: up to three per record (the refilled
                        // buffer holds >= 17 bits after one code, a full peek)
                        rec = sy;
                        olen = 1;
                        uint32_t l2;
                        const uint32_t s2 = FX && fixed ? fixed_peek(win, l2) : lit.peek_sym(win, l2);
                        if (s2 < 256) {
                            win.drop(l2);
                            rec |= s2 << 8;
                            olen = 2;
                            win.refill();
                            uint32_t l3;
                            const uint32_t s3 = FX && fixed ? fixed_peek(win, l3) : lit.peek_sym(win, l3);
                            if (s3 < 256) {
                                win.drop(l3);
                                rec |= s3 << 16;
                                olen = 3;
                            }
                        }
                        rec |= olen << 30;
                    } else if (sy == 256) {
                        st = 1;
                    } else if (sy > 285) {
                        st = 2;
                    } else {
                        // length / distance bases and extra bits in closed form (RFC 1951 3.2.5)
                        const uint32_t li = sy - 257;
                        const uint32_t lx = li < 8 || li == 28 ? 0u : (li - 4) >> 2;
                        const uint32_t lb = li < 8 ? li + 3 : li == 28 ? 258u : ((4 + (li & 3)) << lx) + 3;
                        const uint32_t len = lb + win.bits(lx);
                        win.refill();
                        const uint32_t ds = FX && fixed ? __builtin_bitreverse32(win.peek(5)) >> 27 : dist.decode(win);
                        if (FX && fixed) win.drop(5);
                        const uint32_t dx = ds < 4 ? 0u : (ds >> 1) - 1;
                        const uint32_t db = ds < 4 ? ds + 1 : ((2 + (ds & 1)) << dx) + 1;
                        const uint32_t d = db + win.bits(dx < 14 ? dx : 0u);
                        if (ds > 29 || d > pos) st = 2;
                        rec = (len - 3) | (d - 1) << 8;
                        olen = len;
                    }
                    if (st == 0) {
                        if (pos + olen > ocap) {
                            st = 2;
                        } else if (nrec >= rstride) { // more records than a row holds: the lane kernel's
                            st = 4;
                        } else {
                            stg[(nrec & (kRecStage - 1)) * 64] = rec;
                            nrec++;
                            pos += olen;
                        }
                    }
                }
                // wave-synchronous flush of whole 4-record groups (one 16-byte store each): the
                // wave stores records a few times per member
                if (ballot(st == 0 && nrec - nfl >= kRecFlushAt))
                    if (st == 0) {
                        const uint32_t e = nrec & ~3u;
                        for (uint32_t k = nfl; k < e; k += 4) {
                            typedef uint32_t r_v4u __attribute__((ext_vector_type(4)));
                            const uint32_t s0 = k & (kRecStage - 1);
                            *(PMC_GLB r_v4u *)(row + k) = r_v4u{stg[s0 * 64], stg[(s0 + 1) * 64], stg[(s0 + 2) * 64],
                                                                stg[(s0 + 3) * 64]};
                        }
                        nfl = e;
                    }
            }
        };
        if (ballot(st == 0 && fixed)) phase_a(std::true_type{});
        else phase_a(std::false_type{});
#ifdef PMC_STAMPS
        uint64_t t2 = __builtin_amdgcn_s_memtime();
#endif
        if (st == 1 && win.bitpos() > (uint64_t)in.len * 8) st = 2;
        if (st == 1) {
            const uint32_t t = (uint32_t)((win.bitpos() + 7) >> 3);
            if (t + 8 > in.len) {
                st = 2;
            } else {
                const uint32_t isz = in.byte_at(t + 4) | in.byte_at(t + 5) << 8 | in.byte_at(t + 6) << 16 |
                                     in.byte_at(t + 7) << 24;
                if (isz != pos) {
                    st = 2;
                } else {
                    for (uint32_t k = nfl; k < nrec; k++) row[k] = stg[(k & (kRecStage - 1)) * 64];
                    a.crc_expect[v] =
                        in.byte_at(t) | in.byte_at(t + 1) << 8 | in.byte_at(t + 2) << 16 | in.byte_at(t + 3) << 24;
                }
            }
        }
        if (st == 2) a.rc[v] = kInflateRetry;
        if (st == 4) {
            a.rc[v] = kInflateBig;
            if (a.big_list) a.big_list[atomicAdd(a.big_count, 1u)] = (uint32_t)v;
        }
        // ---- phase B: the wave rebuilds each decoded member in LDS and stores it ----
        wave_sync_global(); // rows visible to the whole wave; phase A's LDS is dead from here
#ifdef PMC_STAMPS
        uint64_t t2b = __builtin_amdgcn_s_memtime();
        uint64_t n_jump = 0, n_recs = 0, n_mem = 0;
#endif
        // Phase B runs in PASSES over the 1024-position image: members of <= 256 output bytes
        // four at a time (a 256-position slice each), larger ones one at a time.  Pipelined per
        // pass: (a) its records (prefetched into registers during the previous pass) become the
        // scan / bitmap tables, (b) the next pass's records are requested, (c) the previous
        // pass's images (in the other LDS image buffer) are stored, (d) the pass resolves in
        // LDS.  A wait for (a)'s registers then covers loads and stores issued a pass earlier.
        uint64_t todo = ballot(st == 1);
#if defined(PMC_STAMPS) || defined(PMC_PHASE_STOP)
        if (a.stop_after == 32) todo = 0;
#endif
        auto rl = [](uint32_t x, int m) { return (uint32_t)__builtin_amdgcn_readlane((int)x, m); };
        auto rl64 = [&](uint64_t x, int m) { return (uint64_t)rl((uint32_t)x, m) | (uint64_t)rl((uint32_t)(x >> 32), m) << 32; };
        auto store_image = [&](PMC_LDS const uint32_t *imgw, uint64_t dptr, uint32_t osz) {
            // dst dword k holds positions 4k - a0 .. 4k - a0 + 3; a lane stores 4 dwords at once
            PMC_GLB uint8_t *dp = (PMC_GLB uint8_t *)dptr;
            const uint32_t a0 = (uint32_t)(dptr & 3);
            PMC_GLB uint32_t *dw = (PMC_GLB uint32_t *)(dptr - a0);
            const uint32_t ndw = (a0 + osz + 3) / 4;
            for (uint32_t k = 4 * lane; k < ndw; k += 256) {
                const int32_t q = (int32_t)(4 * k) - (int32_t)a0; // first position of dword k
                const int32_t j = q >> 2;                          // image dword holding q (j >= -1)
                uint32_t w[5], x[4];
#pragma unroll
                for (int t = 0; t < 5; t++) w[t] = imgw[j + t];
#pragma unroll
                for (int t = 0; t < 4; t++) x[t] = a0 ? __builtin_amdgcn_alignbyte(w[t + 1], w[t], 4 - a0) : w[t];
                if (q >= 0 && (uint32_t)q + 16 <= osz) {
                    typedef uint32_t g_v4u __attribute__((ext_vector_type(4)));
                    *(PMC_GLB g_v4u *)(dw + k) = g_v4u{x[0], x[1], x[2], x[3]};
                } else {
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        const int32_t qt = q + 4 * t;
                        if (qt >= 0 && (uint32_t)qt + 4 <= osz) {
                            dw[k + t] = x[t];
                        } else {
#pragma unroll
                            for (int b = 0; b < 4; b++) {
                                const int32_t p = qt + b;
                                if (p >= 0 && (uint32_t)p < osz) dp[p] = (uint8_t)(x[t] >> (8 * b));
                            }
                        }
                    }
                }
            }
        };
        uint32_t buf = 0;
        auto run_passes = [&](auto Gc, uint64_t set) {
            constexpr int G = decltype(Gc)::value;
            constexpr uint32_t span = 1024 / G;
            uint32_t rg[4] = {0, 0, 0, 0};
            // the next pass: up to G members from t
            auto plan = [&](uint64_t &t, int *pm) {
#pragma unroll
                for (int g = 0; g < G; g++) {
                    pm[g] = t ? __builtin_ctzll(t) : -1;
                    t &= t - 1;
                }
            };
            auto fetch = [&](const int *pm) {
                if (G == 1) {
                    const uint32_t mr = rl(nrec, pm[0]);
                    PMC_GLB const uint32_t *mrow = rows + (uint64_t)pm[0] * rstride;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint32_t k = lane + 64 * j;
                        rg[j] = k < mr ? mrow[k] : 0u;
                    }
                } else {
#pragma unroll
                    for (int g = 0; g < G; g++) {
                        rg[g] = 0;
                        if (pm[g] >= 0 && lane < rl(nrec, pm[g])) rg[g] = rows[(uint64_t)pm[g] * rstride + lane];
                    }
                }
            };
            int cm[G], pm[G], nm[G];
            uint32_t p_osz[G];
            uint64_t p_dst[G], p_v[G];
#pragma unroll
            for (int g = 0; g < G; g++) pm[g] = -1;
            auto flush_prev = [&]() {
                PMC_LDS const uint32_t *img = (PMC_LDS const uint32_t *)(buf ? ob0 : ob1);
#pragma unroll
                for (int g = 0; g < G; g++) {
                    if (pm[g] < 0) continue;
                    store_image(img + (uint32_t)g * span / 4, p_dst[g], p_osz[g]);
                    if (lane == 0) {
                        a.dst_len[p_v[g]] = p_osz[g];
                        a.rc[p_v[g]] = 0;
                    }
                }
            };
            plan(set, nm);
            if (nm[0] >= 0) fetch(nm);
            while (nm[0] >= 0) {
                uint32_t osz[G], mrec[G];
#pragma unroll
                for (int g = 0; g < G; g++) {
                    cm[g] = nm[g];
                    osz[g] = cm[g] >= 0 ? rl(pos, cm[g]) : 0u;
                    mrec[g] = cm[g] >= 0 ? rl(nrec, cm[g]) : 0u;
                }
                PMC_LDS uint8_t *ob = buf ? ob1 : ob0;
                // (a) record starts: scan of the records' output lengths; bitmap of the starts
                const uint32_t ext = G == 1 ? osz[0] : 1024u; // image positions of the pass
                for (uint32_t k = lane; k < (ext + 31) / 32; k += 64) bits[k] = 0;
                wave_sync();
                uint32_t R = 0; // (records before this member's in the pass)
#pragma unroll
                for (int g = 0; g < G; g++) {
                    if (cm[g] < 0) continue;
                    PMC_GLB const uint32_t *mrow = rows + (uint64_t)cm[g] * rstride;
                    const uint32_t P = (uint32_t)g * span, mr = mrec[g];
                    uint32_t carry = 0;
                    for (uint32_t k0 = 0; k0 < mr; k0 += 64) {
                        const uint32_t k = k0 + lane, j = k0 / 64;
                        uint32_t w;
                        if (G == 1) w = j == 0 ? rg[0] : j == 1 ? rg[1] : j == 2 ? rg[2] : j == 3 ? rg[3] : k < mr ? mrow[k] : 0u;
                        else w = j == 0 ? rg[g] : k < mr ? mrow[k] : 0u;
                        const uint32_t ol = k < mr ? rec_olen(w) : 0u;
                        const uint32_t incl = wave_incl_scan_dpp(ol) + carry;
                        const uint32_t s = P + incl - ol;
                        if (k < mr) {
                            // a literal record places its bytes now; a match keeps its distance
                            const uint32_t nl = w >> 30;
#if PMC_REC_DPOS
                            srcv[s] = (uint16_t)(nl ? 0u : ((w >> 8) & 0x7fff) + 1); // (at the start position)
#else
                            recd[R + k] = (uint16_t)(nl ? 0u : ((w >> 8) & 0x7fff) + 1);
#endif
                            lds_or(&bits[s >> 5], 1u << (s & 31));
                            if (nl) ob[s] = (uint8_t)w;
                            if (nl >= 2) ob[s + 1] = (uint8_t)(w >> 8);
                            if (nl == 3) ob[s + 2] = (uint8_t)(w >> 16);
                        }
                        carry = rl(incl, 63);
                    }
                    R += mr;
                    (void)R;
                }
                wave_sync();
                // (b) the next pass's records; (c) the previous pass's images
                plan(set, nm);
                if (nm[0] >= 0) fetch(nm);
                flush_prev();
                // (d) positions, 1024 per round (16 per lane): record, literal byte or source position
#if PMC_REC_DPOS
                uint32_t carry = 0; // (start position + 1) << 16 | distance of the last record start so far
#else
                uint32_t before = 0;
#endif
                for (uint32_t c0 = 0; c0 < ext; c0 += 1024) {
                    const uint32_t p0 = c0 + 16 * lane;
                    // end of the valid positions of the lane's member
                    uint32_t lim = osz[0];
                    if (G > 1) {
                        const uint32_t gl = p0 / span;
#pragma unroll
                        for (int g = 1; g < G; g++)
                            if (gl == (uint32_t)g) lim = osz[g];
                        lim += gl * span;
                    }
                    const uint32_t bw = p0 < lim ? (bits[p0 >> 5] >> (p0 & 16)) & 0xffffu : 0u;
                    uint32_t sp[16];
#if PMC_REC_DPOS
                    // the distances at the lane's 16 positions (valid at record starts) in two 16-byte
                    // reads, and the last start below the lane by a max-scan of (position, distance)
                    uint32_t dv[8];
                    {
                        const rec_v4u d0 = *(PMC_LDS const rec_v4u *)(srcv + p0), d1 = *(PMC_LDS const rec_v4u *)(srcv + p0 + 8);
                        dv[0] = d0.x, dv[1] = d0.y, dv[2] = d0.z, dv[3] = d0.w, dv[4] = d1.x, dv[5] = d1.y, dv[6] = d1.z, dv[7] = d1.w;
                    }
                    uint32_t dls = 0; // the distance at the lane's last start (a select chain: no indexed registers)
#pragma unroll
                    for (int i = 0; i < 16; i++) dls = (bw >> i) & 1u ? (dv[i >> 1] >> (16 * (i & 1))) & 0xffffu : dls;
                    const uint32_t ls = bw ? 31u - (uint32_t)__builtin_clz(bw) : 0u;
                    const uint32_t key = bw ? (p0 + ls + 1) << 16 | dls : 0u;
                    const uint32_t inc = wave_incl_max_dpp(key);
                    uint32_t cur = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x138, 0xf, 0xf, false); // wave_shr:1
                    cur = (cur > carry ? cur : carry) & 0xffffu;
                    carry = rl(inc, 63) > carry ? rl(inc, 63) : carry;
#pragma unroll
                    for (int i = 0; i < 16; i++) {
                        cur = (bw >> i) & 1u ? (dv[i >> 1] >> (16 * (i & 1))) & 0xffffu : cur;
                        const uint32_t p = p0 + i;
                        sp[i] = p < lim && cur ? p - cur : p;
                    }
#else
                    const uint32_t cnt = (uint32_t)__builtin_popcount(bw);
                    const uint32_t incl = wave_incl_scan_dpp(cnt);
                    const uint32_t base = before + incl - cnt; // record starts before p0
                    before += rl(incl, 63);
#pragma unroll
                    for (int i = 0; i < 16; i++) {
                        const uint32_t pr = base + (uint32_t)__builtin_popcount(bw & ((2u << i) - 1));
                        sp[i] = recd[pr ? pr - 1 : 0u];
                    }
#pragma unroll
                    for (int i = 0; i < 16; i++) {
                        const uint32_t p = p0 + i;
                        sp[i] = p < lim && sp[i] ? p - sp[i] : p;
                    }
#endif
                    // (a lane reads and then rewrites only its own 16 positions of src: no sync needed here)
                    uint32_t sw[8];
#pragma unroll
                    for (int i = 0; i < 8; i++) sw[i] = sp[2 * i] | sp[2 * i + 1] << 16;
                    *(PMC_LDS rec_v4u *)(srcv + p0) = rec_v4u{sw[0], sw[1], sw[2], sw[3]};
                    *(PMC_LDS rec_v4u *)(srcv + p0 + 8) = rec_v4u{sw[4], sw[5], sw[6], sw[7]};
                    wave_sync();
                    // pointer jumping: every position ends at the literal it copies (a literal,
                    // and a position past its member's end, points at itself)
                    for (;;) {
                        uint32_t t[16];
#pragma unroll
                        for (int i = 0; i < 16; i++) t[i] = srcv[sp[i]];
                        bool ch = false;
#pragma unroll
                        for (int i = 0; i < 16; i++) {
                            ch |= t[i] != sp[i];
                            sp[i] = t[i];
                        }
                        if (!ballot(ch)) break;
#ifdef PMC_STAMPS
                        n_jump++;
#endif
#pragma unroll
                        for (int i = 0; i < 8; i++) sw[i] = sp[2 * i] | sp[2 * i + 1] << 16;
                        *(PMC_LDS rec_v4u *)(srcv + p0) = rec_v4u{sw[0], sw[1], sw[2], sw[3]};
                        *(PMC_LDS rec_v4u *)(srcv + p0 + 8) = rec_v4u{sw[4], sw[5], sw[6], sw[7]};
                        wave_sync();
                    }
                    uint32_t gb[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int i = 0; i < 16; i++) gb[i >> 2] |= (uint32_t)ob[sp[i]] << (8 * (i & 3));
                    wave_sync();
                    *(PMC_LDS rec_v4u *)(ob + p0) = rec_v4u{gb[0], gb[1], gb[2], gb[3]};
                    wave_sync();
                }
#ifdef PMC_STAMPS
                n_recs += R;
#pragma unroll
                for (int g = 0; g < G; g++) n_mem += cm[g] >= 0;
#endif
#pragma unroll
                for (int g = 0; g < G; g++) {
                    pm[g] = cm[g];
                    p_osz[g] = osz[g];
                    p_dst[g] = cm[g] >= 0 ? rl64(dptr, cm[g]) : 0u;
                    p_v[g] = cm[g] >= 0 ? rl64(v, cm[g]) : 0u;
                }
                buf ^= 1;
            }
            flush_prev();
        };
        const uint64_t small = todo & ballot(pos <= 256);
        run_passes(std::integral_constant<int, 4>{}, small);
        run_passes(std::integral_constant<int, 1>{}, todo & ~small);
        wave_sync();
#ifdef PMC_STAMPS
        uint64_t t3 = __builtin_amdgcn_s_memtime();
        if (threadIdx.x == 0 && a.dbg) {
            atomicAdd((unsigned long long *)&a.dbg[3], (unsigned long long)n_it);
            atomicAdd((unsigned long long *)&a.dbg[4], (unsigned long long)n_act);
            atomicAdd((unsigned long long *)&a.dbg[5], (unsigned long long)(t1 - t0));
            atomicAdd((unsigned long long *)&a.dbg[6], (unsigned long long)(t2 - t1));
            atomicAdd((unsigned long long *)&a.dbg[7], (unsigned long long)(t2b - t2));
            atomicAdd((unsigned long long *)&a.dbg[8], (unsigned long long)(t3 - t2b));
            atomicAdd((unsigned long long *)&a.dbg[9], (unsigned long long)n_jump);
            atomicAdd((unsigned long long *)&a.dbg[10], (unsigned long long)n_recs);
            atomicAdd((unsigned long long *)&a.dbg[11], (unsigned long long)n_mem);
        }
#endif
    }
}

template __global__ void inflate_rec_kernel<1024>(InflateArgs);
template __global__ void inflate_rec_kernel<kRecOutMax>(InflateArgs);

} // namespace pmc
