// pmc_inflate_lane.hip -- gzip member decoding with one LANE per member.
//
// DEFLATE decoding is a chain of data-dependent steps (each symbol's length decides where
// the next one starts), so a wave spends its scalar unit on one member at a time in
// inflate_kernel.  Here each of a wave's 64 lanes decodes its own member, the way a CPU
// core runs zlib's inflate (reference: /root/reference/src/compressor/gzip_compressor.cpp:
// 52-111, zlib 1.2.11 inflate.c / inftrees.c):
//   * bits come from the member in HBM through a 64-bit per-lane bit buffer;
//   * a dynamic block's codes are canonical-decoded: the left-justified code's length is
//     the count of per-length limits it reaches (15 compares against registers), the
//     symbol one LDS load from the lane's (length, symbol)-sorted list (conflict-free
//     columns: entry i of lane l at i * 64 + l).  The code-length code is decoded twice
//     (count, then place), so no per-symbol length array is kept;
//   * fixed blocks decode in closed form, stored blocks are copied;
//   * output goes straight to dst; a match reads its source back from dst 8 bytes at a
//     time (distance >= 8) or replicates its period from registers (distance < 8).
// The fast path only decodes well-formed members.  Anything it does not handle exactly
// -- gzip header flags, incomplete or over-subscribed codes, lists longer than its LDS
// columns, bad symbols or distances, truncation, capacity, length/CRC mismatches -- marks
// the member kInflateRetry, and inflate_kernel (wave per member, zlib's verdict order)
// redoes it.  The CRC-32 is checked by inflate_verify_kernel (wave-parallel) afterwards.
#include <hip/hip_runtime.h>

#include "pmc_device.hpp"
#include "pmc_kernels.hpp"

namespace pmc {

constexpr int kLaneLitCap = 96, kLaneDistCap = 30;
// the wide instance's lit/len lists: members declined only because their lit/len code uses more than 96
// symbols (a third of 30 KB JSON members, up to ~110) take a second pass at 3 waves per CU
constexpr int kLaneWideLit = 128;
// per-lane LDS columns (u16 words, entry i of lane l at word i * 64 + l).  Decode-time:
// symbol lists and bases.  Build-time scratch (counts / offsets, code-length code) lives in
// the output ring's bytes, which are only written once decoding starts.
// (bases: one entry per code length 1..15)
template <int LIT, int DIST>
struct LaneCols {
    static constexpr int kLit = LIT, kDist = DIST;
    static constexpr int kColLit = 0, kColDist = LIT, kColBaseL = LIT + DIST, kColBaseD = kColBaseL + 15;
    static constexpr int kColWords = kColBaseD + 15;
    // lane_lengths' pass 1: symbol `sym` of the lit/len (lit) or distance list goes to entry `at`
    __device__ static __forceinline__ void place(PMC_LDS uint16_t *col, bool lit, uint32_t at, uint32_t sym, uint32_t,
                                                 PMC_LDS const uint8_t *) {
        col[((lit ? kColLit : kColDist) + at) * 64] = (uint16_t)sym;
    }
};
typedef LaneCols<kLaneLitCap, kLaneDistCap> LaneColsL; // the lane kernel's lists
constexpr int kColLit = LaneColsL::kColLit, kColDist = LaneColsL::kColDist, kColBaseL = LaneColsL::kColBaseL;
constexpr int kColBaseD = LaneColsL::kColBaseD, kColWords = LaneColsL::kColWords;
// build columns (u8 entries, entry i of lane l at byte i * 64 + l): counts / offsets per code length
// of the lit/len and distance codes (a count above the lists' capacity declines anyway, so 8 bits
// saturating suffice), the code-length code's bases (int8) and sorted symbols (+19)
constexpr int kBColCntL = 0, kBColCntD = 16, kBColBaseC = 32, kBColCl = 40;
#ifndef PMC_LANE_WIN
#define PMC_LANE_WIN 16
#endif
// input window per lane (dwords, refilled by halves).  The kernel is latency-bound (its
// lanes wait on LDS and L2 most of the time), so LDS per wave sets its speed through occupancy.
constexpr uint32_t kWinDw = PMC_LANE_WIN, kWinHalf = kWinDw / 2;
#ifndef PMC_LANE_RING
#define PMC_LANE_RING 256
#endif
// output ring per lane (bytes; flushed by halves); matches reaching further back than
// kRing - 16 read dst (L2).  (128 fits five waves per CU but measured slower than 256 at four.)
constexpr uint32_t kRing = PMC_LANE_RING, kFlush = kRing / 2;
// the lane kernel's LDS per 64-lane block for lit/len lists of LIT entries: columns | rings | windows
// (MB, the multi-block pass: the build columns get their own region after the windows, because a
// block's tables are built while the other lanes' rings hold live output)
template <int LIT, bool MB = false>
struct LaneLayout {
    typedef LaneCols<LIT, kLaneDistCap> Cols;
    static constexpr uint32_t kRingOff = (uint32_t)Cols::kColWords * 64 * 2; // output rings (LaneOut)
    static constexpr uint32_t kWinOff = kRingOff + kRing / 4 * 64 * 4;       // input windows (LaneWin)
    static constexpr uint32_t kBColOff = kWinOff + kWinDw * 64 * 4;          // MB: build columns
    static constexpr uint32_t kLds = kBColOff + (MB ? (kBColCl + 19) * 64 : 0);
};
constexpr uint32_t kLaneLdsBytes = LaneLayout<kLaneLitCap>::kLds;
constexpr uint32_t kLaneWideLdsBytes = LaneLayout<kLaneWideLit>::kLds;
constexpr uint32_t kLaneMultiLdsBytes = LaneLayout<kLaneWideLit, true>::kLds;
static_assert((kBColCl + 19) * 64 <= kRing * 64, "build columns live in the output rings");

// 16-byte load through a global (not flat) pointer: flat loads also count against lgkmcnt,
// so every LDS wait would wait for them too
__device__ __forceinline__ uint4 gload16(PMC_GLB const uint4 *p) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u v = *(PMC_GLB const v4u *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
struct LaneIn {
    const uint8_t *p;
    uint32_t len;       // member bytes
    PMC_GLB const uint4 *blk; // aligned block base (p rounded down to 16); global, not flat
    uint32_t bi;        // index of the block in `cur`
    uint4 cur, nxt;     // block bi and bi + 1
    uint32_t wi;        // next dword of `cur` to move into buf
    uint64_t buf;       // unread bits, LSB first
    uint32_t n;         // bits in buf
    uint64_t consumed0; // stream bit offset of buf bit 0 when bi/wi were set
    __device__ uint32_t byte_at(uint32_t i) const { return i < len ? (uint32_t)p[i] : 0u; }
    // block k of the stream, or zeros past the member's last block (never touches its page)
    __device__ uint4 block(uint32_t k) const {
        return (uint64_t)k * 16 < ((uintptr_t)p & 15) + (uint64_t)len ? gload16(blk + k) : make_uint4(0, 0, 0, 0);
    }
    __device__ void refill() {
        if (n <= 32) {
            const uint32_t w = wi == 0 ? cur.x : wi == 1 ? cur.y : wi == 2 ? cur.z : cur.w;
            buf |= (uint64_t)w << n;
            n += 32;
            if (++wi == 4) {
                wi = 0;
                bi++;
                cur = nxt;
                nxt = block(bi + 1);
            }
        }
    }
    __device__ uint32_t peek(uint32_t k) const { return (uint32_t)buf & ((1u << k) - 1); }
    __device__ void drop(uint32_t k) {
        buf >>= k;
        n -= k;
    }
    __device__ uint32_t bits(uint32_t k) { // k <= 16
        refill();
        const uint32_t v = peek(k);
        drop(k);
        return v;
    }
    // bits consumed from the member start
    __device__ uint64_t bitpos() const {
        const uint64_t head = (uint64_t)((uintptr_t)p & 15) * 8;
        return ((uint64_t)bi * 16 + (uint64_t)wi * 4) * 8 - n - head;
    }
    __device__ void seek(uint64_t bp) { // restart at member bit bp
        const uint64_t a = bp + (uint64_t)((uintptr_t)p & 15) * 8; // bit offset from blk
        bi = (uint32_t)(a >> 7);
        wi = (uint32_t)((a >> 5) & 3);
        cur = block(bi);
        nxt = block(bi + 1);
        buf = 0;
        n = 0;
        refill();
        drop((uint32_t)(a & 31));
    }
};

// Bit reader of the decode loop: the next kWinDw dwords of the member sit in an LDS window
// (column layout, stream dword j at slot j % kWinDw).  Windows advance by half for every
// lane that can at the same time (wave-synchronous refill), so the wave waits on global
// loads a few times per member instead of whenever any one lane's buffer runs low.
struct LaneWin {
    PMC_LDS uint32_t *w; // slot s at w[s * 64]
    PMC_GLB const uint4 *blk; // member rounded down to 16 bytes
    uint32_t nblk;       // blocks holding member bytes
    uint32_t head;       // member start - blk, in bits
    uint32_t wlo;        // first dword held
    uint32_t nd;         // next dword to move into buf
    uint64_t buf;
    uint32_t n;
    __device__ uint4 block(uint32_t k) const { return k < nblk ? gload16(blk + k) : make_uint4(0, 0, 0, 0); }
    __device__ void load_half(uint32_t d0) { // dwords d0 .. d0 + kWinHalf - 1 (aligned) into their slots
#pragma unroll
        for (int b = 0; b < (int)kWinHalf / 4; b++) {
            const uint4 x = block(d0 / 4 + b);
            const uint32_t s0 = (d0 + 4 * b) & (kWinDw - 1);
            w[(s0 + 0) * 64] = x.x;
            w[(s0 + 1) * 64] = x.y;
            w[(s0 + 2) * 64] = x.z;
            w[(s0 + 3) * 64] = x.w;
        }
    }
    __device__ void start(const LaneIn &in, uint64_t bp) { // at member bit bp
        blk = in.blk;
        head = (uint32_t)(((uintptr_t)in.p & 15) * 8);
        nblk = (uint32_t)((((uintptr_t)in.p & 15) + in.len + 15) / 16);
        const uint64_t a = bp + head;
        nd = (uint32_t)(a >> 5);
        wlo = nd & ~(kWinHalf - 1);
        load_half(wlo);
        load_half(wlo + kWinHalf);
        buf = 0;
        n = 0;
        refill();
        drop((uint32_t)(a & 31));
    }
    __device__ void refill() {
        if (n <= 32) {
            buf |= (uint64_t)w[(nd & (kWinDw - 1)) * 64] << n;
            n += 32;
            nd++;
        }
    }
    __device__ bool needs() const { return nd + 4 > wlo + kWinDw; }
    __device__ void advance() { // retire the older half of the window if it is consumed
        if (nd >= wlo + kWinHalf) {
            load_half(wlo + kWinDw);
            wlo += kWinHalf;
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

// One canonical code of up to 15-bit lengths: per-length limits in registers, bases and the
// sorted symbol list in the lane's LDS column.
typedef uint16_t lane_u16x2 __attribute__((ext_vector_type(2)));
template <int NL, class BT = int16_t, class ST = uint16_t>
struct LaneCode {
    static_assert(NL % 2 == 1, "the NL - 1 limits are compared two at a time");
    // left-justified (15-bit) ends of the codes of length j + 1, j < NL - 1, two per register
    // (limit 2k in the low half, 2k + 1 in the high half)
    uint32_t limp[(NL - 1) / 2];
    PMC_LDS BT *base;
    PMC_LDS ST *sym;
    // from counts cnt[1..NL] (LDS column); returns false unless the code is complete
    // (every well-formed zlib stream's codes are; other shapes go to the wave kernel)
    template <class CT>
    __device__ bool build(PMC_LDS const CT *cnt) {
        int32_t first = 0, offs = 0, left = 1;
#pragma unroll
        for (int L = 1; L <= NL; L++) {
            const int32_t c = cnt[L * 64];
            base[(L - 1) * 64] = (BT)(offs - first);
            first += c;
            if (L < NL) {
                const uint32_t lim = (uint32_t)first << (15 - L); // <= 1 << 15
                if ((L - 1) & 1) limp[(L - 1) / 2] |= lim << 16;
                else limp[(L - 1) / 2] = lim;
            }
            first <<= 1;
            offs += c;
            left = (left << 1) - c;
        }
        return left == 0;
    }
    // code length of the left-justified 15-bit code x: 1 + the number of limits <= x.  x - lim
    // in 16 bits has bit 15 set exactly when x < lim (both <= 1 << 15), so one packed subtract
    // tests two limits; the sign bits gather into one word and a popcount counts them.
    __device__ uint32_t code_len(uint32_t x) const {
        const uint32_t xx = x | x << 16;
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < (NL - 1) / 2; k++) {
            const lane_u16x2 d = __builtin_bit_cast(lane_u16x2, xx) - __builtin_bit_cast(lane_u16x2, limp[k]);
            acc |= (__builtin_bit_cast(uint32_t, d) >> k) & (0x80008000u >> k);
        }
        return (uint32_t)NL - (uint32_t)__builtin_popcount(acc);
    }
    // symbol at the head of the bit buffer without consuming it; *len = its code length
    template <class R>
    __device__ uint32_t peek_sym(const R &in, uint32_t &len) const {
        const uint32_t x = __builtin_bitreverse32(in.peek(15)) >> 17;
        const uint32_t L = code_len(x);
        const int idx = (int)base[(L - 1) * 64] + (int)(x >> (15 - L));
        len = L;
        return sym[idx * 64];
    }
    template <class R>
    __device__ uint32_t decode(R &in) const {
        const uint32_t x = __builtin_bitreverse32(in.peek(15)) >> 17;
        const uint32_t L = code_len(x);
        const int idx = (int)base[(L - 1) * 64] + (int)(x >> (15 - L));
        in.drop(L);
        return sym[idx * 64];
    }
};

template <class R>
__device__ __forceinline__ uint32_t fixed_peek(const R &in, uint32_t &len) {
    const uint32_t x9 = __builtin_bitreverse32(in.peek(9)) >> 23;
    uint32_t sym;
    if ((x9 >> 2) < 24) {
        sym = 256 + (x9 >> 2);
        len = 7;
    } else if ((x9 >> 1) < 192) {
        sym = (x9 >> 1) - 48;
        len = 8;
    } else if ((x9 >> 1) < 200) {
        sym = 280 + (x9 >> 1) - 192;
        len = 8;
    } else {
        sym = 144 + x9 - 400;
        len = 9;
    }
    return sym;
}
template <class R>
__device__ __forceinline__ uint32_t fixed_lit(R &in) {
    const uint32_t x9 = __builtin_bitreverse32(in.peek(9)) >> 23;
    uint32_t sym, len;
    if ((x9 >> 2) < 24) {
        sym = 256 + (x9 >> 2);
        len = 7;
    } else if ((x9 >> 1) < 192) {
        sym = (x9 >> 1) - 48;
        len = 8;
    } else if ((x9 >> 1) < 200) {
        sym = 280 + (x9 >> 1) - 192;
        len = 8;
    } else {
        sym = 144 + x9 - 400;
        len = 9;
    }
    in.drop(len);
    return sym;
}

// Code lengths of a dynamic block through the code-length code; pass 0 counts them
// (cnt columns), pass 1 places every symbol into its list (cnt columns hold offsets).
// Returns false on any malformed sequence.
typedef LaneCode<7, int8_t, uint8_t> LaneClc; // the code-length code, in the byte build columns
template <class C>
__device__ bool lane_lengths(LaneIn &in, const LaneClc &clc, uint32_t nlen, uint32_t nlit, PMC_LDS uint16_t *col,
                             PMC_LDS uint8_t *bcol, int pass, bool &eob_ok) {
    uint32_t k = 0, prev = 0;
    while (k < nlen) {
        in.refill();
        const uint32_t s = clc.decode(in);
        uint32_t val, rep;
        if (s < 16) {
            val = s;
            rep = 1;
        } else if (s == 16) {
            if (k == 0) return false;
            val = prev;
            rep = 3 + in.bits(2);
        } else if (s == 17) {
            val = 0;
            rep = 3 + in.bits(3);
        } else {
            val = 0;
            rep = 11 + in.bits(7);
        }
        if (k + rep > nlen) return false;
        if (val) {
            for (uint32_t r = 0; r < rep; r++, k++) {
                const bool lit = k < nlit;
                PMC_LDS uint8_t *c = bcol + (lit ? kBColCntL : kBColCntD) * 64 + val * 64;
                if (pass == 0) {
                    const uint32_t x = *c;
                    *c = (uint8_t)(x < 255 ? x + 1 : 255u);
                    if (k == 256) eob_ok = true;
                } else {
                    const uint32_t at = *c;
                    *c = (uint8_t)(at + 1);
                    C::place(col, lit, at, lit ? k : k - nlit, val, bcol);
                }
            }
        } else {
            k += rep;
        }
        prev = val;
    }
    return true;
}

// A block's header (after its BFINAL bit) and code tables, `in` at the BTYPE bits; false = decline.
template <class C, class LC, class DC>
__device__ __forceinline__ bool lane_block(LaneIn &in, PMC_LDS uint16_t *col, PMC_LDS uint8_t *bcol, LC &lit,
                           DC &dist, bool &fixed, bool *over, int wide_lit, int wide_dist) {
    const uint32_t btype = in.bits(2);
    if (btype == 0 || btype == 3) return false;
    fixed = btype == 1;
    if (fixed) return true;
    const uint32_t nlit = in.bits(5) + 257, ndist = in.bits(5) + 1, ncl = in.bits(4) + 4;
    if (nlit > 286 || ndist > 30) return false;
    // code-length code: lengths (3 bits each, permuted order), counts, list
    uint64_t cll = 0;
    for (uint32_t k = 0; k < ncl; k++) cll |= (uint64_t)in.bits(3) << (3 * bl_order_cf((int)k));
    for (int L = 0; L < 16; L++) bcol[(kBColCntL + L) * 64] = 0;
    for (uint32_t sy = 0; sy < 19; sy++) {
        const uint32_t L = (uint32_t)(cll >> (3 * sy)) & 7;
        if (L) bcol[(kBColCntL + L) * 64] = (uint8_t)(bcol[(kBColCntL + L) * 64] + 1);
    }
    LaneClc clc;
    clc.base = (PMC_LDS int8_t *)(bcol + kBColBaseC * 64);
    clc.sym = bcol + kBColCl * 64;
    if (!clc.build(bcol + kBColCntL * 64)) return false;
    {
        uint32_t offs = 0;
        for (int L = 1; L < 8; L++) {
            const uint32_t c = bcol[(kBColCntL + L) * 64];
            bcol[(kBColCntL + L) * 64] = (uint8_t)offs;
            offs += c;
        }
        for (uint32_t sy = 0; sy < 19; sy++) {
            const uint32_t L = (uint32_t)(cll >> (3 * sy)) & 7;
            if (L) {
                const uint32_t at = bcol[(kBColCntL + L) * 64];
                bcol[(kBColCntL + L) * 64] = (uint8_t)(at + 1);
                clc.sym[at * 64] = (uint16_t)sy;
            }
        }
    }
    // pass 0: counts of the literal/length and distance codes
    for (int L = 0; L < 16; L++) {
        bcol[(kBColCntL + L) * 64] = 0;
        bcol[(kBColCntD + L) * 64] = 0;
    }
    const uint64_t lens_at = in.bitpos();
    bool eob_ok = false;
    if (!lane_lengths<C>(in, clc, nlit + ndist, nlit, col, bcol, 0, eob_ok) || !eob_ok) return false;
    const uint64_t data_at = in.bitpos();
    uint32_t nl = 0, nd = 0;
    for (int L = 1; L < 16; L++) {
        nl += bcol[(kBColCntL + L) * 64];
        nd += bcol[(kBColCntD + L) * 64];
    }
    if (nl > (uint32_t)C::kLit || nd > (uint32_t)C::kDist) {
        if (over) *over = nl <= (uint32_t)wide_lit && nd <= (uint32_t)wide_dist;
        return false;
    }
    if (!lit.build(bcol + kBColCntL * 64) || !dist.build(bcol + kBColCntD * 64)) return false;
    {
        uint32_t ol = 0, od = 0;
        for (int L = 1; L < 16; L++) {
            const uint32_t cl = bcol[(kBColCntL + L) * 64], cd = bcol[(kBColCntD + L) * 64];
            bcol[(kBColCntL + L) * 64] = (uint8_t)ol;
            bcol[(kBColCntD + L) * 64] = (uint8_t)od;
            ol += cl;
            od += cd;
        }
    }
    in.seek(lens_at);
    lane_lengths<C>(in, clc, nlit + ndist, nlit, col, bcol, 1, eob_ok);
    in.seek(data_at);
    return true;
}

// Header and block header of a single-block fixed/dynamic member, code tables built;
// false = decline (stored or multi-block members, header flags, malformed codes ...).  *over
// (if given) is set when the only reason is C's list capacity: the lane kernel's lists hold it;
// *multi (if given) when the member's first block is not its last (the multi-block pass takes it).
// (wide_lit / wide_dist: the capacity *over tests against)
template <class C, class LC, class DC>
__device__ __forceinline__ bool lane_prepare(LaneIn &in, PMC_LDS uint16_t *col, PMC_LDS uint8_t *bcol, LC &lit,
                             DC &dist, bool &fixed, bool *over = nullptr, int wide_lit = kLaneLitCap,
                             int wide_dist = kLaneDistCap, bool *multi = nullptr, uint32_t *last = nullptr) {
    if (in.len < 18) return false;
    if (in.byte_at(0) != 0x1f || in.byte_at(1) != 0x8b || in.byte_at(2) != 8 || in.byte_at(3) != 0) return false;
    in.seek(80);
    const uint32_t bfinal = in.bits(1);
    if (last) *last = bfinal;
    if (!bfinal && !last) {
        if (multi) *multi = true;
        return false;
    }
    return lane_block<C, LC, DC>(in, col, bcol, lit, dist, fixed, over, wide_lit, wide_dist);
}

// Output of one lane: the last kRing bytes live in an LDS ring (column layout, dword k of
// the ring at word k * 64 of the lane's column) aligned so that ring dwords map onto dst
// dwords; complete dwords go to dst in bursts of >= kFlush bytes.  Keeping the byte-level
// traffic in LDS keeps vmcnt free of thousands of byte stores (on gfx9 loads and stores
// share it, so every later load would wait for them).
struct LaneOut {
    PMC_LDS uint8_t *rb;  // byte view of the lane's ring column (byte q at (q >> 2) * 256 + (q & 3))
    PMC_LDS uint32_t *rw; // dword view (dword k at k * 64)
    PMC_GLB uint32_t *dw; // dst rounded down to 4 bytes (global, not flat: see gload16)
    PMC_GLB uint8_t *dst;
    uint32_t a0;          // dst & 3
    uint32_t pos, flushed; // bytes produced / bytes in dst
    __device__ void put(uint32_t p, uint32_t b) {
        const uint32_t q = (p + a0) & (kRing - 1);
        rb[(q >> 2) * 256 + (q & 3)] = (uint8_t)b;
    }
    __device__ uint32_t ringw(uint32_t k) const { return rw[(k & (kRing / 4 - 1)) * 64]; }
    // 8 bytes starting at output position src (all of them already produced)
    __device__ uint64_t get8(uint32_t src, bool from_ring) const {
        const uint32_t q = src + a0, k = q >> 2, sh = q & 3;
        uint32_t w0, w1, w2;
        if (from_ring) {
            w0 = ringw(k);
            w1 = ringw(k + 1);
            w2 = ringw(k + 2);
        } else {
            w0 = dw[k];
            w1 = dw[k + 1];
            w2 = dw[k + 2];
        }
        return (uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32 | __builtin_amdgcn_alignbyte(w1, w0, sh);
    }
    // write every complete dword below position `upto` (all bytes when `last`)
    __device__ void flush(uint32_t upto, bool last) {
        if (flushed == 0 && a0 && upto > 0) { // head dword: only the member's own bytes
            const uint32_t h = 4 - a0 < upto ? 4 - a0 : upto;
            for (uint32_t j = 0; j < h; j++) dst[j] = rb[((a0 + j) & (kRing - 1)) / 4 * 256 + ((a0 + j) & 3)];
            flushed = h;
        }
        const uint32_t k1 = (upto + a0) >> 2;
        for (uint32_t k = (flushed + a0) >> 2; k < k1; k++) dw[k] = ringw(k);
        if (k1 * 4 > flushed + a0) flushed = k1 * 4 - a0;
        if (last) {
            for (uint32_t p = flushed; p < upto; p++) {
                const uint32_t q = (p + a0) & (kRing - 1);
                dst[p] = rb[(q >> 2) * 256 + (q & 3)];
            }
            flushed = upto;
        }
    }
};

// LIT = kLaneLitCap: every member (a.big_only: those the record kernel marked kInflateBig); a member
// declined only for its lit/len list length is marked kInflateWide, one of several blocks kInflateMulti
// (when a.multi_pass).  LIT = kLaneWideLit: the kInflateWide members only.  MB: the kInflateMulti members,
// block after block (a block boundary re-reads the header and rebuilds the tables from the decode
// window's bit position; values above 16383 bytes, whose members zlib splits every 16383 symbols).
template <int LIT, bool MB>
__global__ void __launch_bounds__(64) inflate_lane_kernel(InflateArgs a) {
    typedef LaneLayout<LIT, MB> LL;
    typedef typename LL::Cols Cols;
    constexpr bool kWide = LIT != kLaneLitCap && !MB;
    extern __shared__ __attribute__((aligned(16))) uint16_t lcol[];
    PMC_LDS uint16_t *col = to_lds<uint16_t>(lcol + threadIdx.x);
    PMC_LDS uint32_t *ring = to_lds<uint32_t>((uint8_t *)lcol + LL::kRingOff) + threadIdx.x;
    PMC_LDS uint8_t *bcol = to_lds<uint8_t>((uint8_t *)lcol + (MB ? LL::kBColOff : LL::kRingOff) + threadIdx.x);
    PMC_LDS uint32_t *winw = to_lds<uint32_t>((uint8_t *)lcol + LL::kWinOff) + threadIdx.x;
    // after the record kernel (a.big_list): only the members it left here -- not a pass over all n members
    // that reads each one's rc and length to skip it (random 4-byte gathers through the visit order)
    const bool listed = a.big_only && a.big_list;
    const uint64_t nv = listed ? (uint64_t)*a.big_count : a.n;
    for (uint64_t vb = (uint64_t)blockIdx.x * 64; vb < nv; vb += (uint64_t)gridDim.x * 64) {
        const uint64_t vi = vb + threadIdx.x;
        const uint64_t v = vi >= nv ? a.n : listed ? (uint64_t)a.big_list[vi] : a.order ? (uint64_t)a.order[vi] : vi;
        const uint32_t in_len = v < a.n ? a.src_len[v] : 0u;
        // st: 0 decoding, 1 end of block reached, 2 declined, 3 no member / empty input, 5 for the wide pass
        uint32_t st = v < a.n ? 0u : 3u;
        if (st == 0 && (MB ? a.rc[v] != kInflateMulti
                           : kWide ? a.rc[v] != kInflateWide : a.big_only && a.rc[v] != kInflateBig))
            st = 3; // not this pass's member (the record kernel's, or decoded by the first lane pass)
        if (st == 0 && in_len == 0) {
            a.rc[v] = PMC_INVALID_INPUT_DEV;
            a.dst_len[v] = 0;
            st = 3;
        }
        if (!ballot(st == 0)) continue; // e.g. the pass over the record kernel's large members
        LaneIn in;
        in.p = st == 0 ? a.src + a.src_off[v] : a.src;
        in.len = st == 0 ? in_len : 0u;
        in.blk = (PMC_GLB const uint4 *)((uintptr_t)in.p & ~(uintptr_t)15);
        LaneCode<15> lit, dist;
        lit.base = (PMC_LDS int16_t *)(col + Cols::kColBaseL * 64);
        lit.sym = col + Cols::kColLit * 64;
        dist.base = (PMC_LDS int16_t *)(col + Cols::kColBaseD * 64);
        dist.sym = col + Cols::kColDist * 64;
        bool fixed = false;
#ifdef PMC_STAMPS
        uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
        bool wide = false;  // declined only for the lit/len list's length: the wide pass takes it
        bool multi = false; // declined only for having several blocks: the multi-block pass takes it
        uint32_t blast = 1; // MB: the current block is the member's last
        if (st == 0 && !lane_prepare<Cols>(in, col, bcol, lit, dist, fixed, &wide, kLaneWideLit, kLaneDistCap, &multi,
                                           MB ? &blast : nullptr))
            st = multi && a.multi_pass ? 7u : kWide || MB || !wide ? 2u : 5u;
#ifdef PMC_STAMPS
        uint64_t t1 = __builtin_amdgcn_s_memtime();
        uint64_t n_it = 0, n_act = 0;
#endif
        LaneWin win;
        win.w = winw;
        win.start(in, st == 0 ? in.bitpos() : 0);
        const uint32_t cap = st == 0 ? a.dst_cap[v] : 0u;
        LaneOut o;
        o.dst = (PMC_GLB uint8_t *)(st == 0 ? a.dst + a.dst_off[v] : a.dst);
        o.a0 = (uint32_t)((uintptr_t)o.dst & 3);
        o.dw = (PMC_GLB uint32_t *)((uintptr_t)o.dst & ~(uintptr_t)3);
        o.rw = ring;
        o.rb = (PMC_LDS uint8_t *)ring;
        o.pos = 0;
        o.flushed = 0;
        uint32_t rem = 0, md = 0; // pending match: bytes left, distance
        // one step per iteration: a symbol, then up to 8 bytes of the current match
        while (ballot(st == 0)) {
#ifdef PMC_STAMPS
            n_it++;
            n_act += __builtin_popcountll(ballot(st == 0));
#endif
            if (ballot(st == 0 && win.needs()))
                if (st == 0) win.advance();
            if (st == 0) {
                if (rem == 0) {
                    win.refill();
                    const uint32_t sy = fixed ? fixed_lit(win) : lit.decode(win);
                    if (sy < 256) {
                        if (o.pos >= cap) {
                            st = 2;
                        } else {
                            o.put(o.pos++, sy);
                            // literals are most of the steps: take the next symbol too when it is
                            // one (the refilled buffer still holds >= 17 bits, a full peek)
                            uint32_t l2;
                            const uint32_t s2 = fixed ? fixed_peek(win, l2) : lit.peek_sym(win, l2);
                            if (s2 < 256 && o.pos < cap) {
                                win.drop(l2);
                                o.put(o.pos++, s2);
                                win.refill();
                                uint32_t l3;
                                const uint32_t s3 = fixed ? fixed_peek(win, l3) : lit.peek_sym(win, l3);
                                if (s3 < 256 && o.pos < cap) {
                                    win.drop(l3);
                                    o.put(o.pos++, s3);
                                }
                            }
                        }
                    } else if (sy == 256) {
                        st = MB && !blast ? 6u : 1u;
                    } else if (sy > 285) {
                        st = 2;
                    } else {
                        // length / distance bases and extra bits in closed form (RFC 1951 3.2.5)
                        const uint32_t li = sy - 257;
                        const uint32_t lx = li < 8 || li == 28 ? 0u : (li - 4) >> 2;
                        const uint32_t lb = li < 8 ? li + 3 : li == 28 ? 258u : ((4 + (li & 3)) << lx) + 3;
                        const uint32_t len = lb + win.bits(lx);
                        win.refill();
                        const uint32_t ds = fixed ? __builtin_bitreverse32(win.peek(5)) >> 27 : dist.decode(win);
                        if (fixed) win.drop(5);
                        const uint32_t dx = ds < 4 ? 0u : (ds >> 1) - 1;
                        const uint32_t db = ds < 4 ? ds + 1 : ((2 + (ds & 1)) << dx) + 1;
                        const uint32_t d = db + win.bits(dx < 14 ? dx : 0u);
                        if (ds > 29 || d > o.pos || o.pos + len > cap) {
                            st = 2;
                        } else if (d < 8) { // period d: replicate it, later chunks copy from d' >= 8 back
                            uint64_t pat = o.get8(o.pos - d, true) & ((1ull << (8 * d)) - 1);
                            for (uint32_t w = d; w < 8; w <<= 1) pat |= pat << (8 * w);
                            const uint32_t m = len < 8 ? len : 8;
#pragma unroll
                            for (uint32_t j = 0; j < 8; j++)
                                if (j < m) o.put(o.pos + j, (uint32_t)(pat >> (8 * j)));
                            o.pos += m;
                            rem = len - m;
                            md = d * ((8 + d - 1) / d);
                        } else {
                            rem = len;
                            md = d;
                        }
                    }
                }
                if (st == 0 && rem) {
                    const uint32_t m = rem < 8 ? rem : 8;
                    const uint64_t x = o.get8(o.pos - md, md <= kRing - 16);
#pragma unroll
                    for (uint32_t j = 0; j < 8; j++)
                        if (j < m) o.put(o.pos + j, (uint32_t)(x >> (8 * j)));
                    o.pos += m;
                    rem -= m;
                }
                if (MB && st == 6) { // end of a block that is not the last: the next one's header and tables
                    in.seek(win.bitpos());
                    blast = in.bits(1);
                    bool ov = false;
                    if (lane_block<Cols>(in, col, bcol, lit, dist, fixed, &ov, kLaneWideLit, kLaneDistCap)) {
                        win.start(in, in.bitpos());
                        st = 0;
                    } else {
                        st = 2; // stored blocks, longer lists, malformed codes: the wave kernel
                    }
                }
            }
            // wave-synchronous flush: every lane writes its complete dwords at once, so the
            // wave waits for stores a few times per member instead of once per lane flush
            if (ballot(st == 0 && o.pos - o.flushed >= kFlush))
                if (st == 0) o.flush(o.pos, false);
        }
#ifdef PMC_STAMPS
        uint64_t t2 = __builtin_amdgcn_s_memtime();
#endif
        if (st == 1) {
            if (win.bitpos() > (uint64_t)in.len * 8) st = 2;
        }
        if (st == 1) {
            const uint32_t t = (uint32_t)((win.bitpos() + 7) >> 3);
            if (t + 8 > in.len) {
                st = 2;
            } else {
                const uint32_t isz = in.byte_at(t + 4) | in.byte_at(t + 5) << 8 | in.byte_at(t + 6) << 16 |
                                     in.byte_at(t + 7) << 24;
                if (isz != o.pos) {
                    st = 2;
                } else {
                    o.flush(o.pos, true);
                    a.crc_expect[v] =
                        in.byte_at(t) | in.byte_at(t + 1) << 8 | in.byte_at(t + 2) << 16 | in.byte_at(t + 3) << 24;
                    a.dst_len[v] = o.pos;
                    a.rc[v] = 0;
                }
            }
        }
        if (st == 2) a.rc[v] = kInflateRetry;
        if (st == 5) a.rc[v] = kInflateWide;
        if (st == 7) a.rc[v] = kInflateMulti;
#ifdef PMC_STAMPS
        // dbg slots 3..7 (the wave kernels' 0..5 see only retried members): wave iterations
        // of the decode loop, active lane-iterations, cycles in prepare, decode, finish
        uint64_t t3 = __builtin_amdgcn_s_memtime();
        if (threadIdx.x == 0 && a.dbg) {
            atomicAdd((unsigned long long *)&a.dbg[3], (unsigned long long)n_it);
            atomicAdd((unsigned long long *)&a.dbg[4], (unsigned long long)n_act);
            atomicAdd((unsigned long long *)&a.dbg[5], (unsigned long long)(t1 - t0));
            atomicAdd((unsigned long long *)&a.dbg[6], (unsigned long long)(t2 - t1));
            atomicAdd((unsigned long long *)&a.dbg[7], (unsigned long long)(t3 - t2));
        }
#endif
    }
}

template __global__ void inflate_lane_kernel<kLaneLitCap, false>(InflateArgs);
template __global__ void inflate_lane_kernel<kLaneWideLit, false>(InflateArgs);
template __global__ void inflate_lane_kernel<kLaneWideLit, true>(InflateArgs);

// ---- visit order: counting sort of member indices by compressed length ------------------
// Blocks take contiguous slices; bins are per-block LDS counts, one global add per used bin.
__device__ __forceinline__ uint32_t order_bin(uint32_t len) { return len < kOrderBins ? len : kOrderBins - 1; }
__global__ void __launch_bounds__(256) order_hist_kernel(const uint32_t *src_len, uint64_t n, uint32_t *hist) {
    __shared__ uint32_t h[kOrderBins];
    for (uint32_t k = threadIdx.x; k < kOrderBins; k += blockDim.x) h[k] = 0;
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x, b0 = (uint64_t)blockIdx.x * per;
    const uint64_t b1 = b0 + per < n ? b0 + per : n;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) atomicAdd(&h[order_bin(src_len[i])], 1u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kOrderBins; k += blockDim.x)
        if (h[k]) atomicAdd(&hist[k], h[k]);
}
// exclusive scan of the bins in place (one block of 1024 threads, two bins each)
__global__ void __launch_bounds__(1024) order_scan_kernel(uint32_t *hist) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x, a = hist[2 * t], b = hist[2 * t + 1];
    part[t] = a + b;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint32_t v = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const uint32_t ex = part[t] - (a + b);
    hist[2 * t] = ex;
    hist[2 * t + 1] = ex + a;
}
__global__ void __launch_bounds__(256) order_scatter_kernel(const uint32_t *src_len, uint64_t n, uint32_t *cursor,
                                                            uint32_t *order) {
    __shared__ uint32_t h[kOrderBins];
    for (uint32_t k = threadIdx.x; k < kOrderBins; k += blockDim.x) h[k] = 0;
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x, b0 = (uint64_t)blockIdx.x * per;
    const uint64_t b1 = b0 + per < n ? b0 + per : n;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) atomicAdd(&h[order_bin(src_len[i])], 1u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kOrderBins; k += blockDim.x)
        if (h[k]) h[k] = atomicAdd(&cursor[k], h[k]); // this block's range in bin k
    __syncthreads();
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) order[atomicAdd(&h[order_bin(src_len[i])], 1u)] = (uint32_t)i;
}

// CRC-32 of the members g + j (j in `todo`) of a batch of byte strings, returned in lane j.
// Members of up to kCrcQuarterMax bytes go four to a wave: quarter q (16 lanes) takes the
// q-th member of the round, lane s of it the s-th 64-byte piece counted from the member's
// END, front-padded with zero bytes.  A piece runs slicing-by-8 from register 0 (17 dwords from
// five 16-byte loads, v_alignbyte for the member's byte alignment); the quarter then folds its pieces in
// four DPP row_shl levels, shifting the earlier half past 64*2^k bytes with a 4x256 table,
// and the init value's share 0xFFFFFFFF x^(8 len) comes from c_crc_ones (zeros in front of
// a register-0 CRC leave it unchanged, so the padding is free).  Longer members take the
// whole wave (wave_crc32).  `mylen` is lane j's member length.
__device__ __forceinline__ uint32_t crc_piece64(const uint8_t *buf, uint64_t off, uint32_t len, uint32_t s,
                                                PMC_LDS const uint32_t *s8) {
    const int64_t pend = (int64_t)len - (int64_t)kCrcPiece * s, pbeg = pend - kCrcPiece;
    const uint64_t base = (uint64_t)buf + off;
    const uint64_t ab = (uint64_t)((int64_t)base + pbeg) & ~(uint64_t)3;
    const uint32_t sh = (uint32_t)(base + (uint64_t)pend) & 3;
    const int32_t lead = pbeg < 0 ? (int32_t)-pbeg : 0;
    // the piece's 17 dwords from five 16-byte loads (one pass of the address unit per 16 bytes, not
    // per dword: with 64 lanes on 32 lines per instruction, 17 dword loads had made this kernel
    // L1-bound), each block clamped to the member's first / last 16-byte block (a block that holds
    // none of the member's bytes only feeds bytes the lead mask or the alignment drop)
    const uint64_t a16 = ab & ~(uint64_t)15, lo16 = base & ~(uint64_t)15, hi16 = (base + len - 1) & ~(uint64_t)15;
    const uint32_t o = (uint32_t)(ab - a16) >> 2;
    uint32_t d[20];
#pragma unroll
    for (int b = 0; b < 5; b++) {
        uint64_t p = a16 + 16 * b;
        p = p < lo16 ? lo16 : p;
        p = p > hi16 ? hi16 : p;
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const v4u v = *(const PMC_GLB v4u *)p;
        d[4 * b] = v.x;
        d[4 * b + 1] = v.y;
        d[4 * b + 2] = v.z;
        d[4 * b + 3] = v.w;
    }
    uint32_t w[17];
#pragma unroll
    for (int i = 0; i < 17; i++) w[i] = o == 0 ? d[i] : o == 1 ? d[i + 1] : o == 2 ? d[i + 2] : d[i + 3];
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint32_t x[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int i = 2 * k + h;
            uint32_t v = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
            const int32_t r = lead - 4 * i;
            v = r <= 0 ? v : (r >= 4 ? 0u : v & (0xFFFFFFFFu << (8 * r)));
            x[h] = v;
        }
        const uint32_t a0 = x[0] ^ c, a1 = x[1];
        c = s8[7 * 256 + (a0 & 0xff)] ^ s8[6 * 256 + ((a0 >> 8) & 0xff)] ^ s8[5 * 256 + ((a0 >> 16) & 0xff)] ^
            s8[4 * 256 + (a0 >> 24)] ^ s8[3 * 256 + (a1 & 0xff)] ^ s8[2 * 256 + ((a1 >> 8) & 0xff)] ^
            s8[1 * 256 + ((a1 >> 16) & 0xff)] ^ s8[a1 >> 24];
    }
    return c;
}

template <int K>
__device__ __forceinline__ uint32_t crc_fold_level(uint32_t v, PMC_LDS const uint32_t *zp) {
    const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + (1 << K), 0xf, 0xf, false);
    PMC_LDS const uint32_t *z = zp + K * 1024;
    return v ^ z[t & 0xff] ^ z[256 + ((t >> 8) & 0xff)] ^ z[512 + ((t >> 16) & 0xff)] ^ z[768 + (t >> 24)];
}

__device__ uint32_t wave_crc32_members(const uint8_t *buf, const uint64_t *off, uint64_t g, uint64_t todo,
                                       uint32_t mylen, PMC_LDS const uint32_t *s8, PMC_LDS const uint32_t *zp) {
    const int l = lane_id(), q = l >> 4, s = l & 15;
    uint32_t res = 0;
    uint64_t small = todo & ballot(mylen <= kCrcQuarterMax);
    uint64_t large = todo & ~small;
    while (small) {
        int jq[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            jq[t] = small ? __builtin_ctzll(small) : 64;
            small &= small - 1;
        }
        const int j = q == 0 ? jq[0] : q == 1 ? jq[1] : q == 2 ? jq[2] : jq[3];
        const uint32_t len = (uint32_t)__shfl((int)mylen, j & 63);
        uint32_t c = 0;
        if (j < 64 && kCrcPiece * (uint32_t)s < len) c = crc_piece64(buf, off[g + (uint64_t)j], len, (uint32_t)s, s8);
        c = crc_fold_level<0>(c, zp);
        c = crc_fold_level<1>(c, zp);
        c = crc_fold_level<2>(c, zp);
        c = crc_fold_level<3>(c, zp);
        c = ~(c ^ c_crc_ones[len <= kCrcQuarterMax ? len : 0]);
        const int src = l == jq[0] ? 0 : l == jq[1] ? 16 : l == jq[2] ? 32 : l == jq[3] ? 48 : -1;
        const uint32_t mine = (uint32_t)__shfl((int)c, src & 63);
        res = src >= 0 ? mine : res;
    }
    while (large) {
        const int j = __builtin_ctzll(large);
        large &= large - 1;
        const uint32_t len = (uint32_t)__shfl((int)mylen, j);
        const uint32_t c = wave_crc32(buf + off[g + (uint64_t)j], len, s8);
        res = l == j ? c : res;
    }
    return res;
}

__device__ __forceinline__ void load_crc_tables(PMC_LDS uint32_t *s8, PMC_LDS uint32_t *zp) {
    for (int k = threadIdx.x; k < 8 * 256; k += blockDim.x) s8[k] = c_crc_slice8[k];
    for (int k = threadIdx.x; k < 4 * 4 * 256; k += blockDim.x) zp[k] = c_crc_zpiece[k];
    __syncthreads();
}

// CRC-32 of every member the lane kernel decoded; a mismatch sends the member to the wave
// kernel for zlib's verdict.
__global__ void __launch_bounds__(512) inflate_verify_kernel(InflateArgs a) {
    __shared__ uint32_t s8[8 * 256], zp[4 * 4 * 256];
    load_crc_tables(to_lds<uint32_t>(s8), to_lds<uint32_t>(zp));
    const int wpb = blockDim.x / 64, l = lane_id();
    const uint64_t wave = (uint64_t)blockIdx.x * wpb + threadIdx.x / 64, nwaves = (uint64_t)gridDim.x * wpb;
    // (a.verify_group members per wave: a small batch spreads over more waves)
    const uint32_t G = a.verify_group ? a.verify_group : 64u;
    for (uint64_t g = wave * G; g < a.n; g += nwaves * G) {
        const uint64_t vl = g + (uint64_t)l;
        const bool ok = (uint32_t)l < G && vl < a.n && a.rc[vl] == 0;
        const uint32_t mylen = ok ? a.dst_len[vl] : 0;
        const uint32_t c = wave_crc32_members(a.dst, a.dst_off, g, ballot(ok), mylen, to_lds<const uint32_t>(s8),
                                              to_lds<const uint32_t>(zp));
        if (ok && c != a.crc_expect[vl]) a.rc[vl] = kInflateRetry;
    }
}

// crc[i] = CRC-32 (gzip trailer) of buf[off[i] .. off[i] + len[i]) -- the verify pass's
// engine as a batch entry point
__global__ void __launch_bounds__(512) crc32_batch_kernel(const uint8_t *buf, const uint64_t *off, const uint32_t *len,
                                                          uint64_t n, uint32_t *crc) {
    __shared__ uint32_t s8[8 * 256], zp[4 * 4 * 256];
    load_crc_tables(to_lds<uint32_t>(s8), to_lds<uint32_t>(zp));
    const int wpb = blockDim.x / 64, l = lane_id();
    const uint64_t wave = (uint64_t)blockIdx.x * wpb + threadIdx.x / 64, nwaves = (uint64_t)gridDim.x * wpb;
    for (uint64_t g = wave * 64; g < n; g += nwaves * 64) {
        const uint64_t vl = g + (uint64_t)l;
        const bool ok = vl < n;
        const uint32_t c = wave_crc32_members(buf, off, g, ballot(ok), ok ? len[vl] : 0, to_lds<const uint32_t>(s8),
                                              to_lds<const uint32_t>(zp));
        if (ok) crc[vl] = c;
    }
}

} // namespace pmc
