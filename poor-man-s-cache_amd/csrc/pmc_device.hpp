// pmc_device.hpp -- gfx950 device primitives shared by the codec kernels.
//
// Wave64 helpers (ballot / shuffle reductions / scans), the zlib constant tables in
// __constant__ memory, and a lane-parallel CRC-32 (the gzip trailer checksum zlib's
// read_buf folds in, deflate.c / crc32.c) for a byte string resident in LDS or HBM.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pmc_trees.hpp"

namespace pmc {

constexpr int kWave = 64;

// LDS-typed pointers: accesses compile to ds_* with 32-bit addresses wherever the pointer
// itself lives (a generic pointer kept in a struct in scratch degrades to flat_* ops).
#define PMC_LDS __attribute__((address_space(3)))
// global-typed pointers: global_* loads (vmcnt only) instead of flat_* (vmcnt + lgkmcnt)
#define PMC_GLB __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ PMC_LDS T *to_lds(void *p) {
    return (PMC_LDS T *)(p);
}
__device__ __forceinline__ uint32_t lds_add(PMC_LDS uint32_t *p, uint32_t v) {
    return __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
}
__device__ __forceinline__ uint32_t lds_or(PMC_LDS uint32_t *p, uint32_t v) {
    return __atomic_fetch_or(p, v, __ATOMIC_RELAXED);
}
constexpr uint32_t kCrcPoly = 0xEDB88320u;
constexpr int kCrcShiftEntries = 4096; // x^(128*d) mod P for d < 4096 (16-byte steps)

// zlib trees.c static tables (make_tables() is constexpr; copied once at load time).
extern __constant__ Tables c_tables;
extern __constant__ uint32_t c_crc_table[256];
extern __constant__ uint32_t c_crc_shift16[kCrcShiftEntries];  // x^(8*16*d)   mod P
extern __constant__ uint32_t c_crc_shift64k[kCrcShiftEntries]; // x^(8*65536*d) mod P
// quarter-wave CRC (wave_crc32_members): a member of up to kCrcQuarterMax bytes takes 16
// lanes, each lane one kCrcPiece-byte piece
constexpr uint32_t kCrcPiece = 64;
constexpr uint32_t kCrcQuarterMax = 16 * kCrcPiece;
extern __constant__ uint32_t c_crc_slice8[8 * 256];              // slicing-by-8: T_k = byte then k zero bytes
extern __constant__ uint32_t c_crc_zpiece[4 * 4 * 256];          // [level k][byte j][b]: (b << 8j) x^(8*64*2^k)
extern __constant__ uint32_t c_crc_ones[kCrcQuarterMax + 1];     // 0xFFFFFFFF x^(8*len): the init's share

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    uint32_t lo = rfl((uint32_t)v), hi = rfl((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Intra-wave ordering point for LDS/global hand-offs between lanes of one wave.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// Ordering point strong enough for per-wave scratch in global memory (waits for stores).
__device__ __forceinline__ void wave_sync_global() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t t = __shfl_xor(v, o);
        v = t > v ? t : v;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ uint32_t wave_xor_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o);
    return v;
}
// inclusive prefix sum across the wave
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o);
        if (l >= o) v += t;
    }
    return v;
}
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v) {
    int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t t = __shfl_up(v, o);
        if (l >= o) v += t;
    }
    return v;
}

// ---- DPP-based wave primitives (no LDS round trip) --------------------------------------
// inclusive prefix sum over the wave: row_shr 1,2,4,8 inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 carry the row totals (GFX9-family DPP; lanes shifted in read 0)
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    return v;
}
// inclusive max-scan over the wave (same DPP pattern; lanes shifted in read 0, the identity
// for unsigned max)
__device__ __forceinline__ uint32_t wave_incl_max_dpp(uint32_t v) {
    uint32_t t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    v = t > v ? t : v;
    return v;
}
// row-level butterfly with quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror:
// afterwards every lane holds the max of its 16-lane row.
__device__ __forceinline__ uint32_t dpp_row_max(uint32_t v) {
    uint32_t t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);
    v = t > v ? t : v;
    return v;
}
// max over the wave, result uniform (SGPR).  All 64 lanes must be active.
__device__ __forceinline__ uint32_t wave_max_dpp(uint32_t v) {
    v = dpp_row_max(v);
    uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    a = a > b ? a : b;
    c = c > d ? c : d;
    return a > c ? a : c;
}
__device__ __forceinline__ uint32_t readlane(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return (uint64_t)readlane((uint32_t)(v >> 32), l) << 32 | readlane((uint32_t)v, l);
}
// v_writelane without inline asm: compare + select (2 VALU, no hazards to pad)
__device__ __forceinline__ uint32_t writelane(uint32_t old, uint32_t v, int l) {
    return lane_id() == l ? v : old;
}
// number of lanes below this one in mask
__device__ __forceinline__ uint32_t popc_lt(uint64_t mask) {
    return (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// N u16 counters packed two per VGPR.  Every access goes through unrolled selects on the index, so the
// array stays in registers (an indexed private array would live in scratch): per-lane tables of the
// lane-per-value kernels (trees, inflate code tables) without LDS round trips.
template <int N>
struct RegU16 {
    static constexpr int kW = (N + 1) / 2;
    uint32_t w[kW];
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int j = 0; j < kW; j++) w[j] = 0;
    }
    __device__ __forceinline__ uint32_t get(uint32_t i) const {
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < kW; j++) x = (i >> 1) == (uint32_t)j ? w[j] : x;
        return (x >> ((i & 1u) * 16)) & 0xffffu;
    }
    __device__ __forceinline__ void add(uint32_t i, int32_t v) { // (fields never go below 0 in use)
        const uint32_t d = (uint32_t)v << ((i & 1u) * 16);
#pragma unroll
        for (int j = 0; j < kW; j++) w[j] += (i >> 1) == (uint32_t)j ? d : 0u;
    }
    __device__ __forceinline__ void set(uint32_t i, uint32_t v) {
        const uint32_t sh = (i & 1u) * 16;
#pragma unroll
        for (int j = 0; j < kW; j++)
            w[j] = (i >> 1) == (uint32_t)j ? (w[j] & ~(0xffffu << sh)) | (v & 0xffffu) << sh : w[j];
    }
};

// GF(2) product a*b mod P in the reflected CRC-32 domain (zlib 1.2.12 multmodp).
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll 8
    for (int k = 31; k >= 0; k--) {
        p ^= ((a >> k) & 1u) ? b : 0u;
        b = (b >> 1) ^ (kCrcPoly & (0u - (b & 1u)));
    }
    return p;
}

// x^(8*16*d) mod P for any chunk distance d.
__device__ __forceinline__ uint32_t crc_shift_chunks(uint32_t d) {
    uint32_t k = c_crc_shift16[d & (kCrcShiftEntries - 1)];
    if (d >= (uint32_t)kCrcShiftEntries) k = multmodp(k, c_crc_shift64k[d >> 12]);
    return k;
}

// CRC-32 of buf[0..len) computed by the whole wave.  The message is cut into 16-byte
// chunks aligned from its END (chunk d covers [len-16(d+1), len-16d)); lane l takes
// chunks d = l, l+64, ...  Each chunk's register (from 0, or from 0xFFFFFFFF for the
// chunk holding byte 0) is shifted past the d*16 bytes that follow it by one GF(2)
// multiply with x^(128 d) mod P, and the wave XOR-reduces.  By linearity of the CRC
// register this equals the serial crc32().  `tab` is a 256-entry table (LDS).
template <class BytePtr, class TabPtr>
__device__ inline uint32_t wave_crc32(BytePtr buf, uint32_t len, TabPtr tab) {
    uint32_t nchunks = (len + 15) >> 4;
    uint32_t acc = 0;
    for (uint32_t d = (uint32_t)lane_id(); d < nchunks; d += 64) {
        int64_t end = (int64_t)len - 16 * (int64_t)d;
        int64_t beg = end - 16;
        uint32_t c = 0;
        if (beg <= 0) {
            beg = 0;
            c = 0xFFFFFFFFu;
        }
        for (int64_t k = beg; k < end; k++) c = tab[(c ^ buf[k]) & 0xff] ^ (c >> 8);
        acc ^= d ? multmodp(crc_shift_chunks(d), c) : c;
    }
    acc = wave_xor_u32(acc);
    if (len == 0) return 0;
    return ~acc;
}

// x^(8r) mod P for r < 16 (reflected domain: 0x80000000 is x^0; a multiply by x shifts right and
// folds the polynomial in)
struct CrcX8 {
    uint32_t v[16];
};
constexpr CrcX8 make_crc_x8() {
    CrcX8 t{};
    uint32_t p = 0x80000000u;
    for (int r = 0; r < 16; r++) {
        t.v[r] = p;
        for (int b = 0; b < 8; b++) p = (p >> 1) ^ ((p & 1u) ? kCrcPoly : 0u);
    }
    return t;
}
// xor over the wave, result uniform: row butterflies by DPP (quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror), then the four row totals.  All 64 lanes must be active.
__device__ __forceinline__ uint32_t wave_xor_dpp(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);
    return readlane(v, 0) ^ readlane(v, 16) ^ readlane(v, 32) ^ readlane(v, 48);
}
// CRC-32 of buf[0..len) (bytes in LDS, read as words `bw`; the buffer may be read up to 4 bytes
// past len) by the whole wave with slicing-by-8 (`s8`: c_crc_slice8 in LDS, 8 KiB).  16-byte
// chunks aligned from the END as in wave_crc32, but every chunk starts from register 0 with zero
// bytes in front of byte 0 (which leave a register-0 CRC unchanged), so a chunk is two table steps
// of eight independent lookups instead of sixteen dependent ones; the init value's share
// 0xFFFFFFFF x^(8 len) is added once.
__device__ inline uint32_t wave_crc32_s8(PMC_LDS const uint32_t *bw, uint32_t len, PMC_LDS const uint32_t *s8) {
    constexpr CrcX8 kX8 = make_crc_x8();
    const uint32_t nchunks = (len + 15) >> 4;
    uint32_t acc = 0;
    for (uint32_t d = (uint32_t)lane_id(); d < nchunks; d += 64) {
        const int32_t beg = (int32_t)len - 16 * (int32_t)(d + 1);
        const int32_t wb = beg >> 2, lead = beg < 0 ? -beg : 0;
        const uint32_t sh = (uint32_t)beg & 3u;
        uint32_t w[5], x[4];
#pragma unroll
        for (int i = 0; i < 5; i++) w[i] = bw[wb + i > 0 ? wb + i : 0];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t v = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
            const int32_t r = lead - 4 * i;
            x[i] = r <= 0 ? v : (r >= 4 ? 0u : v & (0xFFFFFFFFu << (8 * r)));
        }
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const uint32_t a0 = x[2 * k] ^ c, a1 = x[2 * k + 1];
            c = s8[7 * 256 + (a0 & 0xff)] ^ s8[6 * 256 + ((a0 >> 8) & 0xff)] ^ s8[5 * 256 + ((a0 >> 16) & 0xff)] ^
                s8[4 * 256 + (a0 >> 24)] ^ s8[3 * 256 + (a1 & 0xff)] ^ s8[2 * 256 + ((a1 >> 8) & 0xff)] ^
                s8[1 * 256 + ((a1 >> 16) & 0xff)] ^ s8[a1 >> 24];
        }
        acc ^= d ? multmodp(crc_shift_chunks(d), c) : c;
    }
    acc = wave_xor_dpp(acc);
    if (len == 0) return 0;
    const uint32_t ones = len <= kCrcQuarterMax ? c_crc_ones[len]
                                                : multmodp(multmodp(crc_shift_chunks(len >> 4), kX8.v[len & 15]),
                                                           0xFFFFFFFFu);
    return ~(acc ^ ones);
}

} // namespace pmc
