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

constexpr int kLaneLitCap = 128, kLaneDistCap = 32;
// per-lane LDS columns (u16 words): symbol lists, code-length code list, counts/offsets, bases
constexpr int kColLit = 0, kColDist = kColLit + kLaneLitCap, kColCl = kColDist + kLaneDistCap;
constexpr int kColCntL = kColCl + 19, kColCntD = kColCntL + 16, kColBaseL = kColCntD + 16;
constexpr int kColBaseD = kColBaseL + 16, kColBaseC = kColBaseD + 16, kColWords = kColBaseC + 8;
constexpr uint32_t kLaneTabOff = (uint32_t)kColWords * 64 * 2;     // length/distance base tables
constexpr uint32_t kLaneLdsBytes = kLaneTabOff + 64 * 4;

// Bit reader over a member in HBM.  Input arrives as aligned 16-byte blocks, one block
// ahead of the one being consumed, so the load a refill depends on was issued ~4 refills
// earlier (loads and stores share vmcnt on gfx9: an immediately-used load would also wait
// for every output byte stored before it).  Aligned blocks never cross a page, so reading
// the tail of the last one is safe.
struct LaneIn {
    const uint8_t *p;
    uint32_t len;       // member bytes
    const uint4 *blk;   // aligned block base (p rounded down to 16)
    uint32_t bi;        // index of the block in `cur`
    uint4 cur, nxt;     // block bi and bi + 1
    uint32_t wi;        // next dword of `cur` to move into buf
    uint64_t buf;       // unread bits, LSB first
    uint32_t n;         // bits in buf
    uint64_t consumed0; // stream bit offset of buf bit 0 when bi/wi were set
    __device__ uint32_t byte_at(uint32_t i) const { return i < len ? (uint32_t)p[i] : 0u; }
    // block k of the stream, or zeros past the member's last block (never touches its page)
    __device__ uint4 block(uint32_t k) const {
        return (uint64_t)k * 16 < ((uintptr_t)p & 15) + (uint64_t)len ? blk[k] : make_uint4(0, 0, 0, 0);
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

// One canonical code of up to 15-bit lengths: per-length limits in registers, bases and the
// sorted symbol list in the lane's LDS column.
template <int NL>
struct LaneCode {
    uint32_t lim[NL]; // left-justified (15-bit) end of the codes of length j + 1
    PMC_LDS int16_t *base;
    PMC_LDS uint16_t *sym;
    // from counts cnt[1..NL] (LDS column); returns false unless the code is complete
    // (every well-formed zlib stream's codes are; other shapes go to the wave kernel)
    __device__ bool build(PMC_LDS const uint16_t *cnt) {
        int32_t first = 0, offs = 0, left = 1;
#pragma unroll
        for (int L = 1; L <= NL; L++) {
            const int32_t c = cnt[L * 64];
            base[L * 64] = (int16_t)(offs - first);
            first += c;
            lim[L - 1] = (uint32_t)first << (15 - L);
            first <<= 1;
            offs += c;
            left = (left << 1) - c;
        }
        return left == 0;
    }
    __device__ uint32_t decode(LaneIn &in) const {
        const uint32_t x = __builtin_bitreverse32(in.peek(15)) >> 17;
        uint32_t L = 1;
#pragma unroll
        for (int j = 0; j < NL - 1; j++) L += x >= lim[j] ? 1u : 0u;
        const int idx = (int)base[L * 64] + (int)(x >> (15 - L));
        in.drop(L);
        return sym[idx * 64];
    }
};

__device__ __forceinline__ uint32_t fixed_lit(LaneIn &in) {
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
__device__ bool lane_lengths(LaneIn &in, const LaneCode<7> &clc, uint32_t nlen, uint32_t nlit, PMC_LDS uint16_t *col,
                             int pass, bool &eob_ok) {
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
                PMC_LDS uint16_t *c = col + (lit ? kColCntL : kColCntD) * 64 + val * 64;
                if (pass == 0) {
                    *c = (uint16_t)(*c + 1);
                    if (k == 256) eob_ok = true;
                } else {
                    const uint32_t at = *c;
                    *c = (uint16_t)(at + 1);
                    col[((lit ? kColLit : kColDist) + at) * 64] = (uint16_t)(lit ? k : k - nlit);
                }
            }
        } else {
            k += rep;
        }
        prev = val;
    }
    return true;
}

__device__ void lane_copy(uint8_t *out, uint32_t pos, uint32_t dist, uint32_t len, uint32_t cap) {
    if (dist >= 8) {
        uint32_t k = 0;
        for (; k < len && pos + k + 4 <= cap; k += 8) {
            const uintptr_t a = (uintptr_t)(out + pos - dist + k);
            const uint32_t *q = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
            const uint32_t sh = (uint32_t)(a & 3);
            const uint32_t q0 = q[0], q1 = q[1], q2 = q[2];
            const uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(q2, q1, sh) << 32 | __builtin_amdgcn_alignbyte(q1, q0, sh);
            const uint32_t m = len - k < 8 ? len - k : 8;
#pragma unroll
            for (uint32_t j = 0; j < 8; j++)
                if (j < m) out[pos + k + j] = (uint8_t)(v >> (8 * j));
        }
        for (; k < len; k++) out[pos + k] = out[pos - dist + k]; // (last bytes of dst: no over-read)
    } else {
        uint64_t pat = 0;
        for (uint32_t j = 0; j < dist; j++) pat |= (uint64_t)out[pos - dist + j] << (8 * j);
        uint32_t idx = 0;
        for (uint32_t k = 0; k < len; k++) {
            out[pos + k] = (uint8_t)(pat >> (8 * idx));
            idx = idx + 1 == dist ? 0 : idx + 1;
        }
    }
}

// Decodes one member; returns 0 (output written, CRC still to check) or kInflateRetry.
__device__ int lane_inflate(LaneIn &in, uint8_t *out, uint32_t cap, PMC_LDS uint16_t *col,
                            PMC_LDS const uint32_t *ltab, PMC_LDS const uint32_t *dtab, uint32_t *out_len,
                            uint32_t *crc_expect) {
    if (in.len < 18) return kInflateRetry;
    if (in.byte_at(0) != 0x1f || in.byte_at(1) != 0x8b || in.byte_at(2) != 8 || in.byte_at(3) != 0) return kInflateRetry;
    in.seek(80);
    LaneCode<15> lit, dist;
    lit.base = (PMC_LDS int16_t *)(col + kColBaseL * 64);
    lit.sym = col + kColLit * 64;
    dist.base = (PMC_LDS int16_t *)(col + kColBaseD * 64);
    dist.sym = col + kColDist * 64;
    uint32_t pos = 0, bfinal;
    do {
        bfinal = in.bits(1);
        const uint32_t btype = in.bits(2);
        if (btype == 0) {
            uint64_t bp = (in.bitpos() + 7) & ~(uint64_t)7;
            const uint32_t o = (uint32_t)(bp >> 3);
            if (o + 4 > in.len) return kInflateRetry;
            const uint32_t L = in.byte_at(o) | in.byte_at(o + 1) << 8, NL = in.byte_at(o + 2) | in.byte_at(o + 3) << 8;
            if ((L ^ 0xffffu) != NL || o + 4 + L > in.len || pos + L > cap) return kInflateRetry;
            for (uint32_t k = 0; k < L; k++) out[pos + k] = in.p[o + 4 + k];
            pos += L;
            in.seek((uint64_t)(o + 4 + L) * 8);
            continue;
        }
        if (btype == 3) return kInflateRetry;
        const bool fixed = btype == 1;
        if (!fixed) {
            const uint32_t nlit = in.bits(5) + 257, ndist = in.bits(5) + 1, ncl = in.bits(4) + 4;
            if (nlit > 286 || ndist > 30) return kInflateRetry;
            // code-length code: lengths (3 bits each, permuted order), counts, list
            uint64_t cll = 0;
            for (uint32_t k = 0; k < ncl; k++) cll |= (uint64_t)in.bits(3) << (3 * c_cl_order[k]);
            for (int L = 0; L < 16; L++) col[(kColCntL + L) * 64] = 0;
            for (uint32_t s = 0; s < 19; s++) {
                const uint32_t L = (uint32_t)(cll >> (3 * s)) & 7;
                if (L) col[(kColCntL + L) * 64] = (uint16_t)(col[(kColCntL + L) * 64] + 1);
            }
            LaneCode<7> clc;
            clc.base = (PMC_LDS int16_t *)(col + kColBaseC * 64);
            clc.sym = col + kColCl * 64;
            if (!clc.build(col + kColCntL * 64)) return kInflateRetry;
            {
                uint32_t offs = 0;
                for (int L = 1; L < 8; L++) {
                    const uint32_t c = col[(kColCntL + L) * 64];
                    col[(kColCntL + L) * 64] = (uint16_t)offs;
                    offs += c;
                }
                for (uint32_t s = 0; s < 19; s++) {
                    const uint32_t L = (uint32_t)(cll >> (3 * s)) & 7;
                    if (L) {
                        const uint32_t at = col[(kColCntL + L) * 64];
                        col[(kColCntL + L) * 64] = (uint16_t)(at + 1);
                        clc.sym[at * 64] = (uint16_t)s;
                    }
                }
            }
            // pass 0: counts of the literal/length and distance codes
            for (int L = 0; L < 16; L++) {
                col[(kColCntL + L) * 64] = 0;
                col[(kColCntD + L) * 64] = 0;
            }
            const uint64_t lens_at = in.bitpos();
            bool eob_ok = false;
            if (!lane_lengths(in, clc, nlit + ndist, nlit, col, 0, eob_ok) || !eob_ok) return kInflateRetry;
            const uint64_t data_at = in.bitpos();
            uint32_t nl = 0, nd = 0;
            for (int L = 1; L < 16; L++) {
                nl += col[(kColCntL + L) * 64];
                nd += col[(kColCntD + L) * 64];
            }
            if (nl > (uint32_t)kLaneLitCap || nd > (uint32_t)kLaneDistCap) return kInflateRetry;
            if (!lit.build(col + kColCntL * 64) || !dist.build(col + kColCntD * 64)) return kInflateRetry;
            // counts -> running offsets, pass 1: place the symbols
            {
                uint32_t ol = 0, od = 0;
                for (int L = 1; L < 16; L++) {
                    const uint32_t cl = col[(kColCntL + L) * 64], cd = col[(kColCntD + L) * 64];
                    col[(kColCntL + L) * 64] = (uint16_t)ol;
                    col[(kColCntD + L) * 64] = (uint16_t)od;
                    ol += cl;
                    od += cd;
                }
            }
            in.seek(lens_at);
            lane_lengths(in, clc, nlit + ndist, nlit, col, 1, eob_ok);
            in.seek(data_at);
        }
        for (;;) {
            in.refill();
            const uint32_t s = fixed ? fixed_lit(in) : lit.decode(in);
            if (s < 256) {
                if (pos >= cap) return kInflateRetry;
                out[pos++] = (uint8_t)s;
                continue;
            }
            if (s == 256) break;
            if (s > 285) return kInflateRetry;
            const uint32_t le = ltab[s - 257];
            const uint32_t len = (le & 0xffff) + in.bits(le >> 16);
            in.refill();
            const uint32_t ds = fixed ? __builtin_bitreverse32(in.peek(5)) >> 27 : dist.decode(in);
            if (fixed) in.drop(5);
            if (ds > 29) return kInflateRetry;
            const uint32_t de = dtab[ds];
            const uint32_t d = (de & 0xffff) + in.bits(de >> 16);
            if (d > pos || pos + len > cap) return kInflateRetry;
            lane_copy(out, pos, d, len, cap);
            pos += len;
        }
        if (in.bitpos() > (uint64_t)in.len * 8) return kInflateRetry;
    } while (!bfinal);
    const uint32_t t = (uint32_t)((in.bitpos() + 7) >> 3);
    if (in.bitpos() > (uint64_t)in.len * 8 || t + 8 > in.len) return kInflateRetry;
    const uint32_t isz = in.byte_at(t + 4) | in.byte_at(t + 5) << 8 | in.byte_at(t + 6) << 16 | in.byte_at(t + 7) << 24;
    if (isz != pos) return kInflateRetry;
    *crc_expect = in.byte_at(t) | in.byte_at(t + 1) << 8 | in.byte_at(t + 2) << 16 | in.byte_at(t + 3) << 24;
    *out_len = pos;
    return 0;
}

__global__ void __launch_bounds__(64) inflate_lane_kernel(InflateArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lcol[];
    PMC_LDS uint16_t *col = to_lds<uint16_t>(lcol + threadIdx.x);
    PMC_LDS uint32_t *ltab = to_lds<uint32_t>((uint8_t *)lcol + kLaneTabOff), *dtab = ltab + 32;
    if (threadIdx.x < 29) ltab[threadIdx.x] = (uint32_t)c_lbase[threadIdx.x] | (uint32_t)c_lext[threadIdx.x] << 16;
    if (threadIdx.x < 30) dtab[threadIdx.x] = (uint32_t)c_dbase[threadIdx.x] | (uint32_t)c_dext[threadIdx.x] << 16;
    __syncthreads();
    for (uint64_t v = (uint64_t)blockIdx.x * 64 + threadIdx.x; v < a.n; v += (uint64_t)gridDim.x * 64) {
        const uint32_t in_len = a.src_len[v];
        if (in_len == 0) {
            a.rc[v] = PMC_INVALID_INPUT_DEV;
            a.dst_len[v] = 0;
            continue;
        }
        LaneIn in;
        in.p = a.src + a.src_off[v];
        in.len = in_len;
        in.blk = reinterpret_cast<const uint4 *>((uintptr_t)in.p & ~(uintptr_t)15);
        uint32_t olen = 0, crc = 0;
        const int rc = lane_inflate(in, a.dst + a.dst_off[v], a.dst_cap[v], col, ltab, dtab, &olen, &crc);
        a.rc[v] = rc;
        a.dst_len[v] = olen;
        a.crc_expect[v] = crc;
    }
}

// CRC-32 of every member the lane kernel decoded (wave per member); a mismatch sends the
// member to the wave kernel for zlib's verdict.
__global__ void __launch_bounds__(256) inflate_verify_kernel(InflateArgs a) {
    __shared__ uint32_t crc_tab[256];
    for (int k = threadIdx.x; k < 256; k += blockDim.x) crc_tab[k] = c_crc_table[k];
    __syncthreads();
    const int wpb = blockDim.x / 64, l = lane_id();
    const uint64_t wave = (uint64_t)blockIdx.x * wpb + threadIdx.x / 64, nwaves = (uint64_t)gridDim.x * wpb;
    for (uint64_t g = wave * 64; g < a.n; g += nwaves * 64) {
        const uint64_t vl = g + (uint64_t)l;
        const int32_t myrc = vl < a.n ? a.rc[vl] : -1;
        uint64_t todo = ballot(vl < a.n && myrc == 0);
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint64_t v = g + (uint64_t)j;
            const uint32_t c = wave_crc32(a.dst + a.dst_off[v], a.dst_len[v], to_lds<const uint32_t>(crc_tab));
            if (l == 0 && c != a.crc_expect[v]) a.rc[v] = kInflateRetry;
        }
    }
}

} // namespace pmc
