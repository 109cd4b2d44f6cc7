// pmc_deflate.hip -- batched gzip (zlib 1.2.11 level 9) compression on gfx950.
//
// Replaces GzipCompressor::Compress (/root/reference/src/compressor/gzip_compressor.cpp:3-50,
// called from src/kvs/kvs.cpp:183) for many independent values at once.  Bytes out are
// identical to zlib's deflateInit2(9, Z_DEFLATED, 31, 8, Z_DEFAULT_STRATEGY) + deflate(Z_FINISH).
//
// Work decomposition (one wave64 per value; a workgroup holds W independent waves; the
// grid is persistent and waves stride over the batch):
//   1. stage the value in LDS (coalesced), CRC-32 it lane-parallel (pmc_device.hpp)
//   2. hash every position: h(p) = (b[p]<<10 ^ b[p+1]<<5 ^ b[p+2]) & 0x7fff  -- zlib's
//      UPDATE_HASH after 3 steps (HASH_SHIFT 5, 15 bits) -- and radix-sort positions
//      stably by hash (3 x 5-bit LSD passes in LDS).  zlib's head/prev chain of position i
//      is then the contiguous run S[rank(i)-1], S[rank(i)-2], ... of equal hash.
//   3. zlib's deflate_slow lazy parse runs serially (wave-uniform scalar state), but every
//      longest_match call evaluates 64 chain candidates at once, one per lane: LCP by
//      4-byte compares (v_alignbyte on LDS words), wave max-reduction keyed
//      (len << 16 | ~index) so the nearest candidate wins ties exactly as zlib's strict `>`.
//   4. symbols go to a per-wave HBM slab in coalesced 64-token stores; frequencies to the
//      LDS trees.  Every 16383 symbols (and at the end) the block is flushed:
//      lane 0 builds the three Huffman trees with zlib's exact heap (pmc_trees.hpp), the
//      wave picks stored/fixed/dynamic like _tr_flush_block, lane 0 writes the tree
//      header, and the wave emits all symbols in parallel: per-symbol bit lengths ->
//      wave prefix sum -> ds_or_b32 into the LDS output image.
//   5. gzip header / trailer, copy-out to HBM.
// Values too large for the LDS working set take the same code with the working set in a
// per-wave HBM slab (kHbm variant).
#include <hip/hip_runtime.h>

#include "pmc_device.hpp"
#include "pmc_kernels.hpp"

namespace pmc {

constexpr uint32_t kMinMatch = 3, kMaxMatch = 258, kMinLookahead = 262;
constexpr uint32_t kWSize = 32768, kMaxDist = kWSize - kMinLookahead; // 32506
constexpr uint32_t kTooFar = 4096, kGoodLength = 32, kMaxLazy = 258, kMaxChain = 4096;
constexpr uint32_t kSymsPerBlock = 16383; // lit_bufsize - 1 (memLevel 8)

// ---------------------------------------------------------------------------------
// Per-wave working set.  Key = hash << kKeyShift | position.
template <bool kHbm>
struct Arena;

template <>
struct Arena<false> { // LDS-resident, positions < 65536
    using Key = uint32_t;
    using Rank = uint16_t;
    static constexpr int kKeyShift = 16;
    static constexpr uint64_t kPosMask = 0xffff;
};
template <>
struct Arena<true> { // HBM-resident, any size
    using Key = uint64_t;
    using Rank = uint32_t;
    static constexpr int kKeyShift = 32;
    static constexpr uint64_t kPosMask = 0xffffffffull;
};

__host__ __device__ inline uint64_t align16(uint64_t x) { return (x + 15) & ~(uint64_t)15; }

// Byte layout of one wave's working set for capacity n (max value length).
struct DeflateLayout {
    uint64_t trees, bytes, S, rank, work, total;
    uint64_t out_words; // capacity of the output image in 32-bit words
};

template <bool kHbm>
__host__ __device__ inline DeflateLayout deflate_layout(uint64_t n) {
    using A = Arena<kHbm>;
    DeflateLayout L;
    uint64_t off = 0;
    L.trees = off;
    off += align16(sizeof(Trees));
    L.bytes = off;
    off += align16(n + 32);
    L.S = off;
    off += align16(sizeof(typename A::Key) * (n + 1));
    L.rank = off;
    off += align16(sizeof(typename A::Rank) * (n + 1));
    L.work = off;
    uint64_t sortw = align16(sizeof(typename A::Key) * (n + 1)) + 32 * 64 * sizeof(uint32_t);
    uint64_t outb = align16(gzip_bound(n) + 16);
    L.out_words = outb / 4;
    off += sortw > outb ? sortw : outb;
    L.total = align16(off);
    return L;
}

uint64_t deflate_wave_bytes(bool hbm, uint64_t n) {
    return hbm ? deflate_layout<true>(n).total : deflate_layout<false>(n).total;
}

// ---------------------------------------------------------------------------------
// Bit sink used by lane 0 for block headers and trees (send_bits, LSB first).
struct LaneBits {
    uint32_t *out;
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

template <class Word>
__device__ inline void or_bits(Word *out, uint64_t pos, uint64_t v, int n) {
    if (n == 0) return;
    uint64_t w = pos >> 5;
    int s = (int)(pos & 31);
    uint32_t lo = (uint32_t)(v << s);
    uint32_t mid = (uint32_t)((s ? (v >> (32 - s)) : (v >> 32)));
    uint32_t hi = s ? (uint32_t)(v >> (64 - s)) : 0u;
    if (lo) atomicOr(&out[w], lo);
    if (n + s > 32 && mid) atomicOr(&out[w + 1], mid);
    if (n + s > 64 && hi) atomicOr(&out[w + 2], hi);
}

// ---------------------------------------------------------------------------------
template <bool kHbm>
struct DeflateWave {
    using A = Arena<kHbm>;
    using Key = typename A::Key;
    using Rank = typename A::Rank;

    Trees *tr;
    uint8_t *b;   // value bytes (+zero padding)
    uint32_t *bw; // same, as words
    Key *S;
    Rank *rank;
    uint8_t *work;
    uint32_t *outw;
    uint8_t *outb;
    uint32_t *tok; // per-wave HBM symbol slab (kSymsPerBlock entries)
    const uint32_t *crc_tab;
    uint64_t out_words;
    // diagnostic phase stamps (PMC_STAMPS builds only; never quoted as timings)
    uint64_t st[8];
    uint64_t t_last;
    __device__ void stamp(int k) {
#ifdef PMC_STAMPS
        uint64_t t = __builtin_amdgcn_s_memtime();
        st[k] += t - t_last;
        t_last = t;
#endif
    }

    __device__ void sync() {
        if (kHbm) wave_sync_global();
        else wave_sync();
    }

    __device__ uint32_t load4(uint64_t p) const {
        uint32_t w0 = bw[p >> 2], w1 = bw[(p >> 2) + 1];
        return __builtin_amdgcn_alignbyte(w1, w0, (uint32_t)(p & 3));
    }

    // LCP of positions i and q (q < i), capped at cap.  Bytes past the value are zero;
    // the cap (nice = min(258, len-i)) makes them irrelevant, as in zlib.
    __device__ uint32_t lcp(uint64_t i, uint64_t q, uint32_t cap) const {
        uint32_t l = 0;
        if (kHbm) {
            // HBM working set: 32 bytes per round trip (9 independent dword loads per side, then
            // compares), not one dependent 4-byte load pair per step -- a 258-byte match had cost
            // 65 global round trips per candidate (1 MiB values: 0.02 GiB/s)
            while (l < cap) {
                const uint64_t a = i + l, c = q + l;
                const uint32_t sa = (uint32_t)(a & 3), sc = (uint32_t)(c & 3);
                uint32_t wa[9], wc[9];
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    wa[k] = bw[(a >> 2) + k];
                    wc[k] = bw[(c >> 2) + k];
                }
                uint32_t m = 32;
#pragma unroll
                for (int k = 7; k >= 0; k--) {
                    const uint32_t x = __builtin_amdgcn_alignbyte(wa[k + 1], wa[k], sa) ^
                                       __builtin_amdgcn_alignbyte(wc[k + 1], wc[k], sc);
                    m = x ? 4 * (uint32_t)k + ((uint32_t)__builtin_ctz(x) >> 3) : m;
                }
                l += m;
                if (m < 32) break;
            }
            return l < cap ? l : cap;
        }
        while (l < cap) {
            uint32_t x = load4(i + l) ^ load4(q + l);
            if (x) {
                l += (uint32_t)__builtin_ctz(x) >> 3;
                break;
            }
            l += 4;
        }
        return l < cap ? l : cap;
    }

    // ---- stage 2: stable LSD radix sort of positions by hash (3 x 5 bits) ----------------
    __device__ void sort_positions(uint64_t npos) {
        const int l = lane_id();
        Key *A0 = reinterpret_cast<Key *>(work);
        uint32_t *cnt = reinterpret_cast<uint32_t *>(work + align16(sizeof(Key) * (npos + 1)));
        uint64_t c = (npos + 63) / 64; // chunk per lane (stability: lane-major chunks)
        for (uint64_t p = l; p < npos; p += 64) {
            uint32_t h = ((uint32_t)b[p] << 10 ^ (uint32_t)b[p + 1] << 5 ^ (uint32_t)b[p + 2]) & 0x7fffu;
            A0[p] = ((Key)h << A::kKeyShift) | (Key)p;
        }
        sync();
        Key *src = A0, *dst = S;
        for (int pass = 0; pass < 3; pass++) {
            const int sh = A::kKeyShift + 5 * pass;
            for (int d = 0; d < 32; d++) cnt[d * 64 + l] = 0;
            for (uint64_t j = 0; j < c; j++) {
                uint64_t idx = (uint64_t)l * c + j;
                if (idx < npos) cnt[((src[idx] >> sh) & 31) * 64 + l]++;
            }
            sync();
            // exclusive scan over the 2048 counters in (digit, lane) order
            uint32_t v[32], s = 0;
#pragma unroll
            for (int k = 0; k < 32; k++) {
                v[k] = cnt[l * 32 + k];
                s += v[k];
            }
            uint32_t base = wave_incl_scan(s) - s;
#pragma unroll
            for (int k = 0; k < 32; k++) {
                uint32_t t = v[k];
                cnt[l * 32 + k] = base;
                base += t;
            }
            sync();
            for (uint64_t j = 0; j < c; j++) {
                uint64_t idx = (uint64_t)l * c + j;
                if (idx < npos) {
                    Key k = src[idx];
                    uint32_t at = cnt[((k >> sh) & 31) * 64 + l]++;
                    dst[at] = k;
                }
            }
            sync();
            Key *t = src;
            src = dst;
            dst = t;
        }
        // passes write S, A0, S: the sorted keys are in S; build rank[]
        for (uint64_t k = l; k < npos; k += 64) rank[S[k] & A::kPosMask] = (Rank)k;
        sync();
    }

    // ---- longest_match(i) with prev_length b0 (deflate.c), over the sorted chain ----------
    // Returns the match length (> b0) or 0; *q_out = nearest candidate achieving it.
    __device__ uint32_t search(uint64_t i, uint32_t b0, uint64_t B, uint64_t len, uint64_t *q_out) {
        const int l = lane_id();
        const uint32_t C = b0 >= kGoodLength ? (kMaxChain >> 2) : kMaxChain;
        const uint32_t nice = (uint32_t)((len - i) < kMaxMatch ? (len - i) : kMaxMatch);
        const int64_t r = (int64_t)rank[i];
        const uint64_t hi = (uint64_t)(S[r] >> A::kKeyShift);
        uint32_t examined = 0, best = 0;
        uint64_t bestq = 0;
        for (int64_t kb = r - 1;; kb -= 64) {
            int64_t k = kb - l;
            bool valid = k >= 0;
            uint64_t q = 0;
            if (valid) {
                Key key = S[k];
                valid = (uint64_t)(key >> A::kKeyShift) == hi;
                q = (uint64_t)(key & A::kPosMask);
            }
            uint32_t ord = examined + (uint32_t)l;
            uint64_t d = i - q;
            valid = valid && q > B && (ord == 0 ? d <= kMaxDist : d < kMaxDist) && ord < C;
            uint64_t m = ballot(valid);
            // valid lanes form a prefix (contiguous equal-hash run, decreasing positions)
            uint32_t npre = ~m == 0 ? 64u : (uint32_t)__builtin_ctzll(~m);
            if (npre == 0) break;
            uint32_t cl = (uint32_t)l < npre ? lcp(i, q, nice) : 0u;
            uint32_t key = (cl << 16) | (0xffffu - ord);
            uint32_t mx = rfl(wave_max_u32(key));
            uint32_t mlen = mx >> 16;
            if (mlen > best) {
                best = mlen;
                int src = (int)((0xffffu - (mx & 0xffffu)) - examined);
                bestq = (uint64_t)__shfl((long long)q, src);
                bestq = rfl64(bestq);
            }
            examined += npre;
            if (best >= nice || npre < 64 || examined >= C) break;
        }
        *q_out = bestq;
        return best > b0 ? best : 0u;
    }

    // ---- block flush (_tr_flush_block) ------------------------------------------------------
    __device__ uint64_t flush_block(uint32_t ntok, uint64_t block_start, uint64_t block_end, uint64_t B,
                                    bool last, uint64_t bitpos) {
        const int l = lane_id();
        const Tables &T = c_tables;
        sync();
        // trees + sizes on lane 0
        uint32_t opt_lenb = 0, static_lenb = 0;
        int l_max = 0, d_max = 0, mbi = 0;
        stamp(2);
        if (l == 0) {
            BlockPlan p = plan_block(*tr, T);
            opt_lenb = p.opt_lenb;
            static_lenb = p.static_lenb;
            l_max = p.l_max;
            d_max = p.d_max;
            mbi = p.max_blindex;
        }
        sync();
        stamp(3);
        opt_lenb = rfl(opt_lenb);
        static_lenb = rfl(static_lenb);
        l_max = rfl(l_max);
        d_max = rfl(d_max);
        mbi = rfl(mbi);
        const uint64_t stored_len = block_end - block_start;
        const bool can_store = block_start >= B; // block bytes still in the window
        if (stored_len + 4 <= (uint64_t)opt_lenb && can_store) {
            // stored block: 3 header bits, byte align, LEN, NLEN, raw bytes
            if (l == 0) {
                LaneBits lb{outw, bitpos};
                lb.put((0u << 1) + (last ? 1u : 0u), 3);
            }
            bitpos += 3;
            bitpos = (bitpos + 7) & ~(uint64_t)7;
            uint64_t o = bitpos >> 3;
            sync();
            if (l < 4) {
                uint32_t v = l < 2 ? (uint32_t)stored_len : ~(uint32_t)stored_len;
                outb[o + l] = (uint8_t)(v >> (8 * (l & 1)));
            }
            for (uint64_t k = l; k < stored_len; k += 64) outb[o + 4 + k] = b[block_start + k];
            bitpos += (4 + stored_len) * 8;
            sync();
        } else {
            const bool fixed = static_lenb == opt_lenb;
            const CtData *lt = fixed ? T.static_ltree : tr->ltree;
            const CtData *dt = fixed ? T.static_dtree : tr->dtree;
            uint64_t hb = 0;
            if (l == 0) {
                LaneBits lb{outw, bitpos};
                lb.put(((fixed ? 1u : 2u) << 1) + (last ? 1u : 0u), 3);
                if (!fixed) {
                    BlockPlan p{opt_lenb, static_lenb, l_max, d_max, mbi};
                    send_all_trees(*tr, T, lb, p);
                }
                hb = lb.pos;
            }
            bitpos = rfl64(hb);
            sync();
            // symbols: 64 per step, bits by wave prefix sum, OR'ed into the image
            for (uint32_t t0 = 0; t0 < ntok; t0 += 64) {
                uint32_t t = t0 + (uint32_t)l;
                int nb = 0;
                uint64_t v = 0;
                if (t < ntok) v = token_bits(T, lt, dt, tok[t], nb);
                uint32_t incl = wave_incl_scan((uint32_t)nb);
                if (nb) or_bits(outw, bitpos + incl - (uint32_t)nb, v, nb);
                bitpos += rfl(__shfl(incl, 63));
            }
            sync();
            if (l == 0) {
                LaneBits lb{outw, bitpos};
                lb.put(lt[kEndBlock].fc, lt[kEndBlock].dl);
            }
            bitpos += lt[kEndBlock].dl;
            if (last) bitpos = (bitpos + 7) & ~(uint64_t)7;
            sync();
        }
        // init_block
        for (int n = l; n < kLCodes; n += 64) tr->ltree[n].fc = 0;
        if (l < kDCodes) tr->dtree[l].fc = 0;
        if (l < kBLCodes) tr->bltree[l].fc = 0;
        sync();
        if (l == 0) tr->ltree[kEndBlock].fc = 1;
        sync();
        stamp(4);
        return bitpos;
    }

    // ---- large values: the stitched token stream of pmc_deflate_large.hip ----------------------------
    // Blocks of 16383 symbols (zlib's lit_bufsize - 1: _tr_tally reports the flush at the 16383rd),
    // then the rest (possibly none) as the last block, each through flush_block.  Histograms are
    // counted by LDS atomics as the tokens are copied to the wave's slab; token positions follow from
    // a prefix sum of their lengths.  `hist`: 320 u32 of LDS (lit/len | dist).
    __device__ int run_lv(const uint8_t *src, uint64_t len, uint8_t *dst, uint32_t dst_cap, uint32_t *dst_len,
                          const LargeArgs &L, uint32_t ov, PMC_LDS uint32_t *hist) {
        const int l = lane_id();
        const Tables &T = c_tables;
        const uint32_t crc = wave_crc32(src, (uint32_t)len, crc_tab);
        for (uint64_t k = l; k < out_words; k += 64) outw[k] = 0;
        for (int k = l; k < 320; k += 64) hist[k] = 0;
        sync();
        if (l < 10) {
            const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 2, 3};
            outb[l] = hdr[l];
        }
        sync();
        uint64_t bitpos = 80, pos = 0, block_start = 0, last_start = 0;
        uint32_t ntok = 0;
        auto flush = [&](bool last) {
            // freqs -> the trees (init_block: END_BLOCK counted once)
            for (int s = l; s < kLCodes; s += 64) tr->ltree[s].fc = (uint16_t)(s == kEndBlock ? 1u : hist[s]);
            if (l < kDCodes) tr->dtree[l].fc = (uint16_t)hist[kLCodes + l];
            if (l < kBLCodes) tr->bltree[l].fc = 0;
            sync();
            // the window base at the flush's loop top (fill_window's slides so far): a stored block needs
            // its bytes still in the window (deflate.c _tr_flush_block's buf != NULL)
            const uint64_t t = last ? len : last_start + 1;
            uint64_t B = 0;
            for (;;) {
                const uint64_t wend = len < B + 2 * kWSize ? len : B + 2 * kWSize;
                if (t - B >= kWSize + kMaxDist && t + kMinLookahead > wend) B += kWSize;
                else break;
            }
            wave_sync_global(); // slab stores visible to the emitting lanes
            bitpos = flush_block(ntok, block_start, pos, B, last, bitpos);
            block_start = pos;
            ntok = 0;
            for (int k = l; k < 320; k += 64) hist[k] = 0;
            sync();
        };
        const uint32_t g0 = L.lv_seg0[ov], g1 = L.lv_seg0[ov + 1];
        for (uint32_t g = g0; g < g1; g++) {
            const uint32_t *tk = L.tok + L.seg_tok0[g];
            uint32_t t = L.seg_tok[(uint64_t)g * 4 + 1];
            const uint32_t te = L.seg_tok[(uint64_t)g * 4 + 2];
            while (t < te) {
                uint32_t take = te - t < 64 ? te - t : 64;
                take = take < kSymsPerBlock - ntok ? take : kSymsPerBlock - ntok;
                const bool in = (uint32_t)l < take;
                const uint32_t x = in ? tk[t + l] : 0u, dist = x >> 16, lc = x & 0xff;
                if (in) {
                    tok[ntok + l] = x;
                    if (dist) {
                        lds_add(&hist[T.length_code[lc] + kLiterals + 1], 1u);
                        lds_add(&hist[kLCodes + d_code(T, dist - 1)], 1u);
                    } else {
                        lds_add(&hist[lc], 1u);
                    }
                }
                const uint32_t tl = in ? (dist ? lc + kMinMatch : 1u) : 0u;
                const uint32_t incl = wave_incl_scan_dpp(tl);
                last_start = pos + readlane(incl - tl, (int)take - 1);
                pos += readlane(incl, 63);
                ntok += take;
                t += take;
                // zlib's deflate_slow tallies a value's last literal after its loop, where a full symbol buffer
                // does not flush (deflate.c: _tr_tally_lit, then FLUSH_BLOCK(s, 1)): when that literal is the
                // block's 16383rd symbol it ends the final block, not a block of its own before an empty one
                const bool tail_lit = pos == len && readlane(dist, (int)take - 1) == 0u;
                if (ntok == kSymsPerBlock && !tail_lit) flush(false);
            }
        }
        flush(true);
        uint64_t nbytes = bitpos >> 3;
        if (l < 8) {
            uint32_t v = l < 4 ? crc : (uint32_t)len;
            outb[nbytes + l] = (uint8_t)(v >> (8 * (l & 3)));
        }
        nbytes += 8;
        sync();
        if (nbytes > dst_cap || pos != len) return pos != len ? kDeflateRetry : PMC_E_CAPACITY_DEV;
        if ((((uintptr_t)dst) & 3) == 0) {
            uint32_t *d4 = reinterpret_cast<uint32_t *>(dst);
            uint64_t full = nbytes >> 2;
            for (uint64_t k = l; k < full; k += 64) d4[k] = outw[k];
            if ((uint64_t)l < (nbytes & 3)) dst[full * 4 + l] = outb[full * 4 + l];
        } else {
            for (uint64_t k = l; k < nbytes; k += 64) dst[k] = outb[k];
        }
        if (l == 0) *dst_len = (uint32_t)nbytes;
        return 0;
    }

    // ---- one value -------------------------------------------------------------------------
    __device__ int run(const uint8_t *src, uint64_t len, uint8_t *dst, uint32_t dst_cap, uint32_t *dst_len) {
        const int l = lane_id();
        // 1. stage bytes (+32 zero bytes) and zero the output image
        const uint64_t padded = (len + 32) & ~(uint64_t)3;
        if ((((uintptr_t)src) & 3) == 0) {
            const uint32_t *s4 = reinterpret_cast<const uint32_t *>(src);
            uint64_t full = len >> 2;
            for (uint64_t k = l; k < padded / 4; k += 64) bw[k] = k < full ? s4[k] : 0u;
            sync();
            if (l < 4 && (full * 4 + l) < len) b[full * 4 + l] = src[full * 4 + l];
        } else {
            for (uint64_t k = l; k < padded / 4; k += 64) bw[k] = 0;
            sync();
            for (uint64_t k = l; k < len; k += 64) b[k] = src[k];
        }
        sync();
        const uint32_t crc = wave_crc32(b, (uint32_t)len, crc_tab);
        stamp(0);
        // 2. hash + sort
        const uint64_t npos = len >= kMinMatch ? len - (kMinMatch - 1) : 0;
        if (npos) sort_positions(npos);
        for (uint64_t k = l; k < out_words; k += 64) outw[k] = 0;
        sync();
        stamp(1);
        if (l < 10) {
            const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 2, 3};
            outb[l] = hdr[l];
        }
        sync();
        // 3+4. deflate_slow
        uint64_t bitpos = 80, i = 0, B = 0, wend = 0, block_start = 0;
        uint32_t match_length = kMinMatch - 1, prev_length, ntok = 0, treg = 0;
        uint64_t match_start = 0, prev_match;
        bool match_available = false;
        auto emit = [&](uint32_t token) {
            if ((uint32_t)l == (ntok & 63)) treg = token;
            if ((ntok & 63) == 63) tok[ntok - 63 + l] = treg;
            if (l == 0) {
                uint32_t dist = token >> 16, lc = token & 0xff;
                if (dist == 0) {
                    tr->ltree[lc].fc++;
                } else {
                    tr->ltree[c_tables.length_code[lc] + kLiterals + 1].fc++;
                    tr->dtree[d_code(c_tables, dist - 1)].fc++;
                }
            }
            ntok++;
        };
        auto flush = [&](uint64_t end, bool last) {
            if ((ntok & 63) != 0 && (uint32_t)l < (ntok & 63)) tok[(ntok & ~63u) + l] = treg;
            wave_sync_global(); // slab stores visible to the emitting lanes
            bitpos = flush_block(ntok, block_start, end, B, last, bitpos);
            block_start = end;
            ntok = 0;
        };
        for (;;) {
            if (wend - i < kMinLookahead) { // fill_window bookkeeping (slides only past 64 KiB)
                do {
                    if (i - B >= kWSize + kMaxDist) B += kWSize;
                    if (wend == len) break;
                    wend = len < B + 2 * kWSize ? len : B + 2 * kWSize;
                } while (wend - i < kMinLookahead && wend < len);
                if (wend == i) break;
            }
            prev_length = match_length;
            prev_match = match_start;
            match_length = kMinMatch - 1;
            if (i + kMinMatch <= len && prev_length < kMaxLazy) {
                uint64_t q = 0;
                uint32_t m = search(i, prev_length, B, len, &q);
                if (m) {
                    match_length = m;
                    match_start = q;
                    if (m == kMinMatch && i - q > kTooFar) match_length = kMinMatch - 1;
                }
            }
            if (prev_length >= kMinMatch && match_length <= prev_length) {
                emit(((uint32_t)(i - 1 - prev_match) << 16) | (prev_length - kMinMatch));
                i += prev_length - 1;
                match_available = false;
                match_length = kMinMatch - 1;
                if (ntok == kSymsPerBlock) flush(i, false);
            } else if (match_available) {
                emit(b[i - 1]);
                if (ntok == kSymsPerBlock) flush(i, false);
                i++;
            } else {
                match_available = true;
                i++;
            }
        }
        if (match_available) emit(b[i - 1]);
        flush(i, true);
        // 5. trailer + copy-out
        uint64_t nbytes = bitpos >> 3;
        if (l < 8) {
            uint32_t v = l < 4 ? crc : (uint32_t)len;
            outb[nbytes + l] = (uint8_t)(v >> (8 * (l & 3)));
        }
        nbytes += 8;
        sync();
        if (nbytes > dst_cap) return PMC_E_CAPACITY_DEV;
        if ((((uintptr_t)dst) & 3) == 0) {
            uint32_t *d4 = reinterpret_cast<uint32_t *>(dst);
            uint64_t full = nbytes >> 2;
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

// ---------------------------------------------------------------------------------
// Persistent kernel: wave w of the grid handles values w, w + nwaves, ...
// kHbm=false: working set in dynamic LDS (wave_bytes each) after a 1 KiB CRC table.
// kHbm=true : working set in scratch + wave * wave_bytes (HBM); CRC table still in LDS.
template <bool kHbm>
__global__ void __launch_bounds__(256) deflate_kernel(DeflateArgs a) {
    // gated launch (the retry pass of the values this call's other paths declined: a lane-order
    // guard fired, a large-pass value of several blocks, a large value whose segments did not
    // stitch): it visits the call's retry list only, and returns at once when it is empty
    const uint32_t nretry = a.gate ? a.rlist[0] : 0u;
    if (a.gate && nretry == 0) return;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint32_t *crc_tab = reinterpret_cast<uint32_t *>(lds);
    for (int k = threadIdx.x; k < 256; k += blockDim.x) crc_tab[k] = c_crc_table[k];
    __syncthreads();
    const int waves_per_block = blockDim.x / 64;
    const int wib = threadIdx.x / 64;
    const uint64_t wave = (uint64_t)blockIdx.x * waves_per_block + wib;
    const uint64_t nwaves = (uint64_t)gridDim.x * waves_per_block;
    uint8_t *base = kHbm ? a.scratch + wave * a.wave_bytes : lds + 1024 + (uint64_t)wib * a.wave_bytes;
    const DeflateLayout L = deflate_layout<kHbm>(a.cap_len);
    DeflateWave<kHbm> W;
    W.tr = reinterpret_cast<Trees *>(base + L.trees);
    W.b = base + L.bytes;
    W.bw = reinterpret_cast<uint32_t *>(base + L.bytes);
    W.S = reinterpret_cast<typename Arena<kHbm>::Key *>(base + L.S);
    W.rank = reinterpret_cast<typename Arena<kHbm>::Rank *>(base + L.rank);
    W.work = base + L.work;
    W.outw = reinterpret_cast<uint32_t *>(base + L.work);
    W.outb = base + L.work;
    W.out_words = L.out_words;
    W.tok = a.tokens + wave * kSymsPerBlock;
    W.crc_tab = crc_tab;
    for (int k = 0; k < 8; k++) W.st[k] = 0;
#ifdef PMC_STAMPS
    W.t_last = __builtin_amdgcn_s_memtime();
#endif
    // init_block once; flush_block re-initialises after each block
    const int l = lane_id();
    for (int n = l; n < kLCodes; n += 64) W.tr->ltree[n].fc = 0;
    if (l < kDCodes) W.tr->dtree[l].fc = 0;
    if (l < kBLCodes) W.tr->bltree[l].fc = 0;
    W.sync();
    if (l == 0) W.tr->ltree[kEndBlock].fc = 1;
    W.sync();
    if (a.gate) {
        for (uint64_t k = wave; k < nretry; k += nwaves) {
            const uint64_t v = a.rlist[1 + k];
            const uint64_t len = a.src_len[v];
            const int rc = W.run(a.src + a.src_off[v], len, a.dst + a.dst_off[v], a.dst_cap[v], a.dst_len + v);
            if (l == 0) {
                a.rc[v] = rc;
                if (rc) a.dst_len[v] = 0;
            }
        }
        return;
    }
    // wave w owns groups of 64 consecutive values: w, w + nwaves, ...; the lengths of a
    // group are read with one coalesced load and the values this variant handles are
    // picked out by ballot
    for (uint64_t g = wave * 64; g < a.n; g += nwaves * 64) {
      const uint64_t vl = g + (uint64_t)l;
      const uint64_t myl = vl < a.n ? a.src_len[vl] : 0;
      // values above cap_len (the call's max_len) are argument errors (arg_check_kernel)
      uint64_t todo = ballot(vl < a.n && (kHbm ? ((myl > a.lds_max_len && myl <= a.cap_len) ||
                                                   (a.retry && a.rc[vl] == kDeflateRetry))
                                                : (myl <= a.lds_max_len)));
      while (todo) {
        const uint64_t v = g + (uint64_t)__builtin_ctzll(todo);
        todo &= todo - 1;
        const uint64_t len = rfl((uint32_t)__shfl((uint32_t)myl, (int)(v - g)));
        if (len == 0) {
            if (l == 0) {
                a.rc[v] = PMC_INVALID_INPUT_DEV;
                a.dst_len[v] = 0;
            }
            continue;
        }
        int rc = W.run(a.src + a.src_off[v], len, a.dst + a.dst_off[v], a.dst_cap[v], a.dst_len + v);
        if (l == 0) {
            a.rc[v] = rc;
            if (rc) a.dst_len[v] = 0;
        }
      }
    }
#ifdef PMC_STAMPS
    if (l == 0 && a.dbg)
        for (int k = 0; k < 8; k++) atomicAdd((unsigned long long *)&a.dbg[k], (unsigned long long)W.st[k]);
#endif
}

template __global__ void deflate_kernel<false>(DeflateArgs);
template __global__ void deflate_kernel<true>(DeflateArgs);

// ---- large values: one wave per value emits its stitched tokens (pmc_deflate_large.hip) -----------
// Per wave: HBM scratch = the output image | the symbol slab; LDS = the Trees (zlib's heap and the
// serial plan_block run on lane 0 against LDS, not HBM) | 320 histogram counters.
constexpr uint64_t kLvTreesBytes = (sizeof(Trees) + 15) & ~(uint64_t)15;
constexpr uint64_t kLvEmitLdsPerWave = kLvTreesBytes + 320 * 4;
uint64_t deflate_lv_emit_wave_bytes(uint64_t n) { return align16(gzip_bound(n) + 16) + (uint64_t)kSlabSyms * 4; }
uint64_t deflate_lv_emit_lds(int waves) { return 1024 + (uint64_t)waves * kLvEmitLdsPerWave; }

__global__ void __launch_bounds__(256) deflate_lv_emit_kernel(DeflateArgs a, LargeArgs L) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint32_t *crc_tab = reinterpret_cast<uint32_t *>(lds);
    for (int k = threadIdx.x; k < 256; k += blockDim.x) crc_tab[k] = c_crc_table[k];
    __syncthreads();
    const int wpb = blockDim.x / 64, wib = threadIdx.x / 64, l = lane_id();
    const uint64_t wave = (uint64_t)blockIdx.x * wpb + wib, nwaves = (uint64_t)gridDim.x * wpb;
    uint8_t *wl = lds + 1024 + (uint64_t)wib * kLvEmitLdsPerWave;
    uint8_t *base = a.scratch + wave * a.wave_bytes;
    DeflateWave<true> W;
    W.tr = reinterpret_cast<Trees *>(wl);
    W.out_words = align16(gzip_bound(a.cap_len) + 16) / 4;
    W.outw = reinterpret_cast<uint32_t *>(base);
    W.outb = base;
    W.tok = reinterpret_cast<uint32_t *>(base + W.out_words * 4);
    W.crc_tab = crc_tab;
    for (int k = 0; k < 8; k++) W.st[k] = 0;
    PMC_LDS uint32_t *hist = to_lds<uint32_t>(wl + kLvTreesBytes);
    for (uint64_t ov = wave; ov < L.nv; ov += nwaves) {
        const uint32_t v = L.lv_val[ov];
        const uint64_t len = a.src_len[v];
        int rc = kDeflateRetry;
        if (!L.fail[ov]) {
            W.b = const_cast<uint8_t *>(a.src + a.src_off[v]);
            W.out_words = align16(gzip_bound(len) + 16) / 4;
            rc = W.run_lv(a.src + a.src_off[v], len, a.dst + a.dst_off[v], a.dst_cap[v], a.dst_len + v, L, (uint32_t)ov,
                          hist);
        }
        if (l == 0) {
            a.rc[v] = rc;
            if (rc) a.dst_len[v] = 0;
            if (rc == kDeflateRetry) { // (the HBM kernel redoes the value)
                atomicAdd(a.guard + 3, 1u);
                retry_push(a, v);
            }
        }
    }
}

} // namespace pmc
