// pmc_inflate.hip -- batched gzip decompression on gfx950.
//
// Replaces GzipCompressor::Decompress (/root/reference/src/compressor/gzip_compressor.cpp:52-111,
// called from src/kvs/kvs.cpp:233) for many independent gzip members at once, with the
// validation verdicts of zlib 1.2.11 inflateInit2(15+16) (see oracle/inflate.c for the
// rule list): -3 for any corruption / CRC / ISIZE mismatch, -5 for truncated input (the
// reference hangs there), 0 on success.
//
// One wave64 per member (persistent grid).  Per member:
//   1. stage the compressed bytes in LDS (coalesced), lane 0 parses the gzip header
//   2. per block: stored -> lane-parallel copy; fixed/dynamic -> decode tables in LDS
//      (9-bit root lookup, canonical fallback for longer codes; built by the wave)
//   3. lane 0 decodes up to 64 tokens (literal / length+distance) into LDS; the wave then
//      materialises them: all literals of the batch in parallel, then each match copied
//      lane-parallel (period replication when distance < length)
//   4. CRC-32 of the output lane-parallel, ISIZE check, copy-out to HBM.
// Members whose output does not fit the LDS image use the same code with the output
// image written straight into dst (kHbm variant).
#include <hip/hip_runtime.h>

#include "pmc_device.hpp"
#include "pmc_kernels.hpp"

namespace pmc {

constexpr int kRootBits = 9;
constexpr uint16_t kEntLong = 0xFFFF, kEntInvalid = 0xFFFE;

__constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27,
                                     31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
                                     257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_cl_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Canonical decoder for one code (zlib inftrees semantics for validity).
struct Huff {
    uint16_t count[16];
    uint16_t offs[16];
    uint16_t symbol[288];
    uint16_t fast[1 << kRootBits]; // sym | len << 9, kEntLong, kEntInvalid
    int32_t max;                   // longest code length, 0 = no codes
    int32_t pad_;
};

struct InflateScratch {
    Huff lit, dist, cl;
    uint16_t lens[320];
    uint32_t tok[64];  // literal: byte; match: 1<<31 | (dist-1)<<8 | (len-3)
    uint32_t tpos[64]; // output position of each token (low 32 bits of the running count)
    int32_t status[4]; // [0] batch status from lane 0
};

__host__ __device__ inline uint64_t a16(uint64_t x) { return (x + 15) & ~(uint64_t)15; }

struct InflateLayout {
    uint64_t scr, in, out, total;
};
template <bool kHbm>
__host__ __device__ inline InflateLayout inflate_layout(uint64_t max_out, uint64_t max_in) {
    InflateLayout L;
    uint64_t off = 0;
    L.scr = off;
    off += a16(sizeof(InflateScratch));
    L.in = off;
    off += kHbm ? 0 : a16(max_in + 32);
    L.out = off;
    off += kHbm ? 0 : a16(max_out + 16);
    L.total = a16(off);
    return L;
}

// Build count/offs/symbol (lane 0) and the fast table (wave).  Returns 0 or -1 (inftrees
// over-subscribed / incomplete rule); is_codes selects the stricter code-length-code rule.
__device__ inline int huff_build(Huff &h, const uint16_t *lens, int n, bool is_codes) {
    const int l = lane_id();
    int bad = 0;
    if (l == 0) {
        for (int k = 0; k < 16; k++) h.count[k] = 0;
        for (int s = 0; s < n; s++) h.count[lens[s]]++;
        int mx = 0;
        for (int len = 15; len >= 1; len--)
            if (h.count[len]) {
                mx = len;
                break;
            }
        h.max = mx;
        if (mx) {
            int left = 1;
            for (int len = 1; len <= 15; len++) {
                left <<= 1;
                left -= h.count[len];
                if (left < 0) bad = 1;
            }
            if (!bad && left > 0 && (is_codes || mx != 1)) bad = 1;
            h.offs[1] = 0;
            for (int len = 1; len < 15; len++) h.offs[len + 1] = (uint16_t)(h.offs[len] + h.count[len]);
            uint16_t o[16];
            for (int k = 0; k < 16; k++) o[k] = h.offs[k];
            for (int s = 0; s < n; s++)
                if (lens[s]) h.symbol[o[lens[s]]++] = (uint16_t)s;
        }
    }
    wave_sync();
    bad = rfl(bad);
    if (bad) return -1;
    const int mx = rfl(h.max);
    // every root entry starts invalid (incomplete codes, or no codes at all)
    for (int e = l; e < (1 << kRootBits); e += 64) h.fast[e] = kEntInvalid;
    wave_sync();
    if (mx == 0) return 0;
    // canonical code of the j-th symbol of length L: first[L] + (j - offs[L])
    uint32_t nsym = h.offs[15] + h.count[15];
    for (uint32_t j = l; j < nsym; j += 64) {
        int s = h.symbol[j];
        int L = lens[s];
        uint32_t first = 0, code = 0;
        for (int k = 1; k <= L; k++) { // first code of length k (canonical)
            first = (first + (k > 1 ? h.count[k - 1] : 0)) << (k > 1 ? 1 : 0);
        }
        code = first + (j - h.offs[L]);
        uint32_t rev = __builtin_bitreverse32(code) >> (32 - L);
        if (L <= kRootBits) {
            for (uint32_t e = rev; e < (1u << kRootBits); e += (1u << L)) h.fast[e] = (uint16_t)(s | (L << 9));
        } else {
            h.fast[rev & ((1u << kRootBits) - 1)] = kEntLong;
        }
    }
    wave_sync();
    return 0;
}

// Lane-0 bit reader over a byte stream with a truncation check.  kWords: the stream is
// LDS-staged, 4-byte aligned and zero padded, so a 64-bit window is 3 aligned dwords;
// otherwise (HBM variant) bytes are fetched individually with a bounds check.
template <bool kWords>
struct Bits {
    const uint8_t *in;
    uint64_t nbits; // total bits available
    uint64_t pos;   // bits consumed
    __device__ uint64_t peek64() const {
        if (kWords) {
            const uint32_t *w = reinterpret_cast<const uint32_t *>(in);
            uint64_t wi = pos >> 5;
            uint32_t s = (uint32_t)(pos & 31);
            uint64_t lo = ((uint64_t)w[wi + 1] << 32) | w[wi];
            uint64_t v = lo >> s;
            if (s) v |= (uint64_t)w[wi + 2] << (64 - s);
            return v;
        }
        uint64_t byte = pos >> 3, nb = (nbits + 7) >> 3;
        uint64_t v = 0;
#pragma unroll
        for (int k = 0; k < 9; k++) {
            uint64_t bb = byte + k < nb ? in[byte + k] : 0;
            v |= k < 8 ? bb << (8 * k) : 0;
            if (k == 8 && (pos & 7)) v = (v >> (pos & 7)) | (bb << (64 - (pos & 7)));
        }
        return v;
    }
    __device__ bool need(uint64_t n) const { return pos + n <= nbits; }
    __device__ uint32_t get(uint32_t n) {
        uint32_t v = (uint32_t)(peek64() & ((n >= 32) ? 0xffffffffull : ((1ull << n) - 1)));
        pos += n;
        return v;
    }
};

// Decode one symbol: >=0 symbol, -1 invalid, -2 truncated.
template <bool kW>
__device__ inline int decode_sym(Bits<kW> &br, const Huff &h) {
    uint64_t w = br.peek64();
    uint16_t e = h.fast[w & ((1u << kRootBits) - 1)];
    if (e != kEntLong) {
        if (e == kEntInvalid) {
            if (!br.need(1)) return -2;
            return -1;
        }
        uint32_t L = e >> 9;
        if (!br.need(L)) return -2;
        br.pos += L;
        return e & 0x1ff;
    }
    int code = 0, first = 0, index = 0;
    for (int len = 1; len <= 15; len++) {
        code |= (int)((w >> (len - 1)) & 1);
        int count = h.count[len];
        if (code - count < first) {
            if (!br.need((uint32_t)len)) return -2;
            br.pos += (uint64_t)len;
            return h.symbol[index + (code - first)];
        }
        index += count;
        first += count;
        first <<= 1;
        code <<= 1;
    }
    return -1;
}

template <bool kHbm>
struct InflateWave {
    InflateScratch *sc;
    uint8_t *inb; // staged input (LDS) or src (HBM variant)
    uint8_t *out; // output image (LDS) or dst (HBM variant)
    const uint32_t *crc_tab;
    uint64_t st[8];
    uint64_t t_last;

    // PMC_STAMPS: 0 stage+header, 1 block headers + code lengths, 2 table builds,
    // 3 symbol decode, 4 materialise, 5 trailer (CRC) + copy-out
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

    // materialise the token batch [0, nt): literals in parallel, then matches in order
    __device__ void materialise(int nt, uint64_t base, uint64_t cap) {
        const int l = lane_id();
        if (l < nt) {
            uint32_t t = sc->tok[l];
            uint64_t p = base + sc->tpos[l];
            if (!(t >> 31) && p < cap) out[p] = (uint8_t)t;
        }
        sync();
        for (int j = 0; j < nt; j++) {
            uint32_t t = sc->tok[j];
            if (!(t >> 31)) continue;
            const uint32_t len = (t & 0xff) + 3, dist = ((t >> 8) & 0x7fff) + 1;
            uint64_t p = base + sc->tpos[j];
            for (uint32_t k = l; k < len; k += 64) {
                uint64_t sidx = dist >= len ? p - dist + k : p - dist + (k % dist);
                if (p + k < cap) out[p + k] = sidx < cap ? out[sidx] : 0;
            }
            sync();
        }
    }

    __device__ int run(const uint8_t *src, uint64_t in_len, uint8_t *dst, uint64_t cap, uint32_t *dst_len) {
        const int l = lane_id();
        // 1. stage input (zero padded)
        if (!kHbm) {
            const uint64_t padded = (in_len + 16) & ~(uint64_t)3;
            uint32_t *iw = reinterpret_cast<uint32_t *>(inb);
            if ((((uintptr_t)src) & 3) == 0) {
                const uint32_t *s4 = reinterpret_cast<const uint32_t *>(src);
                uint64_t full = in_len >> 2;
                for (uint64_t k = l; k < padded / 4; k += 64) iw[k] = k < full ? s4[k] : 0u;
                sync();
                if ((uint64_t)l < (in_len & 3)) inb[full * 4 + l] = src[full * 4 + l];
            } else {
                for (uint64_t k = l; k < padded / 4; k += 64) iw[k] = 0;
                sync();
                for (uint64_t k = l; k < in_len; k += 64) inb[k] = src[k];
            }
            sync();
        }
        // 2. gzip header (lane 0)
        int hrc = 0;
        uint64_t p = 0;
        if (l == 0) {
            const uint8_t *in = inb;
            do {
                if (in_len < 2) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                if (in[0] != 0x1f || in[1] != 0x8b) { hrc = PMC_Z_DATA_ERROR_DEV; break; }
                if (in_len < 4) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                if (in[2] != 8) { hrc = PMC_Z_DATA_ERROR_DEV; break; }
                uint32_t flg = in[3];
                if (flg & 0xe0) { hrc = PMC_Z_DATA_ERROR_DEV; break; }
                if (in_len < 10) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                p = 10;
                if (flg & 0x04) {
                    if (in_len < p + 2) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                    uint64_t xlen = in[p] | ((uint64_t)in[p + 1] << 8);
                    p += 2;
                    if (in_len < p + xlen) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                    p += xlen;
                }
                if (flg & 0x08) {
                    while (p < in_len && in[p] != 0) p++;
                    if (p >= in_len) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                    p++;
                }
                if (flg & 0x10) {
                    while (p < in_len && in[p] != 0) p++;
                    if (p >= in_len) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                    p++;
                }
                if (flg & 0x02) {
                    if (in_len < p + 2) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                    uint32_t hc = in[p] | ((uint32_t)in[p + 1] << 8), c = 0xFFFFFFFFu;
                    for (uint64_t k = 0; k < p; k++) c = crc_tab[(c ^ in[k]) & 0xff] ^ (c >> 8);
                    if (hc != ((~c) & 0xffff)) { hrc = PMC_Z_DATA_ERROR_DEV; break; }
                    p += 2;
                }
            } while (0);
        }
        hrc = rfl(hrc);
        if (hrc) return hrc;
        p = rfl64(p);
        stamp(0);
        Bits<!kHbm> br{inb, in_len * 8, p * 8};
        uint64_t outn = 0; // bytes produced (uniform)
        int last = 0;
        do {
            // ---- block header (lane 0) ----
            int type = 0, rc = 0;
            if (l == 0) {
                if (!br.need(3)) rc = PMC_Z_BUF_ERROR_DEV;
                else {
                    last = (int)br.get(1);
                    type = (int)br.get(2);
                }
            }
            rc = rfl(rc);
            if (rc) return rc;
            last = rfl(last);
            type = rfl(type);
            br.pos = rfl64(br.pos);
            if (type == 0) {
                // stored
                uint32_t len = 0;
                if (l == 0) {
                    br.pos = (br.pos + 7) & ~(uint64_t)7;
                    if (!br.need(32)) rc = PMC_Z_BUF_ERROR_DEV;
                    else {
                        len = br.get(16);
                        uint32_t nlen = br.get(16);
                        if (len != (nlen ^ 0xffff)) rc = PMC_Z_DATA_ERROR_DEV;
                        else if (!br.need(8ull * len)) rc = PMC_Z_BUF_ERROR_DEV;
                    }
                }
                rc = rfl(rc);
                if (rc) return rc;
                len = rfl(len);
                br.pos = rfl64(br.pos);
                const uint64_t ib = br.pos >> 3;
                for (uint64_t k = l; k < len; k += 64)
                    if (outn + k < cap) out[outn + k] = inb[ib + k];
                outn += len;
                br.pos += 8ull * len;
                sync();
                continue;
            }
            if (type == 3) return PMC_Z_DATA_ERROR_DEV;
            if (type == 1) {
                // fixed code lengths (inflate.c fixedtables)
                for (int s = l; s < 320; s += 64) sc->lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
                sync();
                stamp(1);
                huff_build(sc->lit, sc->lens, 288, false);
                huff_build(sc->dist, sc->lens + 288, 32, false);
                stamp(2);
            } else {
                // dynamic: HLIT/HDIST/HCLEN, code-length code, then the code lengths
                int nlen = 0, ndist = 0, ncode = 0;
                if (l == 0) {
                    if (!br.need(14)) rc = PMC_Z_BUF_ERROR_DEV;
                    else {
                        nlen = (int)br.get(5) + 257;
                        ndist = (int)br.get(5) + 1;
                        ncode = (int)br.get(4) + 4;
                        if (nlen > 286 || ndist > 30) rc = PMC_Z_DATA_ERROR_DEV;
                        else {
                            int k;
                            for (k = 0; k < ncode; k++) {
                                if (!br.need(3)) {
                                    rc = PMC_Z_BUF_ERROR_DEV;
                                    break;
                                }
                                sc->lens[c_cl_order[k]] = (uint16_t)br.get(3);
                            }
                            for (; k < 19; k++) sc->lens[c_cl_order[k]] = 0;
                        }
                    }
                }
                rc = rfl(rc);
                if (rc) return rc;
                sync();
                stamp(1);
                if (huff_build(sc->cl, sc->lens, 19, true)) return PMC_Z_DATA_ERROR_DEV;
                stamp(2);
                nlen = rfl(nlen);
                ndist = rfl(ndist);
                if (l == 0) {
                    const int clmax = sc->cl.max;
                    int have = 0;
                    while (have < nlen + ndist) {
                        int sym;
                        if (clmax == 0) {
                            if (!br.need(1)) { rc = PMC_Z_BUF_ERROR_DEV; break; }
                            br.pos += 1;
                            sym = 0;
                        } else {
                            sym = decode_sym(br, sc->cl);
                            if (sym == -2) { rc = PMC_Z_BUF_ERROR_DEV; break; }
                            if (sym < 0) { rc = PMC_Z_DATA_ERROR_DEV; break; }
                        }
                        if (sym < 16) {
                            sc->lens[have++] = (uint16_t)sym;
                        } else {
                            uint32_t len = 0, copy;
                            if (sym == 16) {
                                if (!br.need(2)) { rc = PMC_Z_BUF_ERROR_DEV; break; }
                                if (have == 0) { rc = PMC_Z_DATA_ERROR_DEV; break; }
                                len = sc->lens[have - 1];
                                copy = 3 + br.get(2);
                            } else if (sym == 17) {
                                if (!br.need(3)) { rc = PMC_Z_BUF_ERROR_DEV; break; }
                                copy = 3 + br.get(3);
                            } else {
                                if (!br.need(7)) { rc = PMC_Z_BUF_ERROR_DEV; break; }
                                copy = 11 + br.get(7);
                            }
                            if (have + (int)copy > nlen + ndist) { rc = PMC_Z_DATA_ERROR_DEV; break; }
                            while (copy--) sc->lens[have++] = (uint16_t)len;
                        }
                    }
                    if (!rc && sc->lens[256] == 0) rc = PMC_Z_DATA_ERROR_DEV;
                    // move distance lengths to lens[288..]
                    if (!rc) {
                        for (int k = ndist - 1; k >= 0; k--) sc->lens[288 + k] = sc->lens[nlen + k];
                        for (int k = nlen; k < 288; k++) sc->lens[k] = 0;
                    }
                }
                rc = rfl(rc);
                if (rc) return rc;
                br.pos = rfl64(br.pos);
                sync();
                stamp(1);
                if (huff_build(sc->lit, sc->lens, nlen, false)) return PMC_Z_DATA_ERROR_DEV;
                if (huff_build(sc->dist, sc->lens + 288, ndist, false)) return PMC_Z_DATA_ERROR_DEV;
                stamp(2);
            }
            // ---- symbol decode (lane 0) + materialisation (wave) ----
            for (;;) {
                int nt = 0, st = 0; // st: 0 more, 1 end of block, <0 error
                uint32_t rel = 0;
                if (l == 0) {
                    const uint64_t o0 = outn;
                    uint64_t o = outn;
                    while (nt < 64) {
                        int sym = decode_sym(br, sc->lit);
                        if (sym == -2) { st = PMC_Z_BUF_ERROR_DEV; break; }
                        if (sym < 0) { st = PMC_Z_DATA_ERROR_DEV; break; }
                        if (sym < 256) {
                            sc->tok[nt] = (uint32_t)sym;
                            sc->tpos[nt] = (uint32_t)(o - o0);
                            nt++;
                            o++;
                            continue;
                        }
                        if (sym == 256) { st = 1; break; }
                        sym -= 257;
                        if (sym >= 29) { st = PMC_Z_DATA_ERROR_DEV; break; }
                        if (!br.need(c_lext[sym])) { st = PMC_Z_BUF_ERROR_DEV; break; }
                        uint32_t len = c_lbase[sym] + br.get(c_lext[sym]);
                        int ds = decode_sym(br, sc->dist);
                        if (ds == -2) { st = PMC_Z_BUF_ERROR_DEV; break; }
                        if (ds < 0 || ds >= 30) { st = PMC_Z_DATA_ERROR_DEV; break; }
                        if (!br.need(c_dext[ds])) { st = PMC_Z_BUF_ERROR_DEV; break; }
                        uint32_t dist = c_dbase[ds] + br.get(c_dext[ds]);
                        if (dist > o) { st = PMC_Z_DATA_ERROR_DEV; break; }
                        // match token: bit 31 | (dist-1) << 8 | (len-3)
                        sc->tok[nt] = 0x80000000u | (dist - 1) << 8 | (len - 3);
                        sc->tpos[nt] = (uint32_t)(o - o0);
                        nt++;
                        o += len;
                    }
                    rel = (uint32_t)(o - o0);
                }
                nt = rfl(nt);
                st = rfl(st);
                rel = rfl(rel);
                br.pos = rfl64(br.pos);
                sync();
                stamp(3);
                materialise(nt, outn, cap);
                stamp(4);
                outn += rel;
                if (st < 0) return st;
                if (st == 1) break;
            }
        } while (!last);
        // 3. trailer: CRC-32 then ISIZE (inflate.c CHECK / LENGTH)
        uint64_t tp = (br.pos + 7) >> 3;
        if (in_len < tp + 4) return PMC_Z_BUF_ERROR_DEV;
        if (outn > cap) { // a valid stream so far that needs more room: report the size (no verdict yet)
            if (l == 0) *dst_len = outn > 0xffffffffull ? 0xffffffffu : (uint32_t)outn;
            return PMC_E_CAPACITY_DEV;
        }
        sync();
        uint32_t crc = wave_crc32(out, (uint32_t)outn, crc_tab);
        uint32_t want = inb[tp] | ((uint32_t)inb[tp + 1] << 8) | ((uint32_t)inb[tp + 2] << 16) | ((uint32_t)inb[tp + 3] << 24);
        if (crc != want) return PMC_Z_DATA_ERROR_DEV;
        if (in_len < tp + 8) return PMC_Z_BUF_ERROR_DEV;
        uint32_t isz = inb[tp + 4] | ((uint32_t)inb[tp + 5] << 8) | ((uint32_t)inb[tp + 6] << 16) | ((uint32_t)inb[tp + 7] << 24);
        if (isz != (uint32_t)outn) return PMC_Z_DATA_ERROR_DEV;
        // 4. copy-out
        if (!kHbm) {
            if ((((uintptr_t)dst) & 3) == 0) {
                uint32_t *d4 = reinterpret_cast<uint32_t *>(dst);
                const uint32_t *o4 = reinterpret_cast<const uint32_t *>(out);
                uint64_t full = outn >> 2;
                for (uint64_t k = l; k < full; k += 64) d4[k] = o4[k];
                if ((uint64_t)l < (outn & 3)) dst[full * 4 + l] = out[full * 4 + l];
            } else {
                for (uint64_t k = l; k < outn; k += 64) dst[k] = out[k];
            }
        }
        if (l == 0) *dst_len = (uint32_t)outn;
        stamp(5);
        return 0;
    }
};

// =====================================================================================
// LDS-resident members (the hot path).  Same verdicts and bit consumption order as the
// general InflateWave above (oracle/inflate.c), organised for latency:
//  * headers and code lengths: wave-uniform bit buffer in SGPRs; the code-length code's
//    7-bit table lives in two VGPRs (v_readlane lookup, no LDS round trip per symbol);
//  * code tables: built by the whole wave (per-length counts and in-length ranks by
//    ballot, canonical codes by shuffle) -- no serial per-symbol loop;
//  * literal/length + distance symbols: every lane decodes at one of the 64 bit offsets
//    W + lane of a window (two LDS round trips per window), then a scalar chase walks the
//    tokens through the window with v_readlane only;
//  * tokens of a batch stay in VGPRs (lane t holds token t) until materialised.
// =====================================================================================
struct InfTables {
    uint16_t lfast[1 << kRootBits]; // lit/len root table: sym | len << 9, kEntLong, kEntInvalid
    uint16_t dfast[1 << kRootBits];
    uint16_t lsym[288]; // canonical symbol order (read only for codes longer than the root)
    uint16_t dsym[32];
    uint16_t lens[320];
};
struct InfLdsLayout {
    uint64_t tab, in, out, total;
};
__host__ __device__ inline InfLdsLayout inf_lds_layout(uint64_t max_out, uint64_t max_in) {
    InfLdsLayout L;
    uint64_t off = 0;
    L.tab = off;
    off += a16(sizeof(InfTables));
    L.in = off;
    off += a16(max_in + 64); // zero padding: windows read up to 3 dwords past the bit position
    L.out = off;
    off += a16(max_out + 16);
    L.total = a16(off);
    return L;
}

// wave-uniform LSB-first bit reader over the LDS-staged member
struct SBits {
    PMC_LDS const uint32_t *w;
    uint64_t bb;
    uint32_t bn, wi, nbits;
    __device__ uint32_t pos() const { return wi * 32 - bn; }
    __device__ void refill() {
        if (bn <= 32) {
            bb |= (uint64_t)rfl(w[wi]) << bn;
            wi++;
            bn += 32;
        }
    }
    __device__ void seek(uint32_t p) {
        wi = p >> 5;
        bb = 0;
        bn = 0;
        refill();
        bb >>= (p & 31);
        bn -= (p & 31);
        refill(); // >= 33 bits buffered
    }
    __device__ uint32_t peek(uint32_t n) const { return (uint32_t)bb & ((1u << n) - 1); }
    __device__ void drop(uint32_t n) {
        bb >>= n;
        bn -= n;
    }
    __device__ bool need(uint32_t n) const { return pos() + n <= nbits; }
};

uint64_t inflate_wave_bytes(bool hbm, uint64_t max_out, uint64_t max_in) {
    return hbm ? inflate_layout<true>(max_out, max_in).total : inf_lds_layout(max_out, max_in).total;
}

struct InflateLds {
    PMC_LDS InfTables *T;
    PMC_LDS uint8_t *inb;
    PMC_LDS uint32_t *inw;
    PMC_LDS uint8_t *out;
    PMC_LDS const uint32_t *crc_tab;
    uint32_t lenv, distv; // lane s: base | extra bits << 16 (length codes 257+s, distance codes s)
    uint64_t st[8];
    uint64_t t_last;

    // PMC_STAMPS: 0 stage+header, 1 block headers + code lengths, 2 table builds,
    // 3 symbol decode, 4 materialise, 5 trailer (CRC) + copy-out
    __device__ void stamp(int k) {
#ifdef PMC_STAMPS
        uint64_t t = __builtin_amdgcn_s_memtime();
        st[k] += t - t_last;
        t_last = t;
#endif
    }

    // inftrees.c rules + root table for lens[0..n) (NC chunks of 64 symbols).  Returns 0 or
    // -1 (over-subscribed, or incomplete where not allowed).  cntv: lane L = count[L].
    template <int NC>
    __device__ int build(PMC_LDS const uint16_t *lens, int n, bool is_codes, PMC_LDS uint16_t *fast,
                         PMC_LDS uint16_t *symtab, uint32_t &cntv, int &maxo) {
        const int l = lane_id();
        uint32_t cnt[16];
#pragma unroll
        for (int L = 0; L < 16; L++) cnt[L] = 0;
        uint32_t lc[NC], rk[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const int s = c * 64 + l;
            const uint32_t len = s < n ? lens[s] : 0u;
            uint32_t r = 0;
#pragma unroll
            for (int L = 1; L <= 15; L++) {
                const uint64_t m = ballot(len == (uint32_t)L);
                if (len == (uint32_t)L) r = cnt[L] + popc_lt(m);
                cnt[L] += (uint32_t)__builtin_popcountll(m);
            }
            lc[c] = len;
            rk[c] = r;
        }
        int mx = 0;
#pragma unroll
        for (int L = 1; L <= 15; L++)
            if (cnt[L]) mx = L;
        maxo = mx;
        cntv = 0;
        if (mx == 0) { // no codes: every pattern is invalid (zlib's 1-bit invalid marker)
            for (int e = l; e < (1 << kRootBits); e += 64) fast[e] = kEntInvalid;
            wave_sync();
            return 0;
        }
        int left = 1;
        bool bad = false;
        uint32_t fv = 0, ov = 0, code = 0, off = 0;
#pragma unroll
        for (int L = 1; L <= 15; L++) {
            left <<= 1;
            left -= (int)cnt[L];
            bad |= left < 0;
            fv = l == L ? code : fv; // canonical first code of length L
            ov = l == L ? off : ov;  // index of its first symbol in symtab
            cntv = l == L ? cnt[L] : cntv;
            code = (code + cnt[L]) << 1;
            off += cnt[L];
        }
        if (bad || (left > 0 && (is_codes || mx != 1))) return -1;
        if (left > 0) { // incomplete (a single 1-bit code): the other half stays invalid
            for (int e = l; e < (1 << kRootBits); e += 64) fast[e] = kEntInvalid;
            wave_sync();
        }
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const uint32_t len = lc[c];
            const uint32_t f = (uint32_t)__shfl((int)fv, (int)len), o = (uint32_t)__shfl((int)ov, (int)len);
            if (len) {
                const uint32_t s = (uint32_t)(c * 64 + l);
                const uint32_t rev = __builtin_bitreverse32(f + rk[c]) >> (32 - len);
                if (len <= (uint32_t)kRootBits) {
                    const uint16_t ent = (uint16_t)(s | len << 9);
                    for (uint32_t e = rev; e < (1u << kRootBits); e += 1u << len) fast[e] = ent;
                } else {
                    fast[rev & ((1u << kRootBits) - 1)] = kEntLong;
                }
                if (mx > kRootBits) symtab[o + rk[c]] = (uint16_t)s;
            }
        }
        wave_sync();
        return 0;
    }

    // canonical decode of a code longer than the root (complete codes only: always found)
    __device__ uint32_t slow_decode(uint32_t bits, uint32_t cntv, PMC_LDS const uint16_t *symtab,
                                    uint32_t &L) {
        int code = 0, first = 0, index = 0;
        for (int len = 1; len <= 15; len++) {
            code |= (int)((bits >> (len - 1)) & 1u);
            const int count = (int)readlane(cntv, len);
            if (code - count < first) {
                L = (uint32_t)len;
                return rfl((uint32_t)symtab[index + (code - first)]);
            }
            index += count;
            first += count;
            first <<= 1;
            code <<= 1;
        }
        L = 15;
        return 0xffffu;
    }

    // lanes: 32 stream bits at W + lane, and the root-table entries they index
    __device__ void window(uint32_t W, uint32_t &bits, uint32_t &le, uint32_t &de) const {
        const uint32_t p = W + (uint32_t)lane_id();
        const uint32_t lo = inw[p >> 5], hi = inw[(p >> 5) + 1];
        bits = __builtin_amdgcn_alignbit(hi, lo, p & 31);
        le = T->lfast[bits & ((1u << kRootBits) - 1)];
        de = T->dfast[bits & ((1u << kRootBits) - 1)];
    }

    // write the tokens of the lanes in `act` (stream order = lane order): literals in one
    // store, then matches one after another (a match may read bytes the previous one wrote)
    __device__ void materialise(uint64_t actm, uint32_t tokv, uint32_t tposv, uint32_t o0, uint32_t cap) {
        const uint32_t l = (uint32_t)lane_id();
        const bool act = (actm >> l) & 1;
        const uint32_t p = o0 + tposv;
        if (act && !(tokv >> 31) && p < cap) out[p] = (uint8_t)tokv;
        uint64_t mm = ballot(act && (tokv >> 31));
        while (mm) {
            const int j = __builtin_ctzll(mm);
            mm &= mm - 1;
            const uint32_t t = readlane(tokv, j), pj = o0 + readlane(tposv, j);
            const uint32_t len = (t & 0xff) + 3, dist = ((t >> 8) & 0x7fff) + 1, src0 = pj - dist;
            if (dist >= len) {
                for (uint32_t k = l; k < len; k += 64) {
                    const uint32_t s = src0 + k;
                    const uint8_t v = s < cap ? out[s] : (uint8_t)0;
                    if (pj + k < cap) out[pj + k] = v;
                }
            } else { // overlapping copy: period dist
                for (uint32_t k = l; k < len; k += 64) {
                    const uint32_t s = src0 + k % dist;
                    const uint8_t v = s < cap ? out[s] : (uint8_t)0;
                    if (pj + k < cap) out[pj + k] = v;
                }
            }
        }
        wave_sync();
    }

    // Exact decode of the one token at bit W, with inflate.c's checks in its order.  Returns
    // 0 (token in tok/olen, W advanced), 1 (end of block, W advanced) or a verdict < 0.
    __device__ int scalar_token(uint32_t &W, uint32_t o, uint32_t nbits, uint32_t lcnt, uint32_t dcnt,
                                uint32_t &tok, uint32_t &olen) {
        uint32_t bits, le, de;
        window(W, bits, le, de);
        const uint32_t e = readlane(le, 0);
        uint32_t L, sym;
        if (e < kEntInvalid) {
            L = e >> 9;
            sym = e & 0x1ff;
        } else if (e == kEntInvalid) {
            return W + 1 > nbits ? PMC_Z_BUF_ERROR_DEV : PMC_Z_DATA_ERROR_DEV;
        } else {
            sym = slow_decode(readlane(bits, 0), lcnt, T->lsym, L);
        }
        if (W + L > nbits) return PMC_Z_BUF_ERROR_DEV;
        if (sym < 256) {
            tok = sym;
            olen = 1;
            W += L;
            return 0;
        }
        if (sym == 256) {
            W += L;
            return 1;
        }
        const uint32_t s = sym - 257;
        if (s >= 29) return PMC_Z_DATA_ERROR_DEV;
        const uint32_t lv = readlane(lenv, (int)s), eb = lv >> 16;
        if (W + L + eb > nbits) return PMC_Z_BUF_ERROR_DEV;
        const uint32_t mlen = (lv & 0xffff) + ((readlane(bits, 0) >> L) & ((1u << eb) - 1));
        const uint32_t x = L + eb; // <= 20: the distance code starts inside this window
        const uint32_t f = readlane(de, (int)x);
        uint32_t dL, ds;
        if (f < kEntInvalid) {
            dL = f >> 9;
            ds = f & 0x1ff;
        } else if (f == kEntInvalid) {
            return W + x + 1 > nbits ? PMC_Z_BUF_ERROR_DEV : PMC_Z_DATA_ERROR_DEV;
        } else {
            ds = slow_decode(readlane(bits, (int)x), dcnt, T->dsym, dL);
        }
        if (W + x + dL > nbits) return PMC_Z_BUF_ERROR_DEV;
        if (ds >= 30) return PMC_Z_DATA_ERROR_DEV;
        const uint32_t dv = readlane(distv, (int)ds), deb = dv >> 16;
        if (W + x + dL + deb > nbits) return PMC_Z_BUF_ERROR_DEV;
        const uint32_t dist = (dv & 0xffff) + ((readlane(bits, (int)x) >> dL) & ((1u << deb) - 1));
        if (dist > o) return PMC_Z_DATA_ERROR_DEV;
        tok = 0x80000000u | (dist - 1) << 8 | (mlen - 3);
        olen = mlen;
        W += x + dL + deb;
        return 0;
    }

    __device__ int run(const uint8_t *src, uint32_t in_len, uint8_t *dst, uint32_t cap, uint32_t *dst_len) {
        const int l = lane_id();
        // 1. stage input, zero padded by 64 bytes
        {
            const uint32_t words = (in_len + 64 + 3) >> 2;
            if ((((uintptr_t)src) & 3) == 0) {
                const uint32_t *s4 = reinterpret_cast<const uint32_t *>(src);
                const uint32_t full = in_len >> 2;
                for (uint32_t k = l; k < words; k += 64) inw[k] = k < full ? s4[k] : 0u;
                wave_sync();
                if ((uint32_t)l < (in_len & 3)) inb[full * 4 + l] = src[full * 4 + l];
            } else {
                for (uint32_t k = l; k < words; k += 64) inw[k] = 0;
                wave_sync();
                for (uint32_t k = l; k < in_len; k += 64) inb[k] = src[k];
            }
            wave_sync();
        }
        // 2. gzip header (lane 0; inflate.c HEAD..HCRC)
        int hrc = 0;
        uint32_t p = 0;
        if (l == 0) {
            do {
                if (in_len < 2) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                if (inb[0] != 0x1f || inb[1] != 0x8b) { hrc = PMC_Z_DATA_ERROR_DEV; break; }
                if (in_len < 4) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                if (inb[2] != 8) { hrc = PMC_Z_DATA_ERROR_DEV; break; }
                const uint32_t flg = inb[3];
                if (flg & 0xe0) { hrc = PMC_Z_DATA_ERROR_DEV; break; }
                if (in_len < 10) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                p = 10;
                if (flg & 0x04) {
                    if (in_len < p + 2) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                    const uint32_t xlen = inb[p] | ((uint32_t)inb[p + 1] << 8);
                    p += 2;
                    if (in_len < p + xlen) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                    p += xlen;
                }
                if (flg & 0x08) {
                    while (p < in_len && inb[p] != 0) p++;
                    if (p >= in_len) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                    p++;
                }
                if (flg & 0x10) {
                    while (p < in_len && inb[p] != 0) p++;
                    if (p >= in_len) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                    p++;
                }
                if (flg & 0x02) {
                    if (in_len < p + 2) { hrc = PMC_Z_BUF_ERROR_DEV; break; }
                    uint32_t hc = inb[p] | ((uint32_t)inb[p + 1] << 8), c = 0xFFFFFFFFu;
                    for (uint32_t k = 0; k < p; k++) c = crc_tab[(c ^ inb[k]) & 0xff] ^ (c >> 8);
                    if (hc != ((~c) & 0xffff)) { hrc = PMC_Z_DATA_ERROR_DEV; break; }
                    p += 2;
                }
            } while (0);
        }
        hrc = rfl(hrc);
        if (hrc) return hrc;
        p = rfl(p);
        stamp(0);
        const uint32_t nbits = in_len * 8;
        SBits sb{inw, 0, 0, 0, nbits};
        sb.seek(p * 8);
        uint32_t o = 0; // bytes produced (uniform)
        uint32_t last;
        do {
            sb.refill();
            if (!sb.need(3)) return PMC_Z_BUF_ERROR_DEV;
            last = sb.peek(1);
            const uint32_t type = (sb.peek(3) >> 1) & 3;
            sb.drop(3);
            if (type == 0) { // stored
                sb.seek((sb.pos() + 7) & ~7u);
                if (!sb.need(32)) return PMC_Z_BUF_ERROR_DEV;
                const uint32_t len = sb.peek(16);
                sb.drop(16);
                const uint32_t nlen = sb.peek(16);
                sb.drop(16);
                if (len != (nlen ^ 0xffff)) return PMC_Z_DATA_ERROR_DEV;
                if (!sb.need(8 * len)) return PMC_Z_BUF_ERROR_DEV;
                const uint32_t ib = sb.pos() >> 3;
                for (uint32_t k = l; k < len; k += 64)
                    if (o + k < cap) out[o + k] = inb[ib + k];
                o += len;
                sb.seek(sb.pos() + 8 * len);
                wave_sync();
                continue;
            }
            if (type == 3) return PMC_Z_DATA_ERROR_DEV;
            uint32_t lcnt = 0, dcnt = 0;
            int lmax = 0, dmax = 0;
            if (type == 1) { // fixed code lengths (inflate.c fixedtables)
                for (int s = l; s < 320; s += 64)
                    T->lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
                wave_sync();
                stamp(1);
                build<5>(T->lens, 288, false, T->lfast, T->lsym, lcnt, lmax);
                build<1>(T->lens + 288, 32, false, T->dfast, T->dsym, dcnt, dmax);
                stamp(2);
            } else { // dynamic
                sb.refill();
                if (!sb.need(14)) return PMC_Z_BUF_ERROR_DEV;
                const uint32_t nlen = sb.peek(5) + 257;
                sb.drop(5);
                const uint32_t ndist = sb.peek(5) + 1;
                sb.drop(5);
                const uint32_t ncode = sb.peek(4) + 4;
                sb.drop(4);
                if (nlen > 286 || ndist > 30) return PMC_Z_DATA_ERROR_DEV;
                // code-length code lengths: lane k reads its 3 bits directly
                const uint32_t p0 = sb.pos();
                if (p0 + 3 * ncode > nbits) return PMC_Z_BUF_ERROR_DEV;
                if (l < 19) {
                    const uint32_t q = p0 + 3 * (uint32_t)l;
                    const uint32_t v = __builtin_amdgcn_alignbit(inw[(q >> 5) + 1], inw[q >> 5], q & 31) & 7u;
                    T->lens[c_cl_order[l]] = (uint16_t)((uint32_t)l < ncode ? v : 0u);
                }
                sb.seek(p0 + 3 * ncode);
                wave_sync();
                stamp(1);
                uint32_t ccnt;
                int clmax;
                if (build<1>(T->lens, 19, true, T->lfast, T->lsym, ccnt, clmax)) return PMC_Z_DATA_ERROR_DEV;
                stamp(2);
                // the code-length code (<= 7 bits) as a 128-entry table in two VGPRs
                const uint32_t cl0 = T->lfast[l], cl1 = T->lfast[64 + l];
                const uint32_t total = nlen + ndist;
                uint32_t have = 0, prev = 0;
                while (have < total) {
                    sb.refill();
                    uint32_t sym;
                    if (clmax == 0) { // zlib decodes 0 from its 1-bit invalid marker
                        if (!sb.need(1)) return PMC_Z_BUF_ERROR_DEV;
                        sb.drop(1);
                        sym = 0;
                    } else {
                        const uint32_t idx = sb.peek(7);
                        const uint32_t e = idx < 64 ? readlane(cl0, (int)idx) : readlane(cl1, (int)(idx - 64));
                        const uint32_t L = e >> 9;
                        if (!sb.need(L)) return PMC_Z_BUF_ERROR_DEV;
                        sb.drop(L);
                        sym = e & 0x1ff;
                    }
                    if (sym < 16) {
                        T->lens[have] = (uint16_t)sym;
                        prev = sym;
                        have++;
                    } else {
                        uint32_t val = 0, copy;
                        if (sym == 16) {
                            if (!sb.need(2)) return PMC_Z_BUF_ERROR_DEV;
                            if (have == 0) return PMC_Z_DATA_ERROR_DEV;
                            val = prev;
                            copy = 3 + sb.peek(2);
                            sb.drop(2);
                        } else if (sym == 17) {
                            if (!sb.need(3)) return PMC_Z_BUF_ERROR_DEV;
                            copy = 3 + sb.peek(3);
                            sb.drop(3);
                        } else {
                            if (!sb.need(7)) return PMC_Z_BUF_ERROR_DEV;
                            copy = 11 + sb.peek(7);
                            sb.drop(7);
                        }
                        if (have + copy > total) return PMC_Z_DATA_ERROR_DEV;
                        for (uint32_t k = l; k < copy; k += 64) T->lens[have + k] = (uint16_t)val;
                        have += copy;
                        prev = val;
                    }
                }
                wave_sync();
                if (rfl((uint32_t)T->lens[256]) == 0) return PMC_Z_DATA_ERROR_DEV;
                stamp(1);
                if (build<5>(T->lens, (int)nlen, false, T->lfast, T->lsym, lcnt, lmax)) return PMC_Z_DATA_ERROR_DEV;
                if (build<1>(T->lens + nlen, (int)ndist, false, T->dfast, T->dsym, dcnt, dmax))
                    return PMC_Z_DATA_ERROR_DEV;
                stamp(2);
            }
            // ---- symbols: every lane decodes a whole token at its offset W + lane of a window,
            // a scalar chase follows the next-token links, the path's tokens are written at once
            uint32_t W = sb.pos();
            for (;;) {
                uint32_t bits, le, de;
                window(W, bits, le, de);
                const uint32_t ul = (uint32_t)l;
                const bool lok = le < kEntInvalid;
                const uint32_t L = (le >> 9) & 31, sym = le & 0x1ff, s = sym - 257;
                const bool islit = lok && sym < 256, iseob = lok && sym == 256;
                const bool islen = lok && sym > 256 && sym < 286;
                // length base / extra bits in closed form (inflate.c lbase / lext)
                const uint32_t eb = (s >= 8 && s < 28) ? (s >> 2) - 1 : 0u;
                const uint32_t lbase = s < 8 ? s + 3 : s == 28 ? 258u : ((4 + (s & 3)) << eb) + 3;
                const uint32_t mlen = lbase + ((bits >> L) & ((1u << eb) - 1));
                const uint32_t x2 = ul + L + eb;
                // every lane also decodes "a distance code starting here" (inflate.c dbase / dext),
                // packed dist | bits used << 16 | bad << 31, and the length lane fetches lane x2's
                const uint32_t dL = (de >> 9) & 31, ds = de & 0x1ff;
                const bool dok0 = de < kEntInvalid && ds < 30;
                const uint32_t deb = ds >= 4 ? (ds >> 1) - 1 : 0u;
                const uint32_t dbase = ds < 4 ? ds + 1 : ((2 + (ds & 1)) << deb) + 1;
                const uint32_t dpk = dok0 ? (dbase + ((bits >> dL) & ((1u << deb) - 1))) | (dL + deb) << 16 : 0x80000000u;
                const uint32_t dg = (uint32_t)__shfl((int)dpk, (int)(x2 & 63));
                const bool dok = !(dg >> 31);
                const uint32_t dist = dg & 0xffff;
                const uint32_t nxt = islen ? x2 + ((dg >> 16) & 0xff) : ul + L;
                const bool partial = islen && x2 >= 64;
                const bool fast = (islit || iseob || (islen && !partial && dok)) && W + nxt <= nbits;
                // info: next offset | 0x100 exact path needed | 0x200 end of block | 0x400 re-window
                const uint32_t info =
                    nxt | (partial ? 0x400u : fast ? (iseob ? 0x200u : 0u) : 0x100u);
                const uint32_t tok = islit ? sym : (0x80000000u | (dist - 1) << 8 | (mlen - 3));
                uint64_t path = 0;
                uint32_t x = 0, stop = 0;
                while (x < 64) {
                    const uint32_t f = readlane(info, (int)x);
                    if (f & 0x700) {
                        stop = f;
                        break;
                    }
                    path |= 1ull << x;
                    x = f & 0xff;
                }
                stamp(3);
                if (path) {
                    const bool on = (path >> ul) & 1;
                    const uint32_t ol = on ? (islit ? 1u : mlen) : 0u;
                    const uint32_t incl = wave_incl_scan_dpp(ol), tpos = incl - ol;
                    if (ballot(on && islen && dist > o + tpos)) return PMC_Z_DATA_ERROR_DEV;
                    materialise(path, tok, tpos, o, cap);
                    o += readlane(incl, 63);
                }
                stamp(4);
                if (x >= 64 || (stop & 0x400)) { // window used up / a match's distance lies past it
                    W += x;
                    continue;
                }
                if (stop & 0x200) { // end of block
                    W += stop & 0xff;
                    break;
                }
                // exact single-token decode (code longer than the root, invalid code, truncation)
                W += x;
                uint32_t t1 = 0, n1 = 0;
                const int r1 = scalar_token(W, o, nbits, lcnt, dcnt, t1, n1);
                if (r1 < 0) return r1;
                if (r1 == 1) break;
                materialise(1ull, l == 0 ? t1 : 0u, 0u, o, cap);
                o += n1;
                stamp(3);
            }
            sb.seek(W);
        } while (!last);
        // 3. trailer: CRC-32 then ISIZE (inflate.c CHECK / LENGTH)
        const uint32_t tp = (sb.pos() + 7) >> 3;
        if (in_len < tp + 4) return PMC_Z_BUF_ERROR_DEV;
        if (o > cap) { // a valid stream so far that needs more room: report the size (no verdict yet)
            if (l == 0) *dst_len = o;
            return PMC_E_CAPACITY_DEV;
        }
        const uint32_t crc = wave_crc32(out, o, crc_tab);
        const uint32_t want = inb[tp] | ((uint32_t)inb[tp + 1] << 8) | ((uint32_t)inb[tp + 2] << 16) |
                              ((uint32_t)inb[tp + 3] << 24);
        if (crc != want) return PMC_Z_DATA_ERROR_DEV;
        if (in_len < tp + 8) return PMC_Z_BUF_ERROR_DEV;
        const uint32_t isz = inb[tp + 4] | ((uint32_t)inb[tp + 5] << 8) | ((uint32_t)inb[tp + 6] << 16) |
                             ((uint32_t)inb[tp + 7] << 24);
        if (isz != o) return PMC_Z_DATA_ERROR_DEV;
        // 4. copy-out
        if ((((uintptr_t)dst) & 3) == 0) {
            uint32_t *d4 = reinterpret_cast<uint32_t *>(dst);
            PMC_LDS const uint32_t *o4 = (PMC_LDS const uint32_t *)out;
            const uint32_t full = o >> 2;
            for (uint32_t k = l; k < full; k += 64) d4[k] = o4[k];
            if ((uint32_t)l < (o & 3)) dst[full * 4 + l] = out[full * 4 + l];
        } else {
            for (uint32_t k = l; k < o; k += 64) dst[k] = out[k];
        }
        if (l == 0) *dst_len = o;
        stamp(5);
        return 0;
    }
};

template <bool kHbm>
__global__ void __launch_bounds__(256, 5) inflate_kernel(InflateArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint32_t *crc_tab = reinterpret_cast<uint32_t *>(lds);
    for (int k = threadIdx.x; k < 256; k += blockDim.x) crc_tab[k] = c_crc_table[k];
    __syncthreads();
    const int waves_per_block = blockDim.x / 64;
    const int wib = threadIdx.x / 64;
    const uint64_t wave = (uint64_t)blockIdx.x * waves_per_block + wib;
    const uint64_t nwaves = (uint64_t)gridDim.x * waves_per_block;
    const int l = lane_id();
    uint8_t *base = lds + 1024 + (uint64_t)wib * a.wave_bytes;
    InflateWave<true> Wh;
    InflateLds Wl;
    if (kHbm) {
        const InflateLayout L = inflate_layout<true>(a.lds_max_out, a.lds_max_in);
        Wh.sc = reinterpret_cast<InflateScratch *>(base + L.scr);
        Wh.crc_tab = crc_tab;
        for (int k = 0; k < 8; k++) Wh.st[k] = 0;
    } else {
        const InfLdsLayout L = inf_lds_layout(a.lds_max_out, a.lds_max_in);
        Wl.T = (PMC_LDS InfTables *)(base + L.tab);
        Wl.inb = to_lds<uint8_t>(base + L.in);
        Wl.inw = to_lds<uint32_t>(base + L.in);
        Wl.out = to_lds<uint8_t>(base + L.out);
        Wl.crc_tab = to_lds<const uint32_t>(crc_tab);
        Wl.lenv = l < 29 ? (uint32_t)c_lbase[l] | (uint32_t)c_lext[l] << 16 : 0u;
        Wl.distv = l < 30 ? (uint32_t)c_dbase[l] | (uint32_t)c_dext[l] << 16 : 0u;
        for (int k = 0; k < 8; k++) Wl.st[k] = 0;
    }
#ifdef PMC_STAMPS
    Wh.t_last = Wl.t_last = __builtin_amdgcn_s_memtime();
#endif
    // groups of G members per wave (G = 64 once the batch fills every wave 64 times; a few members, the
    // latency path's, one per wave); this variant's members picked out by ballot
    const uint64_t G = min((uint64_t)64, (a.n + nwaves - 1) / nwaves);
    for (uint64_t g = wave * G; g < a.n; g += nwaves * G) {
        const uint64_t vl = g + (uint64_t)l;
        const bool in = (uint64_t)l < G && vl < a.n;
        uint32_t my_in = 0, my_cap = 0;
        if (in) {
            my_in = a.src_len[vl];
            my_cap = a.dst_cap[vl];
        }
        const bool my_fits = my_cap <= a.lds_max_out && my_in <= a.lds_max_in;
        const bool mine = in && (!a.retry_only || a.rc[vl] == kInflateRetry);
        uint64_t todo = ballot(mine && (kHbm != my_fits));
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint64_t v = g + (uint64_t)j;
            const uint32_t in_len = readlane(my_in, j);
            const uint32_t cap = readlane(my_cap, j);
            const uint8_t *src = a.src + a.src_off[v];
            uint8_t *dst = a.dst + a.dst_off[v];
            if (in_len == 0) {
                if (l == 0) {
                    a.rc[v] = PMC_INVALID_INPUT_DEV;
                    a.dst_len[v] = 0;
                }
                continue;
            }
            if (a.retry_only && a.retried && l == 0) atomicAdd(a.retried, 1u); // (the fast paths declined it)
            int rc;
            if (kHbm) {
                Wh.inb = const_cast<uint8_t *>(src);
                Wh.out = dst;
                rc = Wh.run(src, in_len, dst, cap, a.dst_len + v);
            } else {
                rc = Wl.run(src, in_len, dst, cap, a.dst_len + v);
            }
            if (l == 0) {
                a.rc[v] = rc;
                if (rc && rc != PMC_E_CAPACITY_DEV) a.dst_len[v] = 0;
            }
        }
    }
#ifdef PMC_STAMPS
    if (l == 0 && a.dbg)
        for (int k = 0; k < 8; k++)
            atomicAdd((unsigned long long *)&a.dbg[k], (unsigned long long)(kHbm ? Wh.st[k] : Wl.st[k]));
#endif
}

template __global__ void inflate_kernel<false>(InflateArgs);
template __global__ void inflate_kernel<true>(InflateArgs);

} // namespace pmc
