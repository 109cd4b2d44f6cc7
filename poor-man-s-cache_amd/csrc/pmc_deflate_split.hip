// pmc_deflate_split.hip -- the small-value compressor as three kernels per chunk of values:
//
//   deflate_front_kernel  one wave per value: stage, hash sort, lazy parse (deflate_slow with
//                         on-demand longest_match), symbol histograms -> tokens + histograms
//   deflate_trees_kernel  one LANE per value: zlib trees.c build_tree / gen_bitlen (exact
//                         binary heap, overflow fix-up), scan_tree, build_bl_tree and the
//                         stored/fixed/dynamic choice -> code lengths + block plan
//   deflate_back_kernel   one wave per value: CRC-32, canonical codes, tree headers,
//                         compress_block emission, gzip framing -> output member
//
// Why the middle kernel is lane-parallel: Huffman construction is a long chain of dependent
// heap operations on ~50-300 entries.  Run by a whole wave it is scalar-unit work (the CU's
// one scalar unit is the bottleneck of the wave-per-value kernel); run by one lane it costs
// 1/64 of the issue slots per value and its heap sits in conflict-free LDS columns
// (entry i of lane l at word i * 64 + l).
//
// Output bytes equal deflate_small_kernel's, i.e. zlib 1.2.11 level 9
// (reference: /root/reference/src/compressor/gzip_compressor.cpp:3-50).
#include <hip/hip_runtime.h>

#include "pmc_device.hpp"
#include "pmc_kernels.hpp"

namespace pmc {

// Chunk arrays: histograms and code lengths are one contiguous row per value (the wave-
// per-value kernels read and write them coalesced); the trees kernel's merge lists are
// interleaved by 64-value block (lane-coalesced).

// ---- front -------------------------------------------------------------------------------------
// (7 waves per SIMD: 72 VGPRs; 28 resident waves per CU at 1 KiB, which the LDS also allows)
// CAPC != 0: the working set is laid out for CAPC bytes at compile time (front_cap_class), so the
// kernel holds one parse instance and its LDS arrays sit at constant offsets from the wave's base.
template <uint32_t CAPC>
__global__ void __launch_bounds__(256, 7) deflate_front_kernel(DeflateArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int wpb = blockDim.x / 64, wib = threadIdx.x / 64, l = lane_id();
    const uint64_t lcap = CAPC ? (uint64_t)CAPC : a.cap_len;
    uint8_t *base = lds + (uint64_t)wib * (CAPC ? front_layout(lcap).total : a.wave_bytes);
    const SmallLayout L = small_layout(lcap);
    const FrontLayout F = front_layout(lcap);
    SmallWave w;
    small_wave_init(w, base, L, a, nullptr);
    w.S = to_lds<uint16_t>(base + F.S);
    w.R = to_lds<uint16_t>(base + F.R);
    w.CN = to_lds<uint8_t>(base + F.cn);
    w.HC = to_lds<uint64_t>(base + F.hc);
    w.EV = to_lds<uint32_t>(base + F.ev);
    w.cnp = F.pkb;
    w.s12 = front_s12(lcap) ? 1u : 0u;
    w.lfreq = to_lds<uint32_t>(base + F.freq);
    w.dfreq = w.lfreq + 288;
    w.blfreq = w.dfreq + 32;
    // Values come from a work counter, a.front_batch at a time, the next grab fetched while these
    // run: value costs vary, and a static split left waves idle (a chunk of 555K values over 7168
    // resident waves is 1.2 rounds of 64-value groups).  Grabs on one counter serialise in L2
    // (~11 ns each): small values take several per grab, or the counter bounds the kernel.
    const uint32_t kBatch = a.front_batch;
    uint32_t nx = l == 0 ? atomicAdd(a.cQ, kBatch) : 0u;
    for (;;) {
        const uint64_t g = readlane(nx, 0);
        if (g >= a.count) break;
        nx = l == 0 ? atomicAdd(a.cQ, kBatch) : 0u;
        const uint64_t vl = g + (uint64_t)l;
        const bool in = (uint32_t)l < kBatch && vl < a.count;
        const uint32_t myl = in ? a.src_len[a.first + vl] : 0u;
        // (source offsets load with the lengths: no dependent round trip per value for its address.  An L2
        // prefetch of the grab's next value beside this one's stage loads measured no faster: round 6)
        const uint64_t myo = in ? a.src_off[a.first + vl] : 0u;
        uint64_t todo = ballot(myl != 0 && myl > a.min_len && myl <= a.lds_max_len);
        while (todo) {
            const int jj = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint64_t v = g + (uint64_t)jj, gv = a.first + v;
            const uint32_t len = readlane(myl, jj);
            w.tok = (PMC_GLB uint32_t *)(a.cT + v * a.cap_len);
#ifdef PMC_FAULT_LANE_ORDER // (odd values fail the sort's guard; the even ones reach the back's code-rank guard)
            w.fault_rev = (uint32_t)(gv & 1);
#endif
            const uint8_t *vsrc = a.src + readlane64(myo, jj);
            const uint32_t ntok = w.run_front(vsrc, len);
            if (ntok == kNtokRetry) { // the sort's lane-order guard fired: the HBM kernel redoes the value
                if (l == 0) {
                    a.cN[v] = kNtokRetry;
                    a.cZ[v] = 0;
                    atomicAdd(a.guard, 1u);
                }
                continue;
            }
            // histograms -> column v of the chunk's interleaved u16 table
            uint32_t nz = 0;
            for (int s = l; s < kLCodes + kDCodes; s += 64) {
                const uint32_t f = s < kLCodes ? w.lfreq[s] : w.dfreq[s - kLCodes];
                a.cH[v * kSplitRows + s] = (uint16_t)f;
                nz += (uint32_t)__builtin_popcountll(ballot(s < kLCodes && f != 0));
            }
            if (l == 0) {
                // >= 16383 symbols: zlib flushes a block mid-value; the HBM kernel redoes the value
                a.cN[v] = ntok < kSymsPerBlock ? ntok : kNtokMultiBlock;
                a.cZ[v] = nz;
            }
        }
    }
    small_wave_stamps_out(w, a);
}
template __global__ void deflate_front_kernel<0>(DeflateArgs);
template __global__ void deflate_front_kernel<1024>(DeflateArgs);
template __global__ void deflate_front_kernel<4096>(DeflateArgs);

// ---- trees (one lane per value) ------------------------------------------------------------------
// (RegU16, pmc_device.hpp: round 5 moved bl_count and the bit-length frequencies from the lane's LDS column
// into registers, which with the 79-entry heap of the <= 1 KiB instance takes the kernel from 6 to 8 waves
// per CU: it is LDS-bound and waits on its heap's dependent LDS round trips.  Per-lane VALU is cheap here:
// one instruction serves 64 values.)
// Packed heap entry, as in the wave kernel: (freq << 5 | depth) << 10 | node, so zlib's
// smaller(n, m) (freq, then depth, <=) is key(n) <= key(m) with key = entry >> 10.
template <int CAP>
struct LaneTrees {
    PMC_LDS uint32_t *hp;  // heap, entry i at hp[i * 64]  (column of this lane)
    RegU16<kMaxBits + 1> blc; // bl_count[16]
    RegU16<kBLCodes> blf;     // bit-length tree frequencies [19]
    const uint16_t *hist;  // global, this value's row: hist[sym]
    uint8_t *lens;         // global, this value's row: lens[sym]
    uint32_t *mg;          // global column: merge list, mg[i * 64]
    bool deferred = false;

    __device__ uint32_t H(uint32_t i) const { return hp[i * 64]; }
    __device__ void setH(uint32_t i, uint32_t v) { hp[i * 64] = v; }

    // pqdownheap (trees.c)
    __device__ void down(uint32_t k, uint32_t n) {
        const uint32_t v = H(k), kv = v >> 10;
        uint32_t j = k << 1;
        while (j <= n) {
            uint32_t x = H(j);
            if (j < n) {
                const uint32_t y = H(j + 1);
                if ((y >> 10) <= (x >> 10)) {
                    j++;
                    x = y;
                }
            }
            if (kv <= (x >> 10)) break;
            setH(k, x);
            k = j;
            j <<= 1;
        }
        setH(k, v);
    }

    // build_tree + gen_bitlen (trees.c) for one tree whose frequencies are freq(s), s < elems;
    // leaf lengths go to lens[row0 + s].  Returns max_code (-1 and `deferred` when the
    // heap would exceed CAP entries).
    // kind: 0 lit/len, 1 distance, 2 bit-length tree.  Extra bits and the static trees' code
    // lengths are closed forms (a per-lane indexed load from constant memory per leaf was a
    // vector-memory round trip inside this serial loop).
    __device__ static uint32_t xbits(int kind, uint32_t x) {
        return kind == 0 ? (x >= kLiterals + 1 ? len_extra_cf(x - (kLiterals + 1)) : 0u)
               : kind == 1 ? dist_extra_cf(x)
                           : (x == 16 ? 2u : x == 17 ? 3u : x == 18 ? 7u : 0u);
    }
    __device__ static uint32_t static_len(int kind, uint32_t x) { // static_ltree / static_dtree .Len
        return kind == 1 ? 5u : x < 144 ? 8u : x < 256 ? 9u : x < 280 ? 7u : 8u;
    }
    template <class Freq>
    // (opt / stat: bit counts of one value's block, < 2^32; 32-bit sums of 24-bit products are full-rate
    // VALU ops, 64-bit multiply-adds quarter-rate ones)
    __device__ int build(Freq freq, int elems, uint32_t row0, int kind, int max_length, uint32_t &opt, uint32_t &stat,
                         PMC_GLB const uint16_t *grow = nullptr) {
        int heap_len = 0, max_code = -1;
        if (grow) {
            // frequencies from a 16-byte aligned global row: 32 per batch in four 16-byte loads, the
            // next batch in flight while this one is inserted (HBM latency was paid per 8 values)
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            PMC_GLB const v4u *g4 = (PMC_GLB const v4u *)grow;
            const int nb = (elems + 31) / 32;
            v4u cur[4], nxt[4];
#pragma unroll
            for (int i = 0; i < 4; i++) cur[i] = i * 8 < elems ? g4[i] : v4u{0, 0, 0, 0};
            for (int b = 0; b < nb; b++) {
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int q = (b + 1) * 4 + i;
                    nxt[i] = b + 1 < nb && q * 8 < elems ? g4[q] : v4u{0, 0, 0, 0};
                }
#pragma unroll
                for (int i = 0; i < 4; i++) {
#pragma unroll
                    for (int h = 0; h < 8; h++) {
                        const int nn = b * 32 + i * 8 + h;
                        const uint32_t f = nn < elems ? (cur[i][h >> 1] >> (16 * (h & 1))) & 0xffffu : 0u;
                        if (f) {
                            if (heap_len == CAP) {
                                deferred = true;
                                return -1;
                            }
                            setH(++heap_len, f << 15 | (uint32_t)nn);
                            max_code = nn;
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < 4; i++) cur[i] = nxt[i];
            }
        }
        // (frequencies fetched 8 at a time so the loads overlap)
        for (int n0 = 0; !grow && n0 < elems; n0 += 8) {
            uint32_t f8[8];
#pragma unroll
            for (int k = 0; k < 8; k++) f8[k] = n0 + k < elems ? freq(n0 + k) : 0u;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (f8[k]) {
                    if (heap_len == CAP) {
                        deferred = true;
                        return -1;
                    }
                    setH(++heap_len, f8[k] << 15 | (uint32_t)(n0 + k));
                    max_code = n0 + k;
                }
            }
        }
        while (heap_len < 2) { // at least two codes (dummy leaves of frequency 1)
            const int node = max_code < 2 ? ++max_code : 0;
            setH(++heap_len, 1u << 15 | (uint32_t)node);
            opt--;
            if (kind != 2) stat -= static_len(kind, (uint32_t)node);
        }
        for (int n = heap_len / 2; n >= 1; n--) down((uint32_t)n, (uint32_t)heap_len);
        uint32_t node = (uint32_t)elems, nm = 0;
        do {
            const uint32_t n = H(1);
            setH(1, H((uint32_t)heap_len));
            heap_len--;
            down(1, (uint32_t)heap_len);
            const uint32_t m = H(1);
            mg[(2 * nm) * 64] = n;
            mg[(2 * nm + 1) * 64] = m;
            nm++;
            const uint32_t kn = n >> 10, km = m >> 10, dn = kn & 31, dm = km & 31;
            const uint32_t d = (dn >= dm ? dn : dm) + 1;
            setH(1, ((((kn >> 5) + (km >> 5)) << 5) | d) << 10 | node);
            node++;
            down(1, (uint32_t)heap_len);
        } while (heap_len >= 2);
        // gen_bitlen: merges in reverse (zlib's heap[heap_max..] order: m before n); the
        // lengths of internal nodes reuse the heap's column (node elems + i - 1 at slot i)
        const uint32_t K = nm;
        uint32_t overflow = 0;
        blc.zero();
        setH(K, 0);
        // The merge list is read back 8 merges (16 keys) per batch with the next two batches in flight:
        // one dependent global round trip per merge made this replay the kernel's longest wait.
        constexpr int kB = 8;
        uint32_t cur[2 * kB], nxt[2 * kB], nx2[2 * kB];
        auto fetch = [&](int hi, uint32_t *d) { // merges hi - 1, hi - 2, ..., hi - kB (those >= 0)
#pragma unroll
            for (int t = 0; t < kB; t++) {
                const int j = hi - 1 - t;
                d[2 * t] = j >= 0 ? mg[(2 * j + 1) * 64] : 0u;   // m first (zlib's heap[heap_max..] order)
                d[2 * t + 1] = j >= 0 ? mg[(2 * j) * 64] : 0u;
            }
        };
        // (two batches in flight ahead of the one being replayed)
        fetch((int)K, cur);
        fetch((int)K - kB, nxt);
        for (int i0 = (int)K; i0 >= 1; i0 -= kB) {
            fetch(i0 - 2 * kB, nx2);
#pragma unroll
            for (int t = 0; t < kB; t++) {
                const int i = i0 - t;
                if (i < 1) break;
                const uint32_t L = H((uint32_t)i);
#pragma unroll
                for (int c = 0; c < 2; c++) {
                    const uint32_t key = cur[2 * t + c], x = key & 1023;
                    uint32_t bits = L + 1;
                    if (bits > (uint32_t)max_length) {
                        bits = (uint32_t)max_length;
                        overflow++;
                    }
                    if (x >= (uint32_t)elems) {
                        setH(x - (uint32_t)elems + 1, bits);
                    } else {
                        lens[row0 + x] = (uint8_t)bits;
                        blc.add(bits, 1);
                        const uint32_t f = key >> 15;
                        const uint32_t xb = xbits(kind, x);
                        opt += __umul24(f, bits + xb);
                        if (kind != 2) stat += __umul24(f, static_len(kind, x) + xb);
                    }
                }
            }
#pragma unroll
            for (int t = 0; t < 2 * kB; t++) {
                cur[t] = nxt[t];
                nxt[t] = nx2[t];
            }
        }
        if (overflow) {
            int ov = (int)overflow;
            do {
                int bits = max_length - 1;
                while (blc.get((uint32_t)bits) == 0) bits--;
                blc.add((uint32_t)bits, -1);
                blc.add((uint32_t)bits + 1, 2);
                blc.add((uint32_t)max_length, -1);
                ov -= 2;
            } while (ov > 0);
            // leaves in zlib's heap[--h] order from the top: n_1, m_1, n_2, m_2, ...
            uint32_t idx = 0;
            for (int bits = max_length; bits != 0; bits--) {
                uint32_t n = blc.get((uint32_t)bits);
                while (n != 0) {
                    const uint32_t key = mg[idx * 64], x = key & 1023;
                    idx++;
                    if (x >= (uint32_t)elems) continue;
                    const uint32_t cur = lens[row0 + x];
                    if (cur != (uint32_t)bits) {
                        opt += (uint32_t)((int32_t)bits - (int32_t)cur) * (key >> 15);
                        lens[row0 + x] = (uint8_t)bits;
                    }
                    n--;
                }
            }
        }
        return max_code;
    }

    // send_all_trees (trees.c) of a dynamic block, per lane: HLIT, HDIST, HCLEN, the bit-length code lengths
    // in bl_order, then send_tree over the staged lit/len and distance lengths; the bits go LSB-first to
    // row[1..], their count to row[0].  (The back, a wave per value, spent a third of its time on these
    // serial runs; here one instruction serves 64 values.)  blw: row bytes 304..335 (bl lengths at 12..30).
    __device__ void emit_header(int l_max, int d_max, int mbi, const uint32_t *blw, PMC_GLB uint32_t *row) {
        auto blen = [&](int s) -> uint32_t { return (blw[(12 + s) >> 2] >> (8 * ((12 + s) & 3))) & 0xffu; };
        // canonical bit-length codes (gen_codes): counts and next codes as bytes of 64-bit words
        uint64_t cnt = 0;
#pragma unroll
        for (int s = 0; s < kBLCodes; s++) {
            const uint32_t L = blen(s);
            cnt += L ? 1ull << (8 * L) : 0ull;
        }
        uint64_t nc = 0;
        uint32_t code = 0;
#pragma unroll
        for (int b = 1; b <= kMaxBLBits; b++) {
            code = (code + (uint32_t)((cnt >> (8 * (b - 1))) & 0xffu)) << 1;
            nc |= (uint64_t)code << (8 * b);
        }
        RegU16<kBLCodes> bc; // code | len << 8 per bit-length symbol
#pragma unroll
        for (int s = 0; s < kBLCodes; s++) {
            const uint32_t L = blen(s), c = (uint32_t)(nc >> (8 * L)) & 0xffu;
            nc += L ? 1ull << (8 * L) : 0ull;
            bc.set((uint32_t)s, L ? (__builtin_bitreverse32(c) >> (32 - L)) | L << 8 : 0u);
        }
        uint64_t acc = 0;
        uint32_t an = 0, wi = 1, total = 0;
        auto put = [&](uint32_t v, uint32_t n) {
            acc |= (uint64_t)v << an;
            an += n;
            total += n;
            if (an >= 32) {
                row[wi++] = (uint32_t)acc;
                acc >>= 32;
                an -= 32;
            }
        };
        auto send_code = [&](uint32_t sym) {
            const uint32_t e = bc.get(sym);
            put(e & 0xffu, e >> 8);
        };
        put((uint32_t)(l_max + 1 - 257), 5);
        put((uint32_t)d_max, 5);
        put((uint32_t)(mbi + 1 - 4), 4);
        for (int k = 0; k <= mbi; k++) put(bc.get(bl_order_cf(k)) >> 8, 3);
        for (int tr = 0; tr < 2; tr++) { // send_tree: the lit/len tree, then the distance tree
            const uint32_t row0 = tr ? (uint32_t)kLCodes : 0u;
            const int max_code = tr ? d_max : l_max;
            int prevlen = -1, nextlen = (int)lrow(row0), count = 0, max_count = 7, min_count = 4;
            if (nextlen == 0) max_count = 138, min_count = 3;
            int w0 = -8;
            uint64_t pk = 0;
            for (int n = 0; n <= max_code; n++) {
                const int curlen = nextlen, nx = n + 1;
                if (nx <= max_code) {
                    if (nx >= w0 + 8) {
                        w0 = nx & ~7;
                        pk = 0;
#pragma unroll
                        for (int k = 0; k < 8; k++)
                            pk |= (uint64_t)(w0 + k <= max_code ? lrow(row0 + (uint32_t)(w0 + k)) : 0u) << (8 * k);
                    }
                    nextlen = (int)((pk >> (8 * (nx - w0))) & 0xff);
                } else {
                    nextlen = 0xffff;
                }
                if (++count < max_count && curlen == nextlen) continue;
                if (count < min_count) {
                    do {
                        send_code((uint32_t)curlen);
                    } while (--count != 0);
                } else if (curlen != 0) {
                    if (curlen != prevlen) {
                        send_code((uint32_t)curlen);
                        count--;
                    }
                    send_code(kRep3_6);
                    put((uint32_t)(count - 3), 2);
                } else if (count <= 10) {
                    send_code(kRepz3_10);
                    put((uint32_t)(count - 3), 3);
                } else {
                    send_code(kRepz11_138);
                    put((uint32_t)(count - 11), 7);
                }
                count = 0;
                prevlen = curlen;
                if (nextlen == 0) max_count = 138, min_count = 3;
                else if (curlen == nextlen) max_count = 6, min_count = 3;
                else max_count = 7, min_count = 4;
            }
        }
        if (an) row[wi] = (uint32_t)acc;
        row[0] = total;
    }

    // byte j of the lengths row as staged in the heap column (stage_row)
    __device__ uint32_t lrow(uint32_t j) const { return (hp[(j >> 2) * 64] >> (8 * (j & 3))) & 0xffu; }
    // The lit/len + distance lengths (row bytes 0..319) into the heap column, free between the distance
    // tree's build and the bit-length tree's: twenty 16-byte loads in flight at once, so scan_tree reads
    // LDS.  (Reading the row from HBM eight bytes per step made it ~40 dependent global round trips per
    // value, most of one value's trees latency: 243 us for a lone 1 KiB value.)
    __device__ void stage_row() {
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        v4u r[20];
#pragma unroll
        for (int i = 0; i < 20; i++) r[i] = *(PMC_GLB const v4u *)(lens + 16 * i);
#pragma unroll
        for (int i = 0; i < 20; i++) {
            hp[(4 * i + 0) * 64] = r[i].x;
            hp[(4 * i + 1) * 64] = r[i].y;
            hp[(4 * i + 2) * 64] = r[i].z;
            hp[(4 * i + 3) * 64] = r[i].w;
        }
    }

    // scan_tree (trees.c): bit-length tree frequencies for lengths row[row0 .. row0 + max_code] (staged)
    __device__ void scan(uint32_t row0, int max_code) {
        int prevlen = -1, nextlen = (int)lrow(row0), count = 0, max_count = 7, min_count = 4;
        if (nextlen == 0) max_count = 138, min_count = 3;
        int w0 = -8;
        uint64_t pk = 0; // lengths w0 .. w0 + 7, one byte each (fetched 8 at a time so the loads overlap)
        for (int n = 0; n <= max_code; n++) {
            const int curlen = nextlen, nx = n + 1;
            if (nx <= max_code) {
                if (nx >= w0 + 8) {
                    w0 = nx & ~7;
                    pk = 0;
#pragma unroll
                    for (int k = 0; k < 8; k++)
                        pk |= (uint64_t)(w0 + k <= max_code ? lrow(row0 + (uint32_t)(w0 + k)) : 0u) << (8 * k);
                }
                nextlen = (int)((pk >> (8 * (nx - w0))) & 0xff);
            } else {
                nextlen = 0xffff;
            }
            if (++count < max_count && curlen == nextlen) {
                continue;
            }
            if (count < min_count) {
                blf.add((uint32_t)curlen, count);
            } else if (curlen != 0) {
                if (curlen != prevlen) blf.add((uint32_t)curlen, 1);
                blf.add(kRep3_6, 1);
            } else if (count <= 10) {
                blf.add(kRepz3_10, 1);
            } else {
                blf.add(kRepz11_138, 1);
            }
            count = 0;
            prevlen = curlen;
            if (nextlen == 0) max_count = 138, min_count = 3;
            else if (curlen == nextlen) max_count = 6, min_count = 3;
            else max_count = 7, min_count = 4;
        }
    }
};

template <int CAP>
__device__ void trees_value(const DeflateArgs &a, uint64_t v, uint64_t slot, PMC_LDS uint32_t *col) {
    const uint32_t len = a.src_len[a.first + v];
    if (len == 0 || len <= a.min_len || len > a.lds_max_len || a.cN[v] >= kNtokRetry) return;
    LaneTrees<CAP> t;
    t.hp = col;
    t.hist = a.cH + v * kSplitRows;
    t.lens = a.cL + v * kSplitRows;
    t.mg = a.cG + ((slot >> 6) * kMergeRows) * 64 + (slot & 63); // (by lane slot: coalesced)
    for (uint32_t s = 0; s < kSplitRows; s += 16) *reinterpret_cast<uint4 *>(t.lens + s) = make_uint4(0, 0, 0, 0);
    uint32_t opt = 0, stat = 0;
    auto hist = [&](int s) -> uint32_t { return t.hist[s]; };
    const int l_max = t.build(hist, kLCodes, 0, 0, kMaxBits, opt, stat, (PMC_GLB const uint16_t *)t.hist);
    if (t.deferred) {
        a.cP[v] = kPlanDeferred;
        a.cD[atomicAdd(a.cD + a.count, 1u)] = (uint32_t)v;
        return;
    }
    // the distance frequencies (row u16 286..315, bytes 572..631) staged in heap slots 60..74 with five
    // 16-byte loads at once; the distance tree's leaves fill slots 1..30 only (not four dependent HBM reads)
    {
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        PMC_GLB const v4u *g4 = (PMC_GLB const v4u *)t.hist;
        static_assert(kLCodes * 2 == 35 * 16 + 12 && kDCodes == 30, "distance row at v4u 35, byte 12");
        // (stage_row below also fills heap slots 0..79 with the 20 x 16-byte lengths row: the column has
        // CAP + 1 >= 80 slots)
        static_assert(CAP >= 79, "heap slots 60..74 hold the staged distance frequencies, 0..79 the lengths row");
        v4u d5[5];
#pragma unroll
        for (int i = 0; i < 5; i++) d5[i] = g4[35 + i];
#pragma unroll
        for (int j = 3; j < 18; j++) t.hp[(57 + j) * 64] = d5[j >> 2][j & 3];
    }
    auto dhist = [&](int s) -> uint32_t { return (t.hp[(60 + (s >> 1)) * 64] >> (16 * (s & 1))) & 0xffffu; };
    const int d_max = t.build(dhist, kDCodes, kLCodes, 1, kMaxBits, opt, stat);
    t.blf.zero();
    t.stage_row();
    t.scan(0, l_max);
    t.scan(kLCodes, d_max);
    auto bfreq = [&](int s) -> uint32_t { return t.blf.get((uint32_t)s); };
    t.build(bfreq, kBLCodes, kLCodes + kDCodes, 2, kMaxBLBits, opt, stat);
    // max_blindex from the bit-length code's lengths (row bytes 316..334) loaded at once, not one
    // dependent HBM read per step of the loop
    static_assert(kLCodes + kDCodes == 316 && kSplitRows >= 336, "bl lengths at row bytes 316..334");
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u q0 = *(PMC_GLB const v4u *)(t.lens + 304), q1 = *(PMC_GLB const v4u *)(t.lens + 320);
    const uint32_t blw[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    int mbi = 2;
#pragma unroll
    for (int k = kBLCodes - 1; k >= 3; k--) {
        const int j = 12 + (int)bl_order_cf(k); // byte of row 316 + bl_order(k), counted from 304
        if (mbi == 2 && ((blw[j >> 2] >> (8 * (j & 3))) & 0xffu) != 0) mbi = k;
    }
    opt += 3 * ((uint32_t)mbi + 1) + 5 + 5 + 4;
    uint32_t opt_lenb = (opt + 3 + 7) >> 3;
    const uint32_t static_lenb = (stat + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    const uint32_t type = len + 4 <= opt_lenb ? 0u : static_lenb == opt_lenb ? 1u : 2u;
    const bool hdr = PMC_TREES_HDR && type == 2 && len > kHdrMinLen;
    a.cP[v] = type | (uint32_t)l_max << 2 | (uint32_t)d_max << 11 | (uint32_t)mbi << 16 | (hdr ? kPlanHdr : 0u);
    if (hdr) { // (the bit-length tree's heap overwrote the front of the staged row: stage it again)
        t.stage_row();
        t.emit_header(l_max, d_max, mbi, blw, (PMC_GLB uint32_t *)(a.cB + v * kHdrWords));
    }
}

// Values whose literal/length tree needs more than CAP heap entries are listed in cD (count at
// cD[count]) and planned by the CAP = kLCodes instance, a small grid that walks that list.
template <int CAP>
__global__ void __launch_bounds__(64) deflate_trees_kernel(DeflateArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tl[];
    const uint32_t l = threadIdx.x;
    PMC_LDS uint32_t *col = to_lds<uint32_t>(tl + l);
    if (CAP != kLCodes) {
        // values in cO order: a wave's lanes get heaps of similar size and finish together; the
        // largest heaps first (blocks start in index order), so the kernel's last waves are short
        const uint64_t vi = (uint64_t)blockIdx.x * 64 + l;
        if (vi < a.count) trees_value<CAP>(a, a.cO ? (uint64_t)a.cO[a.count - 1 - vi] : vi, vi, col);
    } else {
        const uint32_t nd = a.cD[a.count];
        for (uint32_t k = blockIdx.x * 64 + l; k < nd; k += gridDim.x * 64)
            trees_value<CAP>(a, a.cD[k], a.cD[k], col);
    }
}
template __global__ void deflate_trees_kernel<kTreesCap>(DeflateArgs);
template __global__ void deflate_trees_kernel<kTreesCap1K>(DeflateArgs);
template __global__ void deflate_trees_kernel<kLCodes>(DeflateArgs);

// ---- back --------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256, 5) deflate_back_kernel(DeflateArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    // slicing-by-8 CRC tables (8 KiB; table 0 is the plain byte table)
    uint32_t *crc_tab = reinterpret_cast<uint32_t *>(lds);
    for (int k = threadIdx.x; k < 8 * 256; k += blockDim.x) crc_tab[k] = c_crc_slice8[k];
    __syncthreads();
    const int wpb = blockDim.x / 64, wib = threadIdx.x / 64, l = lane_id();
    uint8_t *base = lds + kBackTabBytes + (uint64_t)wib * a.wave_bytes;
    const SmallLayout L = small_layout(a.cap_len);
    const BackLayout B = back_layout(a.cap_len);
    SmallWave w;
    small_wave_init(w, base, L, a, crc_tab);
    w.outw = to_lds<uint32_t>(base + B.out);
    w.outb = to_lds<uint8_t>(base + B.out);
    w.out_words = (uint32_t)B.out_words;
    w.lcode = to_lds<uint32_t>(base + B.lcode);
    w.dcode = to_lds<uint32_t>(base + B.dcode);
    w.blcode = to_lds<uint32_t>(base + B.blcode);
    w.runs = to_lds<uint16_t>(base + B.runs);
    w.blfreq = to_lds<uint32_t>(base + B.blfreq);
    w.perm = to_lds<uint16_t>(base + B.perm);
    // (run_back touches only the arrays above; the rest of w still points into the larger
    // small_layout and must stay unused here)
    PMC_LDS uint8_t *Ls = to_lds<uint8_t>(base + B.ls); // code lengths from the trees kernel
    // (work counter as in the front, in batches of 16 values whose lengths, token counts and
    // plans load together: a back value is short, and a round trip per value showed)
    constexpr uint32_t kBatch = 16;
    uint32_t nx = l == 0 ? atomicAdd(a.cQ + 1, kBatch) : 0u;
    for (;;) {
        const uint64_t g = readlane(nx, 0);
        if (g >= a.count) break;
        nx = l == 0 ? atomicAdd(a.cQ + 1, kBatch) : 0u;
        const uint64_t vl = g + (uint64_t)l;
        const bool in = (uint32_t)l < kBatch && vl < a.count;
        const uint32_t myl = in ? a.src_len[a.first + vl] : 0u;
        const uint32_t myn = in ? a.cN[vl] : 0u, myp = in ? a.cP[vl] : 0u;
        const uint32_t myk = a.back_nostage && in ? a.cC[vl] : 0u; // (the batch CRC pass's)
        // (source / destination offsets and capacities of the batch load with its lengths: no
        // dependent round trip per value for its addresses)
        const uint64_t myo = in ? a.src_off[a.first + vl] : 0u, mydo = in ? a.dst_off[a.first + vl] : 0u;
        const uint32_t myc = in ? a.dst_cap[a.first + vl] : 0u;
        // (the small pass, min_len 0, also answers empty values: rc = INVALID_INPUT below)
        uint64_t todo = ballot(in && (a.min_len == 0 || myl > a.min_len) && myl <= a.lds_max_len);
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint64_t v = g + (uint64_t)j, gv = a.first + v;
            const uint32_t len = readlane(myl, j);
            // L2 prefetch of the next value of the batch: one dword per lane touches every 128-byte
            // line of its source bytes, tokens and code-length row, so this value's work hides the
            // HBM latency of the next one's loads (the dword is consumed after run_back, when it
            // has long arrived; one VGPR instead of staging registers).
            uint32_t pf = 0;
            if (todo) {
                const int j2 = __builtin_ctzll(todo);
                const uint64_t v2 = g + (uint64_t)j2;
                const uint32_t len2 = readlane(myl, j2), n2 = readlane(myn, j2);
                const uintptr_t sa = (uintptr_t)(a.src + readlane64(myo, j2)), ta = (uintptr_t)(a.cT + v2 * a.cap_len),
                                la = (uintptr_t)(a.cL + v2 * kSplitRows);
                const uint32_t ns = (uint32_t)(((sa & 127) + len2 + 127) >> 7),
                               nt = n2 >= kNtokRetry ? 0u : (uint32_t)(((ta & 127) + 4ull * n2 + 127) >> 7),
                               nl = (uint32_t)(((la & 127) + kSplitRows + 127) >> 7);
                const uint32_t k = (uint32_t)l;
                const uintptr_t addr = k < ns ? (sa & ~(uintptr_t)127) + 128ull * k
                                       : k < ns + nt ? (ta & ~(uintptr_t)127) + 128ull * (k - ns)
                                                     : (la & ~(uintptr_t)127) + 128ull * (k - ns - nt);
                if (k < ns + nt + nl) pf = *(PMC_GLB const uint32_t *)addr;
            }
            if (len == 0) {
                if (l == 0) {
                    a.rc[gv] = PMC_INVALID_INPUT_DEV;
                    a.dst_len[gv] = 0;
                }
                continue;
            }
            const uint32_t ntok = readlane(myn, j), plan = readlane(myp, j);
            if (ntok >= kNtokRetry) { // several blocks, or the sort's guard fired: the HBM kernel
                if (l == 0) {
                    a.rc[gv] = kDeflateRetry;
                    if (ntok == kNtokMultiBlock) atomicAdd(a.guard + 3, 1u);
                    retry_push(a, gv);
                }
                continue;
            }
            { // the code-length row (336 B; rows and Ls are 16-byte aligned) as dwords
                PMC_GLB const uint32_t *row = (PMC_GLB const uint32_t *)(a.cL + v * kSplitRows);
                PMC_LDS uint32_t *Lw = (PMC_LDS uint32_t *)Ls;
                for (uint32_t k = l; k < kSplitRows / 4; k += 64) Lw[k] = row[k];
            }
            w.tok = (PMC_GLB uint32_t *)(a.cT + v * a.cap_len);
            w.hdr = plan & kPlanHdr ? (PMC_GLB const uint32_t *)(a.cB + v * kHdrWords) : nullptr;
            const int rc = w.run_back(a.src + readlane64(myo, j), len, ntok, plan, Ls, a.dst + readlane64(mydo, j),
                                      readlane(myc, j), a.dst_len + gv, readlane(myk, j), a.back_nostage);
            if (l == 0) {
                a.rc[gv] = rc;
                if (rc) a.dst_len[gv] = 0;
                if (rc == kDeflateRetry) { // (the code-rank guard fired)
                    atomicAdd(a.guard + 1, 1u);
                    retry_push(a, gv);
                }
            }
            asm volatile("" ::"v"(pf));
        }
    }
    small_wave_stamps_out(w, a);
}

} // namespace pmc
