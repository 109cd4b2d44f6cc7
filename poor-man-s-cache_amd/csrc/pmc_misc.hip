// pmc_misc.hip -- helper kernels around the codec: synthetic value generator (SURVEY.md
// §8d), fixed-stride layouts, value comparison, ISIZE trailer reads and the shard router
// (MurmurHash3_x64_128 of "key"+i, /root/reference/src/hash/hash.cpp:4-9 and
// MurmurHash3.cpp:255-332, used by server.cpp:113,121,132 as hash % numShards).
#include <hip/hip_runtime.h>

#include "pmc_device.hpp"
#include "pmc_kernels.hpp"

namespace pmc {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__constant__ char c_alnum[63] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";

// one thread per 8-byte group of one value (same definition as oracle_gen_values)
__global__ void gen_values_kernel(const uint8_t *corpus, uint32_t corpus_len, uint64_t seed, int kind,
                                  uint64_t first, const uint64_t *index, uint32_t n, uint32_t vlen, uint8_t *dst) {
    const uint32_t groups = (vlen + 7) / 8;
    const uint64_t total = (uint64_t)n * groups;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t i = t / groups;
        uint32_t g = (uint32_t)(t - i * groups);
        uint64_t idx = index ? index[i] : first + i;
        uint8_t *d = dst + i * vlen + 8ull * g;
        uint32_t nb = vlen - 8 * g < 8 ? vlen - 8 * g : 8;
        if (kind == 0) {
            uint64_t off = splitmix64(seed ^ idx) % (uint64_t)(corpus_len - vlen + 1);
            const uint8_t *s = corpus + off + 8ull * g;
            for (uint32_t b = 0; b < nb; b++) d[b] = s[b];
        } else {
            uint64_t st = splitmix64(splitmix64(seed ^ idx) + g);
            for (uint32_t b = 0; b < nb; b++) d[b] = (uint8_t)c_alnum[((st >> (8 * b)) & 0xff) % 62];
        }
    }
}

__global__ void fill_layout_kernel(uint64_t *off, uint32_t *len, uint32_t *cap, uint32_t n, uint64_t stride,
                                   uint32_t vlen, uint32_t capv) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (off) off[i] = i * stride;
        if (len) len[i] = vlen;
        if (cap) cap[i] = capv;
    }
}

// one wave per value
__global__ void compare_values_kernel(const uint8_t *a, const uint64_t *a_off, const uint8_t *b, const uint64_t *b_off,
                                      const uint32_t *len, const uint32_t *len_b, uint32_t n, uint32_t *mism) {
    const int l = lane_id();
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    uint32_t bad = 0;
    for (uint64_t v = wave; v < n; v += nw) {
        uint32_t la = len[v];
        bool diff = len_b && len_b[v] != la;
        if (!diff) {
            const uint8_t *pa = a + a_off[v], *pb = b + b_off[v];
            for (uint32_t k = l; k < la && !diff; k += 64) diff = pa[k] != pb[k];
            diff = ballot(diff) != 0;
        }
        if (diff && l == 0) bad++;
    }
    if (l == 0 && bad) atomicAdd(mism, bad);
}

// The batch calls' argument check (include/pmc_codec.h): a value longer than the call's max_len
// is claimed by no deflate variant, so it gets rc = PMC_E_ARG and dst_len = 0 here instead of
// being left unwritten.
__global__ void arg_check_kernel(const uint32_t *src_len, uint64_t n, uint64_t max_len, int32_t *rc,
                                 uint32_t *dst_len) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (src_len[i] > max_len) {
            rc[i] = PMC_E_ARG_DEV;
            dst_len[i] = 0;
        }
}

// Context self-test of the one undocumented hardware behaviour the compressor leans on: the lanes
// of one ds_add_rtn_u32 that hit the same LDS word get their old values in lane order (the hash
// sort's scatter and the canonical-code ranks).  Every trial packs two u16 counters per word as
// the sort's table does; a lane's returned count must equal the number of lower lanes with its
// digit.  pmc_ctx_create runs it once; on any violation the context compresses through the
// kernels that do not depend on it (scripts/micro/lds_atomic_order.hip is the larger probe).
__global__ void __launch_bounds__(256) lane_order_probe_kernel(uint32_t trials, uint32_t *violations) {
    __shared__ uint32_t tab[4][128];
    const int w = threadIdx.x / 64, l = lane_id();
    uint32_t bad = 0;
    for (uint32_t t = 0; t < trials; t++) {
        for (int k = l; k < 128; k += 64) tab[w][k] = 0;
        wave_sync();
        uint32_t x = (uint32_t)(blockIdx.x * 7919u + w * 104729u + t * 31u) * 2654435761u + (uint32_t)l * 40503u;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        const uint32_t alpha = 1u + (t % 7 == 0 ? 255u : t % 9); // 1..256 digits, skewed to few
        const uint32_t d = (x % alpha) & 255u;
        const uint32_t old = lds_add(to_lds<uint32_t>(&tab[w][d >> 1]), 1u << (16 * (d & 1)));
        const uint32_t r = (old >> (16 * (d & 1))) & 0xffffu;
        // lower lanes with the same digit: each lane's digit by a readlane (uniform, every lane active --
        // a __shfl under `j < l` would read lane j while it is switched off, and get 0)
        uint32_t want = 0;
        for (int j = 0; j < 64; j++) {
            const uint32_t dj = (uint32_t)__builtin_amdgcn_readlane((int)d, j);
            want += (uint32_t)j < (uint32_t)l && dj == d ? 1u : 0u;
        }
        bad += r != want ? 1u : 0u;
        wave_sync();
    }
    if (bad) atomicAdd(violations, bad);
}

__global__ void isize_kernel(const uint8_t *src, const uint64_t *off, const uint32_t *len, uint32_t n, uint32_t *isz) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t L = len[i];
        uint32_t v = 0;
        if (L >= 18) {
            const uint8_t *p = src + off[i] + L - 4;
            v = p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
        }
        isz[i] = v;
    }
}

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// MurmurHash3_x64_128(key, len, seed 0)[0] for key = "key" + decimal(idx) (len <= 23 < 32)
__device__ inline uint64_t murmur_key(uint64_t idx) {
    uint8_t k[32] = {'k', 'e', 'y'};
    char dig[20];
    int nd = 0;
    do {
        dig[nd++] = (char)('0' + idx % 10);
        idx /= 10;
    } while (idx);
    int len = 3;
    while (nd) k[len++] = (uint8_t)dig[--nd];
    const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
    uint64_t h1 = 0, h2 = 0, k1, k2;
    const int nblocks = len / 16;
    for (int i = 0; i < nblocks; i++) {
        k1 = k2 = 0;
        for (int b = 0; b < 8; b++) k1 |= (uint64_t)k[16 * i + b] << (8 * b);
        for (int b = 0; b < 8; b++) k2 |= (uint64_t)k[16 * i + 8 + b] << (8 * b);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint8_t *tail = k + nblocks * 16;
    int t = len & 15;
    k1 = k2 = 0;
    for (int b = t - 1; b >= 8; b--) k2 ^= (uint64_t)tail[b] << (8 * (b - 8));
    if (t > 8) { k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; }
    for (int b = (t < 8 ? t : 8) - 1; b >= 0; b--) k1 ^= (uint64_t)tail[b] << (8 * b);
    if (t > 0) { k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1; }
    h1 ^= (uint64_t)len; h2 ^= (uint64_t)len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    return h1 + h2;
}

__global__ void route_kernel(uint64_t first, uint32_t n, uint32_t num_shards, uint32_t n_gpus, uint8_t *gpu) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        gpu[i] = (uint8_t)((murmur_key(first + i) % num_shards) % n_gpus);
}

} // namespace pmc
