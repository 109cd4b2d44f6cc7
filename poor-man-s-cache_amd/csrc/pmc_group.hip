// pmc_group.hip -- one process driving several GPUs (include/pmc_codec.h).
//
// The reference server is one process that routes every key to shard hashFunc(key) % numShards
// (/root/reference/src/server/server.cpp:113,121,132; hash.cpp:4-9).  Here shard s lives on GPU
// s % nGPU, so a host batch is split by that route, each GPU's share goes through its own context
// (pinned staging, copy streams, kernels) on its own host thread, and the results are put back in
// the caller's order.  No data crosses between GPUs: there is no collective.  Compiled into the
// unity TU after pmc_capi.hip (host code only).

#include <thread>

// MurmurHash3_x64_128(key, len, seed 0), first 64-bit word: the reference's hashFunc
// (hash.cpp:4-9 over MurmurHash3.cpp:255-332), restated for the host side of the route.
namespace {
inline uint64_t rotl64h(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t fmix64h(uint64_t k) {
    k = (k ^ (k >> 33)) * 0xff51afd7ed558ccdull;
    k = (k ^ (k >> 33)) * 0xc4ceb9fe1a85ec53ull;
    return k ^ (k >> 33);
}
} // namespace

PMC_API uint64_t pmc_key_hash(const void *key, size_t len) {
    const uint8_t *p = (const uint8_t *)key;
    const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
    uint64_t h1 = 0, h2 = 0;
    const size_t blocks = len / 16;
    for (size_t b = 0; b < blocks; b++) {
        uint64_t k1, k2;
        memcpy(&k1, p + 16 * b, 8);
        memcpy(&k2, p + 16 * b + 8, 8);
        h1 ^= rotl64h(k1 * c1, 31) * c2;
        h1 = (rotl64h(h1, 27) + h2) * 5 + 0x52dce729;
        h2 ^= rotl64h(k2 * c2, 33) * c1;
        h2 = (rotl64h(h2, 31) + h1) * 5 + 0x38495ab5;
    }
    // tail: bytes 8..15 of the last partial block feed k2, bytes 0..7 feed k1 (little endian)
    const uint8_t *t = p + 16 * blocks;
    const size_t rem = len & 15;
    uint64_t k1 = 0, k2 = 0;
    for (size_t i = rem; i > 8; i--) k2 |= (uint64_t)t[i - 1] << (8 * (i - 9));
    for (size_t i = std::min<size_t>(rem, 8); i > 0; i--) k1 |= (uint64_t)t[i - 1] << (8 * (i - 1));
    if (rem > 8) h2 ^= rotl64h(k2 * c2, 33) * c1;
    if (rem > 0) h1 ^= rotl64h(k1 * c1, 31) * c2;
    h1 ^= (uint64_t)len;
    h2 ^= (uint64_t)len;
    h1 += h2;
    h2 += h1;
    h1 = fmix64h(h1);
    h2 = fmix64h(h2);
    return h1 + h2;
}

struct pmc_group {
    std::vector<pmc_ctx *> ctx;
    struct Share {  // pinned gather/scatter buffers of one member
        HostBuf buf;
    };
    std::vector<Share> share;
    std::mutex mu;
};

PMC_API int pmc_group_create(const int *devices, int n, pmc_group **out) {
    if (!out) return PMC_E_ARG;
    *out = nullptr;
    if (!devices || n <= 0) return PMC_E_ARG;
    pmc_group *g = new pmc_group;
    for (int k = 0; k < n; k++) {
        pmc_ctx *c = nullptr;
        const int r = pmc_ctx_create(devices[k], &c);
        if (r) {
            for (auto *x : g->ctx) pmc_ctx_destroy(x);
            delete g;
            return r;
        }
        g->ctx.push_back(c);
    }
    g->share.resize(n);
    *out = g;
    return PMC_OK;
}

PMC_API void pmc_group_destroy(pmc_group *g) {
    if (!g) return;
    for (size_t k = 0; k < g->ctx.size(); k++) {
        (void)hipSetDevice(g->ctx[k]->device);
        g->share[k].buf.release();
        pmc_ctx_destroy(g->ctx[k]);
    }
    delete g;
}

PMC_API int pmc_group_size(pmc_group *g) { return g ? (int)g->ctx.size() : 0; }

PMC_API int pmc_group_route(pmc_group *g, const uint64_t *key_hash, uint32_t num_shards, uint32_t n,
                            uint32_t *member) {
    if (!g || !num_shards || (n && (!key_hash || !member))) return PMC_E_ARG;
    const uint64_t G = g->ctx.size();
    for (uint32_t i = 0; i < n; i++) member[i] = (uint32_t)((key_hash[i] % num_shards) % G);
    return PMC_OK;
}

namespace {
// Runs fn(lo, hi) over [0, m) on up to `threads` host threads (the calling one included).
template <class F>
void par_for(uint32_t m, int threads, F fn) {
    const uint32_t per = 16384;  // values per thread at least: thread start-up is ~10 us
    const int t = (int)std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)threads, (m + per - 1) / per));
    if (t == 1) {
        fn(0u, m);
        return;
    }
    std::vector<std::thread> th;
    const uint32_t step = (m + t - 1) / t;
    for (int k = 1; k < t; k++) {
        const uint32_t lo = k * step, hi = std::min<uint32_t>(m, lo + step);
        if (lo < hi) th.emplace_back([=] { fn(lo, hi); });
    }
    fn(0u, std::min<uint32_t>(m, step));
    for (auto &x : th) x.join();
}

// Member k's share of a group batch: gather its values into pinned memory (back to back), run the
// pipelined pinned call on its context, put each output at the caller's dst_off.  Compress runs in
// packed mode (only the members' real bytes come back over PCIe, ~0.37 of a 1 KiB value's slot);
// decompress in slot mode (value sizes are known).  The gather and the scatter are memcpy loops
// split over `threads` host threads: one thread moving every byte of an 8-GPU batch would bound it.
int group_share(pmc_group *g, int k, Dir dir, const std::vector<uint32_t> &idx, const uint8_t *src,
                const uint64_t *src_off, const uint32_t *src_len, uint8_t *dst, const uint64_t *dst_off,
                const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc, uint32_t max_len, int threads) {
    const uint32_t m = (uint32_t)idx.size();
    if (m == 0) return PMC_OK;
    uint64_t in_b = 0, out_b = 0;
    for (uint32_t i : idx) {
        in_b += src_len[i];
        out_b += dst_cap[i];
    }
    const uint64_t meta = al256(m * 8ull) * 2 + al256(m * 4ull) * 4;
    HostBuf &hb = g->share[k].buf;
    int r = hb.ensure(meta + al256(in_b + 16) + out_b + 64);
    if (r) return r;
    uint8_t *hp = (uint8_t *)hb.p;
    uint64_t *soff = (uint64_t *)hp, *doff = (uint64_t *)(hp + al256(m * 8ull));
    uint32_t *slen = (uint32_t *)(hp + al256(m * 8ull) * 2);
    uint32_t *dcap = (uint32_t *)((uint8_t *)slen + al256(m * 4ull));
    uint32_t *dlen = (uint32_t *)((uint8_t *)dcap + al256(m * 4ull));
    int32_t *src_rc = (int32_t *)((uint8_t *)dlen + al256(m * 4ull));
    uint8_t *s = hp + meta, *d = s + al256(in_b + 16);
    uint64_t so = 0, dof = 0;
    for (uint32_t j = 0; j < m; j++) {
        const uint32_t i = idx[j];
        soff[j] = so;
        slen[j] = src_len[i];
        so += src_len[i];
        doff[j] = dof;
        dcap[j] = dst_cap[i];
        dof += dst_cap[i];
    }
    par_for(m, threads, [&](uint32_t lo, uint32_t hi) {
        for (uint32_t j = lo; j < hi; j++) memcpy(s + soff[j], src + src_off[idx[j]], slen[j]);
    });
    const bool packed = dir == kCompress;
    r = pinned_batch(g->ctx[k], dir, s, soff, slen, m, d, packed ? nullptr : doff, dcap, dlen, src_rc, max_len, 0);
    if (r) return r;
    if (packed) {  // member j at the sum of the successful members' lengths before it
        uint64_t po = 0;
        for (uint32_t j = 0; j < m; j++) {
            doff[j] = po;
            po += src_rc[j] == PMC_OK ? dlen[j] : 0u;
        }
    }
    par_for(m, threads, [&](uint32_t lo, uint32_t hi) {
        for (uint32_t j = lo; j < hi; j++) {
            const uint32_t i = idx[j];
            rc[i] = src_rc[j];
            dst_len[i] = dlen[j];
            if (src_rc[j] == PMC_OK) memcpy(dst + dst_off[i], d + doff[j], dlen[j]);
        }
    });
    return PMC_OK;
}

int group_batch(pmc_group *g, Dir dir, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                const uint64_t *key_hash, uint32_t num_shards, uint32_t n, uint8_t *dst, const uint64_t *dst_off,
                const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc, uint32_t max_len) {
    if (!g || !num_shards ||
        (n && (!src || !src_off || !src_len || !key_hash || !dst || !dst_off || !dst_cap || !dst_len || !rc)))
        return PMC_E_ARG;
    if (n == 0) return PMC_OK;
    std::lock_guard<std::mutex> lock(g->mu);
    const int G = (int)g->ctx.size();
    std::vector<std::vector<uint32_t>> idx(G);
    for (uint32_t i = 0; i < n; i++) idx[(key_hash[i] % num_shards) % (uint64_t)G].push_back(i);
    std::vector<int> res(G, PMC_OK);
    std::vector<std::thread> th;
    // host threads for each member's gather / scatter: the CPUs this process may use, shared out
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    static const int cap = getenv("PMC_GROUP_THREADS") ? atoi(getenv("PMC_GROUP_THREADS")) : 16;
    const int per = std::max(1, std::min(hw, cap > 0 ? cap : hw) / G);
    for (int k = 1; k < G; k++)
        th.emplace_back([&, k] {
            res[k] = group_share(g, k, dir, idx[k], src, src_off, src_len, dst, dst_off, dst_cap, dst_len, rc,
                                 max_len, per);
        });
    res[0] = group_share(g, 0, dir, idx[0], src, src_off, src_len, dst, dst_off, dst_cap, dst_len, rc, max_len,
                         per);
    for (auto &t : th) t.join();
    for (int k = 0; k < G; k++)
        if (res[k]) return res[k];
    return PMC_OK;
}
} // namespace

PMC_API int pmc_group_compress_batch(pmc_group *g, const uint8_t *src, const uint64_t *src_off,
                                     const uint32_t *src_len, const uint64_t *key_hash, uint32_t num_shards,
                                     uint32_t n, uint8_t *dst, const uint64_t *dst_off, const uint32_t *dst_cap,
                                     uint32_t *dst_len, int32_t *rc, uint32_t max_len) {
    return group_batch(g, kCompress, src, src_off, src_len, key_hash, num_shards, n, dst, dst_off, dst_cap, dst_len,
                       rc, max_len);
}

PMC_API int pmc_group_decompress_batch(pmc_group *g, const uint8_t *src, const uint64_t *src_off,
                                       const uint32_t *src_len, const uint64_t *key_hash, uint32_t num_shards,
                                       uint32_t n, uint8_t *dst, const uint64_t *dst_off, const uint32_t *dst_cap,
                                       uint32_t *dst_len, int32_t *rc, uint32_t max_len) {
    return group_batch(g, kDecompress, src, src_off, src_len, key_hash, num_shards, n, dst, dst_off, dst_cap,
                       dst_len, rc, max_len);
}
