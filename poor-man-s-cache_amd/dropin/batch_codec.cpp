// batch_codec.cpp -- see batch_codec.hpp.  One pmc_gzip_compress_batch_host call per SET batch
// and one pmc_gzip_decompress_batch_host call per GET batch; the per-value decisions follow
// /root/reference/src/kvs/kvs.cpp:148,182-196 (SET) and :224,233-234 (GET).
#include "batch_codec.hpp"

#include <sys/mman.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>

#include "gzip_compressor.hpp"
#include "pmc_codec.h"

namespace pmc_batch {

std::vector<StoredValue> CompressForSet(const std::vector<const char *> &values, bool compression_enabled,
                                        pmc_ctx *ctx) {
    const size_t n = values.size();
    std::vector<StoredValue> out(n, StoredValue{nullptr, 0, false, OPERATION_SUCCESS});
    std::vector<uint32_t> pick;  // indices of the values sent to the codec
    std::vector<uint64_t> src_off, dst_off;
    std::vector<uint32_t> src_len, dst_cap;
    std::vector<uint8_t> src;
    uint64_t so = 0, dof = 0;
    for (size_t i = 0; i < n; i++) {
        if (!values[i]) {
            out[i].rc = INVALID_INPUT;
            continue;
        }
        const size_t len = strlen(values[i]);
        if (!compression_enabled || len + 1 < kMinCompressSize) continue;
        pick.push_back((uint32_t)i);
        src_off.push_back(so);
        src_len.push_back((uint32_t)len);
        dst_off.push_back(dof);
        dst_cap.push_back((uint32_t)pmc_gzip_bound(len));
        so += len;
        dof += dst_cap.back();
    }
    if (!pick.empty()) {
        src.resize(so);
        for (size_t k = 0; k < pick.size(); k++) memcpy(src.data() + src_off[k], values[pick[k]], src_len[k]);
        std::vector<uint8_t> dst(dof);
        std::vector<uint32_t> dst_len(pick.size());
        std::vector<int32_t> rc(pick.size(), 0);
        if (!ctx) ctx = pmc_default_ctx();
        int r = ctx ? pmc_gzip_compress_batch_host(ctx, src.data(), src_off.data(), src_len.data(),
                                                   (uint32_t)pick.size(), dst.data(), dst_off.data(), dst_cap.data(),
                                                   dst_len.data(), rc.data())
                    : PMC_E_NO_DEVICE;
        for (size_t k = 0; k < pick.size(); k++) {
            StoredValue &v = out[pick[k]];
            v.rc = r ? r : rc[k];
            if (v.rc != OPERATION_SUCCESS) continue;  // stored raw below, as kvs.cpp:189-191
            v.data = new char[dst_len[k]];
            memcpy(v.data, dst.data() + dst_off[k], dst_len[k]);
            v.size = dst_len[k];
            v.compressed = true;
        }
    }
    for (size_t i = 0; i < n; i++) {
        if (!values[i] || out[i].compressed) continue;
        const size_t sz = strlen(values[i]) + 1;
        out[i].data = new char[sz];
        memcpy(out[i].data, values[i], sz);
        out[i].size = sz;
    }
    return out;
}

namespace {
// A grow-only buffer of uninitialised bytes kept across batches: a server's batches are tens of MB (4,096 x 4 KiB
// values), and a fresh zeroed std::vector per batch paid its page faults and its memset every iteration.
struct Scratch {
    std::unique_ptr<uint8_t[]> p;
    size_t cap = 0;
    uint8_t *get(size_t n) {
        if (n > cap) {
            cap = n + n / 4;
            p.reset(new uint8_t[cap]);
        }
        return p.get();
    }
};
thread_local Scratch g_ddst;  // decompress_packed's output image (request thread)
thread_local Scratch g_cdst;  // the compress job's member image (built on the request thread, one job in flight)

// The members k < n at src + src_off[k] (src_len[k] bytes each) decoded in one host call: out[k] a new[]
// NUL-terminated value of olen[k] bytes, or nullptr (the reference's Decompress failure).  Capacity from
// ISIZE (as GzipCompressor::Decompress), capped at DEFLATE's 1032:1.
void decompress_packed(const uint8_t *src, const std::vector<uint64_t> &src_off, const std::vector<uint32_t> &src_len,
                       std::vector<char *> &out, std::vector<uint32_t> &olen, pmc_ctx *ctx) {
    const size_t n = src_len.size();
    out.assign(n, nullptr);
    olen.assign(n, 0);
    if (!n) return;
    std::vector<uint64_t> dst_off(n);
    std::vector<uint32_t> dst_cap(n);
    uint64_t dof = 0;
    for (size_t k = 0; k < n; k++) {
        uint64_t cap = pmc_gzip_isize(src + src_off[k], src_len[k]);
        if (cap > 1032ull * src_len[k] + 64) cap = 1032ull * src_len[k] + 64;
        dst_off[k] = dof;
        dst_cap[k] = (uint32_t)cap;
        dof += cap;
    }
    uint8_t *dst = g_ddst.get(dof + 1);
    std::vector<uint32_t> dst_len(n);
    std::vector<int32_t> rc(n, 0);
    if (!ctx) ctx = pmc_default_ctx();
    const int r = ctx ? pmc_gzip_decompress_batch_host(ctx, src, src_off.data(), src_len.data(), (uint32_t)n, dst,
                                                       dst_off.data(), dst_cap.data(), dst_len.data(), rc.data())
                      : PMC_E_NO_DEVICE;
    auto place = [&](size_t k, const uint8_t *bytes, uint32_t len) {
        char *v = new char[len + 1];
        memcpy(v, bytes, len);
        v[len] = '\0';
        out[k] = v;
        olen[k] = len;
    };
    std::vector<uint32_t> again;
    for (size_t k = 0; k < n; k++) {
        if (r) break;
        if (rc[k] == OPERATION_SUCCESS) place(k, dst + dst_off[k], dst_len[k]);
        else if (rc[k] == PMC_E_CAPACITY && dst_len[k] > dst_cap[k]) again.push_back((uint32_t)k);
    }
    // members followed by bytes that misstate their size (the reference ignores bytes after the
    // first member, gzip_compressor.cpp:96): PMC_E_CAPACITY carries the decoded size, so one more
    // call with exactly that room gives their bytes or their verdict
    if (!again.empty()) {
        std::vector<uint64_t> s2_off, d2_off;
        std::vector<uint32_t> s2_len, d2_cap, d2_len(again.size());
        std::vector<int32_t> rc2(again.size(), 0);
        uint64_t d2 = 0;
        for (uint32_t k : again) {
            s2_off.push_back(src_off[k]);
            s2_len.push_back(src_len[k]);
            d2_off.push_back(d2);
            d2_cap.push_back(dst_len[k]);
            d2 += dst_len[k];
        }
        std::vector<uint8_t> dst2(d2 + 1);
        const int r2 = pmc_gzip_decompress_batch_host(ctx, src, s2_off.data(), s2_len.data(), (uint32_t)again.size(),
                                                      dst2.data(), d2_off.data(), d2_cap.data(), d2_len.data(), rc2.data());
        for (size_t j = 0; j < again.size() && !r2; j++)
            if (rc2[j] == OPERATION_SUCCESS) place(again[j], dst2.data() + d2_off[j], d2_len[j]);
    }
}
}  // namespace

std::vector<char *> DecompressForGet(const std::vector<Entry> &entries, std::vector<bool> *owned, pmc_ctx *ctx) {
    const size_t n = entries.size();
    std::vector<char *> out(n, nullptr);
    if (owned) owned->assign(n, false);
    std::vector<uint32_t> pick;
    std::vector<uint64_t> src_off;
    std::vector<uint32_t> src_len;
    uint64_t so = 0;
    for (size_t i = 0; i < n; i++) {
        const Entry &e = entries[i];
        if (!e.compressed) {
            out[i] = const_cast<char *>(e.data);
            continue;
        }
        if (!e.data || e.size == 0) continue;  // Decompress's INVALID_INPUT -> nullptr
        pick.push_back((uint32_t)i);
        src_off.push_back(so);
        src_len.push_back((uint32_t)e.size);
        so += e.size;
    }
    if (pick.empty()) return out;
    std::vector<uint8_t> src(so);
    for (size_t k = 0; k < pick.size(); k++) memcpy(src.data() + src_off[k], entries[pick[k]].data, src_len[k]);
    std::vector<char *> vals;
    std::vector<uint32_t> olen;
    decompress_packed(src.data(), src_off, src_len, vals, olen, ctx);
    for (size_t k = 0; k < pick.size(); k++) {
        out[pick[k]] = vals[k];
        if (owned && vals[k]) (*owned)[pick[k]] = true;
    }
    return out;
}

// ---- batch priming (f1 inside the unchanged caller) --------------------------------------------------
namespace {

struct PrimeState {
    // compress: the batch's values back to back, and per value its primed member
    struct Comp {
        uint64_t off;
        uint32_t len;
        char *data;  // new[] member (nullptr once handed out)
        size_t size;
        std::string spare;  // the member bytes, kept for a second SET of the same value
        bool dup;           // the batch holds this value more than once: keep the spare
    };
    std::string cvals;
    std::vector<Comp> comp;
    std::unordered_multimap<uint64_t, uint32_t> cidx;  // content fingerprint -> comp index
    // decompress: members recorded by the dry run, then their primed values
    bool collecting = false;
    std::vector<std::pair<const char *, size_t>> collected;
    struct Dec {
        uint64_t off;  // member bytes in dmembers
        size_t size;
        char *data;    // new[] NUL-terminated value (nullptr once handed out, or on failure)
        size_t len;
        int rc;
        std::string spare;  // the value bytes, kept for a second GET of the same member
        bool dup;           // the dry run read this member more than once: keep the spare
    };
    std::string dmembers;
    std::vector<Dec> dec;
    std::unordered_map<const char *, uint32_t> didx;
    PrimeStats stats{};
};
thread_local PrimeState g_prime;

// cheap content fingerprint (length + three sampled words); candidates are confirmed by memcmp
uint64_t fingerprint(const char *p, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n * 0xFF51AFD7ED558CCDull;
    auto mix = [&](size_t at) {
        uint64_t w = 0;
        memcpy(&w, p + at, n - at < 8 ? n - at : 8);
        h = (h ^ w) * 0xC4CEB9FE1A85EC53ull;
        h ^= h >> 29;
    };
    if (n) {
        mix(0);
        mix(n / 2);
        mix(n > 8 ? n - 8 : 0);
    }
    return h;
}

} // namespace

// ---- device-store mode (f2 inside the unchanged kvs) ------------------------------------------------
namespace {
struct Handle {       // what Entry.value holds for a compressed value in store mode (vSize = 32)
    char magic[4];    // "PMCX": a gzip member starts 1f 8b, so the two never look alike
    uint32_t gen;     // allocation generation: a slot reused for another value never matches a primed one
    pmc_extent ext;   // the member's extent in the device heap
};
static_assert(sizeof(Handle) == 32, "handle size");
constexpr char kHandleMagic[4] = {'P', 'M', 'C', 'X'};
constexpr size_t kHandleSlots = size_t(1) << 26;  // 64M values: 2 GiB of address space, touched as used

struct StoreState {
    bool on = false;
    uint64_t heap_bytes = 0;
    std::once_flag once;
    pmc_store *store = nullptr;
    char *slab = nullptr;  // kHandleSlots x 32 B, mapped at EnableDeviceStore
    std::mutex mu;         // slots (SETs on the request thread, frees from kvs on the same thread, EndBatch)
    std::vector<uint32_t> free_slots;
    uint32_t next = 0, gen = 0;
    size_t live = 0;
};
StoreState g_store;

pmc_store *the_store() {
    std::call_once(g_store.once, [] {
        pmc_ctx *ctx = pmc_default_ctx();
        if (!ctx || pmc_store_create(ctx, g_store.heap_bytes, &g_store.store) != PMC_OK) g_store.store = nullptr;
    });
    return g_store.store;
}

bool in_slab(const void *p) {
    return g_store.slab && (const char *)p >= g_store.slab && (const char *)p < g_store.slab + kHandleSlots * 32;
}

char *handle_new(const pmc_extent &e) {
    std::lock_guard<std::mutex> lk(g_store.mu);
    uint32_t s;
    if (!g_store.free_slots.empty()) {
        s = g_store.free_slots.back();
        g_store.free_slots.pop_back();
    } else if (g_store.next < kHandleSlots) {
        s = g_store.next++;
    } else {
        return nullptr;
    }
    Handle *h = (Handle *)(g_store.slab + (size_t)s * 32);
    memcpy(h->magic, kHandleMagic, 4);
    h->gen = ++g_store.gen;
    h->ext = e;
    g_store.live++;
    return (char *)h;
}

// the extent a live handle names (false: not a handle of this store)
bool handle_extent(const char *p, size_t n, pmc_extent *e) {
    if (n != sizeof(Handle) || !in_slab(p) || ((uintptr_t)(p - g_store.slab) & 31)) return false;
    const Handle *h = (const Handle *)p;
    if (memcmp(h->magic, kHandleMagic, 4) != 0 || !(h->ext.flags & 1)) return false;
    *e = h->ext;
    return true;
}

// extents of the handles collected by a dry run, decoded in one store call: out[k] a new[] NUL-terminated
// value of olen[k] bytes, or nullptr
void store_get(const std::vector<pmc_extent> &ext, std::vector<char *> &out, std::vector<uint32_t> &olen) {
    const size_t n = ext.size();
    out.assign(n, nullptr);
    olen.assign(n, 0);
    pmc_store *st = the_store();
    if (!n || !st) return;
    std::vector<const uint8_t *> resp(n, nullptr);
    std::vector<uint32_t> rlen(n, 0);
    std::vector<int32_t> rc(n, 0);
    if (pmc_store_get_batch(st, ext.data(), (uint32_t)n, PMC_FRAME_RAW, resp.data(), rlen.data(), rc.data()) != PMC_OK)
        return;
    for (size_t k = 0; k < n; k++) {
        if (rc[k] != PMC_OK || !resp[k]) continue;
        char *v = new char[rlen[k] + 1];
        memcpy(v, resp[k], rlen[k]);
        v[rlen[k]] = '\0';
        out[k] = v;
        olen[k] = rlen[k];
    }
}
}  // namespace

void EnableDeviceStore(uint64_t heap_bytes) {
    if (g_store.on) return;
    void *m = mmap(nullptr, kHandleSlots * 32, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (m == MAP_FAILED) return;
    g_store.slab = (char *)m;
    g_store.heap_bytes = heap_bytes;
    g_store.on = true;
}

namespace detail {
bool StoreMode() { return g_store.on; }

bool ReleaseIfHandle(void *p) noexcept {
    if (!in_slab(p)) return false;  // (checked before any lock: the store's own frees come through here too)
    std::lock_guard<std::mutex> lk(g_store.mu);
    Handle *h = (Handle *)p;
    if (memcmp(h->magic, kHandleMagic, 4) == 0) {
        if ((h->ext.flags & 1) && g_store.store) pmc_store_free(g_store.store, &h->ext, 1);
        memset(h, 0, sizeof *h);
        g_store.free_slots.push_back((uint32_t)(((char *)p - g_store.slab) / 32));
        g_store.live--;
    }
    return true;
}

bool StoreCompress(const char *input, size_t len, CompressResult *out) {
    if (!g_store.on) return false;
    pmc_store *st = the_store();
    const uint64_t off = 0;
    const uint32_t l = (uint32_t)len;
    pmc_extent e{};
    int32_t rc = PMC_E_NO_DEVICE;
    if (st) {
        const int r = pmc_store_put_batch(st, (const uint8_t *)input, &off, &l, 1, &e, &rc);
        if (r) rc = r;
    }
    if (rc != PMC_OK) {
        *out = {nullptr, 0, rc};  // kvs stores the raw value (kvs.cpp:188-192)
        return true;
    }
    char *h = handle_new(e);
    if (!h) {
        pmc_store_free(st, &e, 1);
        *out = {nullptr, 0, PMC_Z_MEM_ERROR};
        return true;
    }
    *out = {h, sizeof(Handle), OPERATION_SUCCESS};
    return true;
}

bool StoreDecompress(const char *input, size_t size, DecompressResult *out) {
    pmc_extent e;
    if (!g_store.on || !handle_extent(input, size, &e)) return false;
    std::vector<char *> v;
    std::vector<uint32_t> n;
    store_get({e}, v, n);
    *out = v[0] ? DecompressResult{v[0], OPERATION_SUCCESS} : DecompressResult{nullptr, PMC_Z_DATA_ERROR};
    return true;
}
}  // namespace detail

// One compress batch: its arrays (built on the request thread) and its results; run() touches nothing
// else, so it may run on a helper thread (PrimeCompressAsync) while the request thread does the GETs.
struct CompressJob {
    std::vector<uint64_t> src_off, dst_off;
    std::vector<uint32_t> src_len, dst_cap, dst_len;
    std::vector<int32_t> rc;
    uint8_t *dst = nullptr;       // g_cdst of the request thread that built the job
    std::vector<pmc_extent> ext;  // store mode: the members' extents
    const char *vals = nullptr;
    int r = PMC_OK;
    bool build(PrimeState &P, const std::vector<std::string_view> &values) {
        uint64_t dof = 0;
        for (const auto &v : values) {
            if (v.size() + 1 < kMinCompressSize || v.size() > 0xffffffffull) continue;  // kvs.cpp:182
            src_off.push_back(P.cvals.size());
            src_len.push_back((uint32_t)v.size());
            P.cvals.append(v.data(), v.size());
            dst_off.push_back(dof);
            dst_cap.push_back((uint32_t)pmc_gzip_bound(v.size()));
            dof += dst_cap.back();
        }
        vals = P.cvals.data();  // (stable: nothing appends to cvals until finish())
        if (!g_store.on) dst = g_cdst.get(dof + 1);
        dst_len.resize(src_len.size());
        rc.assign(src_len.size(), 0);
        return !src_len.empty();
    }
    void run(pmc_ctx *ctx) {
        if (g_store.on) {  // the members go straight into HBM extents; only their handles come back
            pmc_store *st = the_store();
            ext.assign(src_len.size(), pmc_extent{});
            r = st ? pmc_store_put_batch(st, (const uint8_t *)vals, src_off.data(), src_len.data(),
                                         (uint32_t)src_len.size(), ext.data(), rc.data())
                   : PMC_E_NO_DEVICE;
            return;
        }
        r = ctx ? pmc_gzip_compress_batch_host(ctx, (const uint8_t *)vals, src_off.data(), src_len.data(),
                                               (uint32_t)src_len.size(), dst, dst_off.data(), dst_cap.data(),
                                               dst_len.data(), rc.data())
                : PMC_E_NO_DEVICE;
    }
    void finish(PrimeState &P) {
        P.stats.batches++;
        for (size_t k = 0; k < src_len.size(); k++) {
            if (r || rc[k] != OPERATION_SUCCESS) continue;  // not primed: Compress runs (and fails) itself
            char *d;
            size_t dsize = dst_len.empty() ? 0 : dst_len[k];
            if (g_store.on) {  // a handle per value; a second SET of the same value in the batch gets its own
                d = handle_new(ext[k]);  // extent through the single-value path (no spare)
                dsize = sizeof(Handle);
                if (!d) {
                    pmc_store_free(the_store(), &ext[k], 1);
                    continue;
                }
            } else {
                d = new char[dsize];
                memcpy(d, dst + dst_off[k], dsize);
            }
            const uint32_t idx = (uint32_t)P.comp.size();
            const uint64_t fp = fingerprint(P.cvals.data() + src_off[k], src_len[k]);
            bool dup = false;  // (an equal value earlier in the batch: both keep their member bytes)
            auto range = P.cidx.equal_range(fp);
            for (auto it = range.first; it != range.second && !g_store.on; ++it) {
                auto &c = P.comp[it->second];
                if (c.len == src_len[k] && memcmp(P.cvals.data() + c.off, P.cvals.data() + src_off[k], c.len) == 0)
                    c.dup = dup = true;
            }
            P.comp.push_back({src_off[k], src_len[k], d, dsize, {}, dup});
            P.cidx.emplace(fp, idx);
        }
    }
};

void PrimeCompress(const std::vector<std::string_view> &values, pmc_ctx *ctx) {
    PrimeState &P = g_prime;
    CompressJob job;
    if (!job.build(P, values)) return;
    job.run(ctx ? ctx : pmc_default_ctx());
    job.finish(P);
}

namespace {
// PrimeCompressAsync's job and helper thread (per request thread)
thread_local std::unique_ptr<CompressJob> g_job;
// joined when its request thread exits between PrimeCompressAsync and PrimeCompressWait (an exception
// unwinding the thread): a joinable std::thread destroyed unjoined would std::terminate the server.
// (Destroyed before g_job, which was constructed first: the helper's job outlives it.)
struct JobThread {
    std::thread t;
    ~JobThread() {
        if (t.joinable()) t.join();
    }
};
thread_local JobThread g_job_thread;
// A context of its own: host calls of one context run one at a time (pmc_codec.h), and this one runs
// beside the default context's decompress batch, on its own stream -- on the default context's
// device, which pmc_default_ctx() fixes at device 0.
pmc_ctx *compress_ctx() {
    static std::once_flag once;
    static pmc_ctx *c = nullptr;
    std::call_once(once, [] {
        if (pmc_ctx_create(0, &c) != PMC_OK) c = nullptr;
    });
    return c ? c : pmc_default_ctx();
}
} // namespace

void PrimeCompressAsync(const std::vector<std::string_view> &values) {
    PrimeCompressWait();
    auto job = std::make_unique<CompressJob>();
    if (!job->build(g_prime, values)) return;
    CompressJob *j = job.get();
    g_job = std::move(job);
    g_job_thread.t = std::thread([j] { j->run(compress_ctx()); });
}

void PrimeCompressWait() {
    if (g_job_thread.t.joinable()) g_job_thread.t.join();
    if (g_job) {
        g_job->finish(g_prime);
        g_job.reset();
    }
}

void BeginCollect() {
    g_prime.collecting = true;
    g_prime.collected.clear();
}

void PrimeCollected(pmc_ctx *ctx) {
    PrimeState &P = g_prime;
    P.collecting = false;
    std::vector<uint32_t> which;
    std::vector<pmc_extent> hext;  // store mode: handles' extents, decoded by one store call
    std::vector<uint32_t> hpos, mpos;
    for (const auto &c : P.collected) {
        auto seen = P.didx.find(c.first);
        if (seen != P.didx.end()) {  // one decode per stored member
            P.dec[seen->second].dup = true;
            continue;
        }
        const uint32_t idx = (uint32_t)P.dec.size();
        P.didx.emplace(c.first, idx);
        P.dec.push_back({P.dmembers.size(), c.second, nullptr, 0, 0, {}, false});
        P.dmembers.append(c.first, c.second);
        pmc_extent e;  // (the stored pointer itself: a handle is recognised by its address in the slab)
        if (g_store.on && handle_extent(c.first, c.second, &e)) {
            hext.push_back(e);
            hpos.push_back((uint32_t)which.size());
        } else {
            mpos.push_back((uint32_t)which.size());
        }
        which.push_back(idx);
    }
    P.collected.clear();
    if (which.empty()) return;
    // (straight from dmembers, where the members already lie back to back; the decoded lengths come back
    // with the values, no strlen over them)
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    for (uint32_t k : mpos) {
        off.push_back(P.dec[which[k]].off);
        len.push_back((uint32_t)P.dec[which[k]].size);
    }
    std::vector<char *> vals(which.size(), nullptr), part;
    std::vector<uint32_t> olen(which.size(), 0), plen;
    if (!mpos.empty()) {
        decompress_packed((const uint8_t *)P.dmembers.data(), off, len, part, plen, ctx);
        for (size_t j = 0; j < mpos.size(); j++) vals[mpos[j]] = part[j], olen[mpos[j]] = plen[j];
    }
    if (!hpos.empty()) {
        store_get(hext, part, plen);
        for (size_t j = 0; j < hpos.size(); j++) vals[hpos[j]] = part[j], olen[hpos[j]] = plen[j];
    }
    P.stats.batches++;
    for (size_t k = 0; k < which.size(); k++) {
        auto &d = P.dec[which[k]];
        if (!vals[k]) {
            d.rc = -1;  // not primed: Decompress runs itself and returns the reference's verdict
            continue;
        }
        d.data = vals[k];
        d.len = olen[k];  // (a value with an embedded NUL: its copies still read as the same C string)
    }
}

void EndBatch() {
    PrimeState &P = g_prime;
    for (auto &c : P.comp) {
        if (c.data && !detail::ReleaseIfHandle(c.data)) delete[] c.data;  // (a handle nobody took: its extent too)
    }
    for (auto &d : P.dec) delete[] d.data;
    P.cvals.clear();
    P.comp.clear();
    P.cidx.clear();
    P.collecting = false;
    P.collected.clear();
    P.dmembers.clear();
    P.dec.clear();
    P.didx.clear();
}

PrimeStats GetPrimeStats() {
    PrimeStats s = g_prime.stats;
    if (g_store.on && g_store.store) {
        uint64_t used = 0, reserved = 0, heap = 0;
        pmc_store_stats(g_store.store, &used, &reserved, &heap);
        std::lock_guard<std::mutex> lk(g_store.mu);
        s.store_values = g_store.live;
        s.store_bytes = used;
    }
    return s;
}

namespace detail {

bool TakeCompressed(const char *input, size_t len, CompressResult *out) {
    PrimeState &P = g_prime;
    if (P.cidx.empty()) return false;
    auto range = P.cidx.equal_range(fingerprint(input, len));
    for (auto it = range.first; it != range.second; ++it) {
        auto &c = P.comp[it->second];
        if (c.len != len || memcmp(P.cvals.data() + c.off, input, len) != 0) continue;
        char *d = c.data;
        if (!d && g_store.on) continue;  // store mode: an equal value later in the batch has its own extent
        if (!d && !c.dup) break;  // handed out, and no spare: the single-value path compresses it again
        if (d) {
            if (c.dup) c.spare.assign(d, c.size);
            c.data = nullptr;  // ownership passes to the caller (Entry.value, freed by kvs)
        } else {               // the same value twice in one batch: its own copy of the member
            d = new char[c.size];
            memcpy(d, c.spare.data(), c.size);
        }
        *out = {d, c.size, OPERATION_SUCCESS};
        P.stats.compress_hits++;
        return true;
    }
    P.stats.compress_misses++;
    return false;
}

bool Collecting(const char *input, size_t size) {
    PrimeState &P = g_prime;
    if (!P.collecting) return false;
    P.collected.emplace_back(input, size);
    return true;
}

bool TakeDecompressed(const char *input, size_t size, DecompressResult *out) {
    PrimeState &P = g_prime;
    if (P.didx.empty()) return false;
    auto it = P.didx.find(input);
    if (it == P.didx.end()) {
        P.stats.decompress_misses++;
        return false;
    }
    auto &d = P.dec[it->second];
    if (d.rc || d.size != size || memcmp(P.dmembers.data() + d.off, input, size) != 0) {
        P.stats.decompress_misses++;
        return false;
    }
    char *v = d.data;
    if (!v && !d.dup) {  // handed out, and no spare (a read the dry run did not see): decompress it again
        P.stats.decompress_misses++;
        return false;
    }
    if (!v) {  // handed out already (a second GET of the key in this batch): a copy of the value
        v = new char[d.len + 1];
        memcpy(v, d.spare.data(), d.len);
        v[d.len] = '\0';
    } else {
        if (d.dup) d.spare.assign(v, d.len);
        d.data = nullptr;  // the caller owns it now (the reference server never frees it)
    }
    *out = {v, OPERATION_SUCCESS};
    P.stats.decompress_hits++;
    return true;
}

} // namespace detail

} // namespace pmc_batch
