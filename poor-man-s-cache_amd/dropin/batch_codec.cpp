// batch_codec.cpp -- see batch_codec.hpp.  One pmc_gzip_compress_batch_host call per SET batch
// and one pmc_gzip_decompress_batch_host call per GET batch; the per-value decisions follow
// /root/reference/src/kvs/kvs.cpp:148,182-196 (SET) and :224,233-234 (GET).
#include "batch_codec.hpp"

#include <cstdint>
#include <cstring>

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

std::vector<char *> DecompressForGet(const std::vector<Entry> &entries, std::vector<bool> *owned, pmc_ctx *ctx) {
    const size_t n = entries.size();
    std::vector<char *> out(n, nullptr);
    if (owned) owned->assign(n, false);
    std::vector<uint32_t> pick;
    std::vector<uint64_t> src_off, dst_off;
    std::vector<uint32_t> src_len, dst_cap;
    uint64_t so = 0, dof = 0;
    for (size_t i = 0; i < n; i++) {
        const Entry &e = entries[i];
        if (!e.compressed) {
            out[i] = const_cast<char *>(e.data);
            continue;
        }
        if (!e.data || e.size == 0) continue;  // Decompress's INVALID_INPUT -> nullptr
        // ISIZE sizes the output (as GzipCompressor::Decompress); DEFLATE expands at most 1032:1
        uint64_t cap = pmc_gzip_isize(e.data, e.size);
        if (cap > 1032ull * e.size + 64) cap = 1032ull * e.size + 64;
        pick.push_back((uint32_t)i);
        src_off.push_back(so);
        src_len.push_back((uint32_t)e.size);
        dst_off.push_back(dof);
        dst_cap.push_back((uint32_t)cap);
        so += e.size;
        dof += cap;
    }
    if (pick.empty()) return out;
    std::vector<uint8_t> src(so), dst(dof + 1);
    for (size_t k = 0; k < pick.size(); k++) memcpy(src.data() + src_off[k], entries[pick[k]].data, src_len[k]);
    std::vector<uint32_t> dst_len(pick.size());
    std::vector<int32_t> rc(pick.size(), 0);
    if (!ctx) ctx = pmc_default_ctx();
    int r = ctx ? pmc_gzip_decompress_batch_host(ctx, src.data(), src_off.data(), src_len.data(),
                                                 (uint32_t)pick.size(), dst.data(), dst_off.data(), dst_cap.data(),
                                                 dst_len.data(), rc.data())
                : PMC_E_NO_DEVICE;
    auto place = [&](size_t k, const uint8_t *bytes, uint32_t len) {
        char *v = new char[len + 1];
        memcpy(v, bytes, len);
        v[len] = '\0';
        out[pick[k]] = v;
        if (owned) (*owned)[pick[k]] = true;
    };
    std::vector<uint32_t> again;
    for (size_t k = 0; k < pick.size(); k++) {
        if (r) break;
        if (rc[k] == OPERATION_SUCCESS) place(k, dst.data() + dst_off[k], dst_len[k]);
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
        const int r2 = pmc_gzip_decompress_batch_host(ctx, src.data(), s2_off.data(), s2_len.data(),
                                                      (uint32_t)again.size(), dst2.data(), d2_off.data(),
                                                      d2_cap.data(), d2_len.data(), rc2.data());
        for (size_t j = 0; j < again.size() && !r2; j++)
            if (rc2[j] == OPERATION_SUCCESS) place(again[j], dst2.data() + d2_off[j], d2_len[j]);
    }
    return out;
}

} // namespace pmc_batch
