// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY (oracle/_ref).
//
// C entry points around the reference's own GzipCompressor, compiled straight from
// /root/reference/src/compressor/gzip_compressor.cpp by oracle/Makefile (target _ref).
// Used (a) by tests/golden/make_golden.py to produce the committed golden vectors and
// (b) by bench.py's cpu_baseline leg ("kind": "reference"): the reference codec timed
// on the host cores, one value per call exactly as src/kvs calls it
// (/root/reference/src/kvs/kvs.cpp:183,233).
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "gzip_compressor.hpp"

extern "C" {

int ref_compress(const char *in, char **out, size_t *out_len) {
    CompressResult r = GzipCompressor::Compress(in);
    *out = r.data;
    *out_len = r.size;
    return r.operationResult;
}

int ref_decompress(const char *in, size_t in_len, char **out) {
    DecompressResult r = GzipCompressor::Decompress(in, in_len);
    *out = r.data;
    return r.operationResult;
}

void ref_free(char *p) { delete[] p; }

const char *ref_zlib_version(void) { return zlibVersion(); }

// Times Compress over n values of vlen bytes (NUL-free; each copied into a NUL-terminated
// buffer first, outside the timed region), then Decompress over the results.
// Values are dealt round-robin to nthreads std::threads.
int ref_bench(const uint8_t *values, uint32_t n, uint32_t vlen, int nthreads, double *t_comp,
              double *t_decomp, uint64_t *comp_bytes) {
    std::vector<std::vector<char>> src(n);
    for (uint32_t i = 0; i < n; i++) {
        src[i].resize(vlen + 1);
        memcpy(src[i].data(), values + (uint64_t)i * vlen, vlen);
        src[i][vlen] = 0;
    }
    std::vector<CompressResult> comp(n);
    std::atomic<int> bad{0};
    auto run = [&](auto &&fn) {
        std::vector<std::thread> th;
        auto t0 = std::chrono::steady_clock::now();
        for (int t = 0; t < nthreads; t++)
            th.emplace_back([&, t] {
                for (uint32_t i = t; i < n; i += nthreads) fn(i);
            });
        for (auto &x : th) x.join();
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    *t_comp = run([&](uint32_t i) { comp[i] = GzipCompressor::Compress(src[i].data()); });
    uint64_t cb = 0;
    for (auto &c : comp) cb += c.size;
    *comp_bytes = cb;
    *t_decomp = run([&](uint32_t i) {
        DecompressResult d = GzipCompressor::Decompress(comp[i].data, comp[i].size);
        if (d.operationResult != 0 || memcmp(d.data, src[i].data(), vlen + 1) != 0) bad++;
        delete[] d.data;
    });
    for (auto &c : comp) delete[] c.data;
    return bad.load();
}

// Full-size parity records (tests/golden/make_full_digests.py): value i of vlen bytes goes
// through the reference Compress; lens[i] = member size, crcs[i] = CRC-32 (zlib crc32) of the
// member's bytes.  The digest of a set is SHA-256 over the (u32 len, u32 crc) records, so a GPU
// run can check all 10M members of the headline workload without moving them to the host.
// Returns the number of values whose Compress failed.
int ref_member_records(const uint8_t *values, uint32_t n, uint32_t vlen, int nthreads, uint32_t *lens,
                       uint32_t *crcs) {
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++)
        th.emplace_back([&, t] {
            std::vector<char> s(vlen + 1);
            for (uint32_t i = t; i < n; i += nthreads) {
                memcpy(s.data(), values + (uint64_t)i * vlen, vlen);
                s[vlen] = 0;
                CompressResult c = GzipCompressor::Compress(s.data());
                if (c.operationResult != 0) {
                    bad++;
                    lens[i] = crcs[i] = 0;
                    continue;
                }
                lens[i] = (uint32_t)c.size;
                crcs[i] = (uint32_t)crc32(0L, (const Bytef *)c.data, (uInt)c.size);
                delete[] c.data;
            }
        });
    for (auto &x : th) x.join();
    return bad.load();
}

// Byte-level full-size parity (make_full_digests.py --bytes): the reference's members themselves, member i
// at dst + i * stride (stride >= the member's size), lens[i] its size.  Returns the number of failures.
int ref_members(const uint8_t *values, uint32_t n, uint32_t vlen, int nthreads, uint8_t *dst, uint64_t stride,
                uint32_t *lens) {
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++)
        th.emplace_back([&, t] {
            std::vector<char> s(vlen + 1);
            for (uint32_t i = t; i < n; i += nthreads) {
                memcpy(s.data(), values + (uint64_t)i * vlen, vlen);
                s[vlen] = 0;
                CompressResult c = GzipCompressor::Compress(s.data());
                if (c.operationResult != 0 || c.size > stride) {
                    bad++;
                    lens[i] = 0;
                    delete[] c.data;
                    continue;
                }
                lens[i] = (uint32_t)c.size;
                memcpy(dst + (uint64_t)i * stride, c.data, c.size);
                delete[] c.data;
            }
        });
    for (auto &x : th) x.join();
    return bad.load();
}
}
