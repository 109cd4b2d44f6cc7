// batch_codec.hpp -- the codec half of SURVEY.md §8 f1 (a batched server path): what a server's
// request loop calls once per epoll batch instead of one GzipCompressor call per value.
//
// The reference compresses inside KeyValueStore::insertEntry, one value at a time
// (/root/reference/src/kvs/kvs.cpp:148, :182-196): vSize = strlen(value) + 1; compress only if
// compression is enabled and vSize >= 30; on rc == 0 store the member and its size with
// compressed = true, otherwise copy the raw value including its NUL.  GET decompresses a
// compressed entry (kvs.cpp:224, :233-234) and hands out the NUL-terminated value, or nullptr if
// decompression fails.  The functions below make the same per-value decisions and return the
// same bytes and ownership (new[] buffers the caller delete[]s), for a whole batch in one
// pmc_gzip_*_batch_host call each.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string_view>
#include <vector>

// (gzip_compressor.hpp is not included here: a TU that also sees the reference's own copy of that
// header through src/kvs -- the f1 server hook -- would get its structs twice)
struct pmc_ctx;
struct CompressResult;
struct DecompressResult;

namespace pmc_batch {

/// Minimum strlen(value) + 1 that the reference compresses (kvs.cpp:182).
constexpr size_t kMinCompressSize = 30;

/// What insertEntry stores for one SET value.
struct StoredValue {
    char *data;       ///< new[]: gzip member if compressed, else the raw value with its NUL
    size_t size;      ///< bytes in data (the member size, or strlen + 1)
    bool compressed;  ///< Entry::compressed (kvs.hpp:38-44)
    int rc;           ///< codec verdict for compressed attempts (0), or the failure code that made
                      ///< the value fall back to a raw copy; INVALID_INPUT for a null value
};

/// SET side: one StoredValue per value, in order.  `compression_enabled` mirrors
/// KeyValueStore's flag.  Values that fail compression are stored raw, as the reference does.
std::vector<StoredValue> CompressForSet(const std::vector<const char *> &values, bool compression_enabled = true,
                                        pmc_ctx *ctx = nullptr);

/// One stored entry read by a GET.
struct Entry {
    const char *data;
    size_t size;
    bool compressed;
};

/// GET side: for each entry, the value a GET returns: compressed entries are decompressed into a
/// NUL-terminated new[] buffer (nullptr if decompression fails, kvs.cpp:233-234); raw entries
/// return their stored pointer unchanged (not a copy, as in kvs.cpp:224).  `owned[i]` says
/// whether result i is a new[] buffer the caller must delete[].
std::vector<char *> DecompressForGet(const std::vector<Entry> &entries, std::vector<bool> *owned = nullptr,
                                     pmc_ctx *ctx = nullptr);

// ---- f1 inside the UNCHANGED caller: priming GzipCompressor for one request batch ----------------
// kvs.cpp keeps calling GzipCompressor::Compress / ::Decompress one value at a time (:183, :233).  A
// server loop that knows its batch (the epoll iteration, server.cpp:361-390) primes those calls first:
// every value of the batch is compressed (and every member decompressed) by ONE device batch call,
// and the per-value calls that follow are answered from the primed results.  State is per thread
// (the reference serves requests on one thread, server.cpp:631-643) and lives until EndBatch().

/// Compress the batch's SET values (the C strings Compress will be called with: strlen'd bytes,
/// values shorter than kMinCompressSize - 1 are skipped).  A later Compress(v) with the same bytes
/// gets the primed member (matched by content: kvs copies the value before compressing it).
void PrimeCompress(const std::vector<std::string_view> &values, pmc_ctx *ctx = nullptr);
/// PrimeCompress with the device batch on a helper thread and a context of its own, so the iteration's
/// GET dry run and decompress batch (BeginCollect .. PrimeCollected, on the default context) overlap it;
/// PrimeCompressWait() joins it and files its results (call it before the values are compressed).
/// The views must stay valid until then.
void PrimeCompressAsync(const std::vector<std::string_view> &values);
void PrimeCompressWait();

/// Between BeginCollect() and PrimeCollected(), Decompress(ptr, size) only records (ptr, size) and
/// returns {nullptr, INVALID_INPUT}: a dry run of the batch's GETs (kvs::get is a pure lookup)
/// learns which stored members they will decompress.  PrimeCollected() decompresses them in one
/// device call; a later Decompress(ptr, size) of the same stored bytes gets the primed value
/// (matched by pointer, size and content, so a buffer freed and reused meanwhile never matches).
void BeginCollect();
void PrimeCollected(pmc_ctx *ctx = nullptr);

/// Drop the primed results the batch did not use (their buffers are freed).
void EndBatch();

/// Counters of the calling thread: primed compress / decompress results handed out, and calls that
/// found no primed result (ran the single-value path).
struct PrimeStats {
    size_t compress_hits, compress_misses, decompress_hits, decompress_misses, batches;
    size_t store_values;   ///< device-store mode: compressed values held in HBM now (live handles)
    uint64_t store_bytes;  ///< ... and the heap bytes their members use
};
PrimeStats GetPrimeStats();

// ---- f2 inside the UNCHANGED kvs: compressed values held in HBM ---------------------------------------
// Device-store mode (a server that calls EnableDeviceStore before its first request): Compress returns,
// instead of the gzip member, a 32-byte handle naming the member's extent in a device store (pmc_store_*),
// and kvs keeps that handle as Entry.value / vSize with compressed = true (kvs.cpp:185-187).  Decompress of a
// handle decodes the extent on the device.  The batch priming above works unchanged (the SET batch is one
// pmc_store_put_batch, the GET dry run's handles one pmc_store_get_batch).  Handles live in a slab of their
// own, so the server's replacement of operator delete[] (kvs frees Entry.value with delete[],
// kvs.hpp:87-98) recognises one by its address and releases its extent: ReleaseIfHandle.
void EnableDeviceStore(uint64_t heap_bytes);

namespace detail {
bool StoreMode();
/// p inside the handle slab: release its extent and slot, return true (else false: not a handle)
bool ReleaseIfHandle(void *p) noexcept;
bool StoreCompress(const char *input, size_t len, CompressResult *out);
bool StoreDecompress(const char *input, size_t size, DecompressResult *out);
} // namespace detail

namespace detail {
// used by GzipCompressor (gzip_compressor.cpp)
bool TakeCompressed(const char *input, size_t len, CompressResult *out);
bool Collecting(const char *input, size_t size);
bool TakeDecompressed(const char *input, size_t size, DecompressResult *out);
} // namespace detail

} // namespace pmc_batch
