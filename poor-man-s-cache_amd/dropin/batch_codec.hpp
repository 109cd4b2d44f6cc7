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
#include <vector>

#include "gzip_compressor.hpp"

struct pmc_ctx;

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

} // namespace pmc_batch
