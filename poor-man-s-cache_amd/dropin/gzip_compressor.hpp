// gzip_compressor.hpp -- drop-in replacement for the reference's
// /root/reference/src/compressor/gzip_compressor.hpp (same macros, structs, class and
// static methods, lines 10-44), backed by the MI355X codec (include/pmc_codec.h) instead
// of zlib.  src/kvs (kvs.cpp:183, :233) compiles and links against it unchanged: build
// this file in place of src/compressor/gzip_compressor.cpp and link libpmc_codec.so.
#pragma once
#include <cstddef>
#include <cstring>
#include <stdexcept>

#define CHUNK_SIZE 16384 // kept for source compatibility (reference output chunk size)
#define INVALID_INPUT -999
#define OPERATION_SUCCESS 0

/// @brief Result of compress operation
struct CompressResult {
    /// @brief Pointer to compressed data (new[]-allocated; caller delete[]s)
    char *data;
    /// @brief Size of data
    size_t size;
    /// @brief 0 on success, -999 on invalid input, otherwise a zlib-style / pmc code
    int operationResult;
};

/// @brief Result of decompress operation
struct DecompressResult {
    /// @brief Pointer to NUL-terminated decompressed data (new[]-allocated)
    char *data;
    /// @brief 0 on success, -999 on invalid input, -3 corrupt, -5 truncated
    int operationResult;
};

class GzipCompressor {
  public:
    /// @brief gzip (zlib level 9 bit-exact) compression of a C string on the GPU.
    static CompressResult Compress(const char *input);

    /// @brief gzip decompression on the GPU; result is NUL-terminated.
    static DecompressResult Decompress(const char *input, size_t input_size);
};
