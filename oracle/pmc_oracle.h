/*
 * pmc_oracle.h -- CPU ORACLE for the value-codec hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker.  The product path (poor-man-s-cache_amd/) never
 * links or calls it; it fails loudly when its HIP library is missing.
 *
 * What it restates: the arithmetic behind the reference's GzipCompressor
 * (/root/reference/src/compressor/gzip_compressor.cpp:3-111), which lives entirely in
 * the third-party zlib it links (not vendored under /root/reference; the reference pins
 * no version, Dockerfile:2 `apk add zlib-dev`).  The restatement follows the published
 * zlib 1.2.11 algorithm (deflate.c: deflate_slow / longest_match / fill_window /
 * slide_hash with configuration_table[9] = {32,258,258,4096}; trees.c; inflate.c;
 * crc32.c) with the reference's parameters deflateInit2(9, Z_DEFLATED, 15+16, 8,
 * Z_DEFAULT_STRATEGY) (gzip_compressor.cpp:12) and inflateInit2(15+16)
 * (gzip_compressor.cpp:62).
 *
 * Parity pin: tests/golden/ holds outputs of the reference Compress itself, compiled
 * from /root/reference/src/compressor/gzip_compressor.cpp by oracle/Makefile into
 * oracle/_ref/ (see tests/golden/make_golden.py).  tests/test_oracle.py checks both
 * restatements byte-for-byte against them.
 */
#ifndef PMC_ORACLE_H
#define PMC_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Worst-case gzip member size for an input of len bytes (any content, any size). */
size_t oracle_gzip_bound(size_t len);

/* Faithful streaming restatement of zlib 1.2.11 deflate level 9 + gzip wrapper.
 * Returns the number of bytes written to out (capacity >= oracle_gzip_bound(len)). */
size_t oracle_gzip_compress(const uint8_t *in, size_t len, uint8_t *out);

/* Data-parallel-shaped restatement (the decomposition the HIP kernels use):
 * per-position hash -> stable sort by hash -> candidate windows -> serial lazy parse
 * -> per-block Huffman -> bit emit.  Must equal oracle_gzip_compress byte for byte. */
size_t oracle_gzip_compress_dp(const uint8_t *in, size_t len, uint8_t *out);

/* gzip-only inflate with zlib 1.2.11 inflateInit2(31) validation rules.
 * Returns 0 (Z_STREAM_END reached), -3 (Z_DATA_ERROR) or -5 (Z_BUF_ERROR: truncated
 * input -- the reference loops forever here; this is the documented
 * divergence), or ORACLE_E_CAPACITY (-101) when the stream decodes past out_cap: output beyond
 * out_cap is counted but not stored, *out_len receives the decoded size and the caller retries
 * with that capacity (the reference grows its buffer instead, gzip_compressor.cpp:71-77, so
 * capacity is never a verdict).  Bytes after the first member's trailer are ignored
 * (gzip_compressor.cpp:96 stops at Z_STREAM_END). */
#define ORACLE_E_CAPACITY (-101)
int oracle_gzip_decompress(const uint8_t *in, size_t in_len, uint8_t *out, size_t out_cap,
                           size_t *out_len);

uint32_t oracle_crc32(uint32_t crc, const uint8_t *p, size_t n);

/* Instrumentation for DESIGN.md: counts from the last oracle_gzip_compress_dp call. */
typedef struct {
    uint64_t positions, searches, candidates, literals, matches, blocks;
    uint64_t stored_blocks, fixed_blocks, dynamic_blocks;
} oracle_stats;
void oracle_get_stats(oracle_stats *s);

/* splitmix64-based synthetic value generator shared with the GPU generator
 * (SURVEY.md §8d): value i of size V is corpus[off_i : off_i+V],
 * off_i = splitmix64(seed ^ i) mod (corpus_len - V + 1). kind 1 = random [A-Za-z0-9]. */
uint64_t oracle_splitmix64(uint64_t x);
uint64_t oracle_murmur3_x64_128_h1(const uint8_t *data, int len, uint32_t seed);
void oracle_gen_values(const uint8_t *corpus, size_t corpus_len, uint64_t seed, int kind,
                       uint64_t first, uint32_t n, uint32_t vlen, uint8_t *out);
void oracle_gen_values_idx(const uint8_t *corpus, size_t corpus_len, uint64_t seed, int kind,
                           const uint64_t *index, uint32_t n, uint32_t vlen, uint8_t *out);
void oracle_route_keys(uint64_t first, uint64_t n, uint32_t num_shards, uint32_t n_gpus, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
