/*
 * pmc_codec.h -- C-ABI of the MI355X-native value codec (libpmc_codec.so).
 *
 * Drop-in boundary for the reference's src/compressor.  The reference
 * exposes two static C++ methods, called only from src/kvs:
 *   GzipCompressor::Compress(const char*)            /root/reference/src/compressor/gzip_compressor.hpp:37
 *                                                     (impl gzip_compressor.cpp:3-50; caller kvs.cpp:183)
 *   GzipCompressor::Decompress(const char*, size_t)  /root/reference/src/compressor/gzip_compressor.hpp:43
 *                                                     (impl gzip_compressor.cpp:52-111; caller kvs.cpp:233)
 * The reference links them at build time (no FFI); poor-man-s-cache_amd/dropin/
 * gzip_compressor.{hpp,cpp} re-implements that class on top of this ABI so src/kvs links
 * unchanged.  Everything here is plain pointers and sizes; no torch or HIP types appear
 * in the signatures (streams are passed as void* = hipStream_t).
 *
 * Output bytes are bit-identical to the reference Compress (zlib 1.2.11, level 9,
 * windowBits 15+16, memLevel 8, default strategy) on the same input bytes.
 *
 * Return codes mirror the reference (gzip_compressor.hpp:10-12) and zlib:
 */
#ifndef PMC_CODEC_H
#define PMC_CODEC_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define PMC_OK 0                 /* OPERATION_SUCCESS (gzip_compressor.hpp:12)            */
#define PMC_INVALID_INPUT (-999) /* INVALID_INPUT: null or empty (gzip_compressor.hpp:11) */
#define PMC_Z_DATA_ERROR (-3)    /* corrupt stream, CRC/ISIZE mismatch, not gzip           */
#define PMC_Z_MEM_ERROR (-4)     /* device allocation failed                               */
#define PMC_Z_BUF_ERROR (-5)     /* truncated stream (reference hangs here)     */
#define PMC_E_NO_DEVICE (-100)   /* no usable gfx950 device / HIP runtime error            */
#define PMC_E_CAPACITY (-101)    /* output capacity too small; decompress: dst_len = needed  */
#define PMC_E_ARG (-102)         /* invalid argument                                       */

/* One device + streams + scratch.  The host-memory calls (single value, *_batch_host,
 * *_batch_pinned) lock the context, so threads may share one (the drop-in shares the default
 * context, keeping the reference's reentrant static methods reentrant) and they restore the
 * caller's current HIP device.  The device-resident batch calls only enqueue work: see their
 * note on streams below. */
typedef struct pmc_ctx pmc_ctx;

/* Create a context on HIP device `device` (gfx950).  Returns PMC_OK or PMC_E_NO_DEVICE. */
int pmc_ctx_create(int device, pmc_ctx **out);
void pmc_ctx_destroy(pmc_ctx *ctx);
/* Default context (device 0), created on first use; used by the drop-in. */
pmc_ctx *pmc_default_ctx(void);
const char *pmc_last_error(void);
/* Library version string and the device arch it was built for ("gfx950"). */
const char *pmc_version(void);

/* Worst-case gzip member size for an input of `len` bytes. */
size_t pmc_gzip_bound(size_t len);

/* ---- single value, host memory (what GzipCompressor::Compress/Decompress wrap) ----
 * pmc_gzip_compress: compress in[0..in_len) into out (capacity out_cap >= pmc_gzip_bound).
 *   in_len == 0 or in == NULL -> PMC_INVALID_INPUT (gzip_compressor.cpp:4).
 * pmc_gzip_decompress: decompress the first gzip member of in[0..in_len) (bytes after its
 *   trailer are ignored, as the reference's inflate loop stops at Z_STREAM_END,
 *   gzip_compressor.cpp:96); *out_len receives the size.  The caller sizes `out` from
 *   pmc_gzip_isize() (the last 4 bytes: right unless bytes follow the member).  If the stream
 *   decodes past out_cap the call returns PMC_E_CAPACITY with *out_len = the decoded size and
 *   no verdict yet: call again with that much room (the reference grows its buffer instead,
 *   :71-77, so capacity is never one of its verdicts). */
int pmc_gzip_compress(pmc_ctx *ctx, const void *in, size_t in_len, void *out, size_t out_cap,
                      size_t *out_len);
int pmc_gzip_decompress(pmc_ctx *ctx, const void *in, size_t in_len, void *out, size_t out_cap,
                        size_t *out_len);
/* ISIZE trailer of a gzip member (last 4 bytes, little endian); 0 if in_len < 18. */
uint32_t pmc_gzip_isize(const void *in, size_t in_len);

/* ---- batched, DEVICE-resident (the hot path) ------------------------------------------
 * Value i occupies src[src_off[i] .. src_off[i]+src_len[i]); its gzip member is written to
 * dst[dst_off[i] ..), at most dst_cap[i] bytes, its length to dst_len[i] and its status to
 * rc[i].  All arrays are device pointers; the call only enqueues work on `stream`
 * (hipStream_t, NULL = legacy default stream) and returns -- except that a compress call whose
 * max_len exceeds the split pipeline's limit (~31.8 KB) reads the number and lengths of its large
 * values back to plan their scratch, so it waits for the stream up to that point.  max_len is an upper bound on
 * src_len[] (for compress) or on the decompressed sizes (for decompress); it selects the
 * kernel variant (LDS-resident vs HBM-resident working set).  Compress: a value with
 * src_len[i] > max_len is not compressed; it gets rc[i] = PMC_E_ARG, dst_len[i] = 0
 * (checked on the device).  Values are independent, so a batch may be split arbitrarily
 * across calls and GPUs.  Scratch is per context and per direction: the library orders two
 * compress calls (or two decompress calls) of one context that are issued on different
 * streams (the later one waits for the earlier one on the device); a compress and a
 * decompress call of one context may run concurrently on two streams.
 * Compress: src_len[i] == 0 -> rc PMC_INVALID_INPUT (reference semantics).  Input bytes
 *   may contain NULs (binary safe; the single-value drop-in keeps the reference's strlen).
 * Decompress: dst_cap[i] should be >= the decompressed size (ISIZE); use
 *   pmc_gzip_isize_batch to read the trailers on device.  Bytes after a member's trailer are
 *   ignored (gzip_compressor.cpp:96).  A member that decodes past dst_cap[i] gets
 *   rc[i] = PMC_E_CAPACITY and dst_len[i] = its decoded size (no verdict yet; decode it again
 *   with that capacity). */
int pmc_gzip_compress_batch(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                            const uint32_t *src_len, uint32_t n, uint8_t *dst, const uint64_t *dst_off,
                            const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc, uint32_t max_len,
                            void *stream);
int pmc_gzip_decompress_batch(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                              const uint32_t *src_len, uint32_t n, uint8_t *dst, const uint64_t *dst_off,
                              const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc, uint32_t max_len,
                              void *stream);
/* crc[i] = CRC-32 (the gzip trailer's, zlib crc32.c) of buf[off[i] .. off[i] + len[i]), all
 * device-resident; the engine of decompression's CRC check, exported for callers that verify
 * stored members themselves.  Stream-ordered like the batch calls above. */
int pmc_crc32_batch(pmc_ctx *ctx, const uint8_t *buf, const uint64_t *off, const uint32_t *len,
                    uint32_t n, uint32_t *crc, void *stream);
/* isize[i] = ISIZE trailer of member i (0 if src_len[i] < 18). */
int pmc_gzip_isize_batch(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                         const uint32_t *src_len, uint32_t n, uint32_t *isize, void *stream);

/* ---- batched, HOST-resident (what a batched server path would call) --------------------
 * Same layout, all pointers in host memory.  Stages through pinned buffers with
 * hipMemcpyAsync H2D -> kernel -> D2H on the context's stream and waits for completion.
 * dst_off may be NULL: outputs are then packed back to back in dst (dst_off[i] = sum of
 * previous dst_cap[]). */
int pmc_gzip_compress_batch_host(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                 const uint32_t *src_len, uint32_t n, uint8_t *dst,
                                 const uint64_t *dst_off, const uint32_t *dst_cap, uint32_t *dst_len,
                                 int32_t *rc);
int pmc_gzip_decompress_batch_host(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                   const uint32_t *src_len, uint32_t n, uint8_t *dst,
                                   const uint64_t *dst_off, const uint32_t *dst_cap, uint32_t *dst_len,
                                   int32_t *rc);

/* ---- batched, PINNED host memory, pipelined (the PCIe-inclusive path) --------------------
 * Same layout as the host-resident calls, but every pointer is host memory that the caller has
 * pinned (hipHostMalloc / hipHostRegister).  The batch is cut into chunks of `chunk` values
 * (0 = max(65536, n/16)); the H2D copy of chunk c+1 and the D2H copy of chunk c-1 run on two
 * context-owned copy streams beside chunk c's kernels, so the PCIe legs hide behind the codec.
 * Chunk c's source bytes are copied as the range [min src_off, max src_off+src_len) of its
 * values.  max_len as for the device calls.  Returns after the last chunk has landed.
 *   Slot mode (dst_off given): output i at dst + dst_off[i].  If a chunk's slots tile one range
 *     in index order (dst_off[i+1] == dst_off[i] + dst_cap[i]) that range is written back whole
 *     (slot bytes past dst_len[i], and failed values' slots, hold unspecified bytes); any other
 *     layout (gaps, permuted or interleaved slots) is compacted on the device and each output is
 *     copied to its dst_off on the host, so only [dst_off[i], dst_off[i] + dst_len[i]) of
 *     successful values is written.
 *   Packed mode (dst_off NULL): outputs back to back in index order (output i at the sum of
 *     dst_len[j] over j < i with rc[j] == 0; a failed value takes no bytes).  The device
 *     compacts each chunk, so only the real output bytes cross PCIe; dst must hold
 *     sum(dst_cap).  This is what a SET batch wants: ~C bytes per value back, not dst_cap.
 * Replaces nothing in the reference (which has no batch API); it is the host side of
 * SURVEY.md §8(d)'s host-to-host rate and the call a batched server path (§8 f1) makes. */
int pmc_gzip_compress_batch_pinned(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                   const uint32_t *src_len, uint32_t n, uint8_t *dst, const uint64_t *dst_off,
                                   const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc, uint32_t max_len,
                                   uint32_t chunk);
int pmc_gzip_decompress_batch_pinned(pmc_ctx *ctx, const uint8_t *src, const uint64_t *src_off,
                                     const uint32_t *src_len, uint32_t n, uint8_t *dst, const uint64_t *dst_off,
                                     const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc, uint32_t max_len,
                                     uint32_t chunk);

/* ---- device-resident compressed value store -----------------------
 * Keeps the compressed bytes of cache values in HBM instead of host memory: the reference's
 * Entry.value of a compressed entry (/root/reference/src/kvs/kvs.hpp:38-44, filled at
 * kvs.cpp:185-187) becomes a pmc_extent, an extent of one device heap.  The caller keeps its own
 * key index (the reference's hash table stays on the host) and stores the extent in it.
 *   put: values (host memory) -> pinned staging -> H2D -> compress into the put's device staging
 *        -> lengths come back -> extents of the MEMBER's size (rounded to 16 B) are allocated and
 *        the members compacted into them on the device: the heap holds ~C bytes per value.
 *   get: extents -> decompress on the device into a packed response image, optionally framed
 *        as the server's wire format (f3: the custom protocol's value + 0x1F, or a RESP bulk
 *        string "$<len>\r\n<value>\r\n", /root/reference/src/server/protocol.cpp:399-406,
 *        466-497) -> one D2H into the store's pinned buffer; resp[i] points into it (valid
 *        until the next get on this store), ready for sendmsg without another copy.
 *   free: extents return to the store's free lists (size classes).
 * Calls are synchronous (return after the device work completed).  A put and a get (or
 * read_members) may run at the same time from two threads (compress and decompress streams,
 * separate staging); two puts, or two gets, are serialized. */
typedef struct pmc_store pmc_store;
typedef struct pmc_extent {
    uint64_t off;     /* byte offset in the store's device heap */
    uint32_t cap;     /* bytes reserved */
    uint32_t len;     /* compressed (gzip member) bytes */
    uint32_t raw_len; /* value bytes (the member's ISIZE) */
    uint32_t flags;   /* 0 = empty, 1 = live */
} pmc_extent;
#define PMC_FRAME_RAW 0    /* the value bytes only                                       */
#define PMC_FRAME_CUSTOM 1 /* value + 0x1F (custom protocol response, protocol.hpp:17)   */
#define PMC_FRAME_RESP 2   /* "$<len>\r\n" value "\r\n" (RESP bulk string)               */
/* heap_bytes: device heap size (the extents live here; 0 = 1 GiB). */
int pmc_store_create(pmc_ctx *ctx, uint64_t heap_bytes, pmc_store **out);
void pmc_store_destroy(pmc_store *s);
/* Compress value i (src + src_off[i], src_len[i] bytes, host memory) into a new extent:
 * ext[i] (flags 1) and rc[i] = 0, or rc[i] = PMC_Z_MEM_ERROR (heap full) / a codec code with
 * ext[i].flags = 0.  Returns PMC_OK unless the call itself failed; then every value's rc[i] holds
 * the failure, ext[i].flags = 0 and no extent stays allocated. */
int pmc_store_put_batch(pmc_store *s, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                        uint32_t n, pmc_extent *ext, int32_t *rc);
/* Decompress extents into framed responses (frame = PMC_FRAME_*): resp[i], resp_len[i], rc[i]. */
int pmc_store_get_batch(pmc_store *s, const pmc_extent *ext, uint32_t n, int frame, const uint8_t **resp,
                        uint32_t *resp_len, int32_t *rc);
/* The same with a frame per extent (frames[i] = PMC_FRAME_*): one batch answers connections of
 * both protocols, as one epoll iteration of the reference server does (server.cpp:434-478 frames
 * custom and RESP requests side by side; responses at protocol.cpp:399-406 and :466-497). */
int pmc_store_get_batch_frames(pmc_store *s, const pmc_extent *ext, uint32_t n, const uint8_t *frames,
                               const uint8_t **resp, uint32_t *resp_len, int32_t *rc);
/* Copy extents' compressed bytes (gzip members) to host memory: member i at dst + dst_off[i]. */
int pmc_store_read_members(pmc_store *s, const pmc_extent *ext, uint32_t n, uint8_t *dst,
                           const uint64_t *dst_off);
/* Release extents (flags set to 0); freeing an empty extent is a no-op. */
int pmc_store_free(pmc_store *s, pmc_extent *ext, uint32_t n);
/* used: bytes held by live extents; reserved: heap bytes handed out so far; heap: heap size. */
int pmc_store_stats(pmc_store *s, uint64_t *used, uint64_t *reserved, uint64_t *heap);

/* ---- fixed-slot device slab (device-resident callers) ---------------------
 * For callers whose keys, values and bookkeeping already live on the device (bench.py --mix,
 * BASELINE configs[2]): slot s holds at most one gzip member, at pmc_slab_data() + s * stride
 * (stride = pmc_gzip_bound(max_value_len) rounded to 16 B), its length in pmc_slab_lengths()[s]
 * (0 = empty).  All arrays are device pointers; set / get only enqueue on `stream`.
 *   set: compress value i (src_len[i] <= max_value_len) into slot[i] and record its length (0 on
 *        failure); the slots of one set call must be distinct.
 *   get: decompress slot[i] into dst + dst_off[i] (an empty slot gives PMC_INVALID_INPUT).
 * A set and a get may run concurrently on two streams (the caller orders a get after the set
 * whose member it must see); two sets (or two gets) on different streams are ordered by the library. */
typedef struct pmc_slab pmc_slab;
int pmc_slab_create(pmc_ctx *ctx, uint32_t slots, uint32_t max_value_len, pmc_slab **out);
void pmc_slab_destroy(pmc_slab *s);
uint8_t *pmc_slab_data(pmc_slab *s);
uint32_t *pmc_slab_lengths(pmc_slab *s);
uint64_t pmc_slab_stride(pmc_slab *s);
int pmc_slab_set(pmc_slab *s, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                 const uint32_t *slot, uint32_t n, int32_t *rc, void *stream);
int pmc_slab_get(pmc_slab *s, const uint32_t *slot, uint32_t n, uint8_t *dst, const uint64_t *dst_off,
                 const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc, void *stream);

/* ---- several GPUs from one process -----------------------------------------
 * The reference server is one process that routes key k to shard hashFunc(k) % numShards
 * (/root/reference/src/server/server.cpp:113,121,132).  A group holds one context per entry of
 * `devices` (entries may repeat: two contexts on one GPU behave like two GPUs); value i of a group
 * batch goes to member (key_hash[i] % num_shards) % n, each member's share runs through its own
 * context's pinned pipelined call on its own host thread, and outputs land at dst_off[i] in the
 * caller's order.  All pointers are host memory (any, not necessarily pinned).  No collective. */
typedef struct pmc_group pmc_group;
/* hashFunc(key) of the reference: MurmurHash3_x64_128(key, len, seed 0)[0] (hash.cpp:4-9). */
uint64_t pmc_key_hash(const void *key, size_t len);
int pmc_group_create(const int *devices, int n, pmc_group **out);
void pmc_group_destroy(pmc_group *g);
int pmc_group_size(pmc_group *g);
/* member[i] = (key_hash[i] % num_shards) % pmc_group_size(g) */
int pmc_group_route(pmc_group *g, const uint64_t *key_hash, uint32_t num_shards, uint32_t n, uint32_t *member);
int pmc_group_compress_batch(pmc_group *g, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                             const uint64_t *key_hash, uint32_t num_shards, uint32_t n, uint8_t *dst,
                             const uint64_t *dst_off, const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc,
                             uint32_t max_len);
int pmc_group_decompress_batch(pmc_group *g, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                               const uint64_t *key_hash, uint32_t num_shards, uint32_t n, uint8_t *dst,
                               const uint64_t *dst_off, const uint32_t *dst_cap, uint32_t *dst_len, int32_t *rc,
                               uint32_t max_len);

/* ---- benchmark / test helpers (device, enqueue only) -----------------------------------
 * Synthetic values of SURVEY.md §8d: value i of vlen bytes written to dst + i*vlen, with
 * global index idx = index ? index[i] : first+i.  kind 0 = slice of corpus at
 * splitmix64(seed ^ idx) % (corpus_len-vlen+1); kind 1 = random [A-Za-z0-9] (8-byte group g:
 * splitmix64(splitmix64(seed ^ idx) + g)).  corpus and index are device pointers. */
int pmc_gen_values(const uint8_t *corpus, uint32_t corpus_len, uint64_t seed, int kind, uint64_t first,
                   const uint64_t *index, uint32_t n, uint32_t vlen, uint8_t *dst, void *stream);
/* Fixed-stride layout: off[i] = i*stride, len[i] = vlen (device arrays). */
int pmc_fill_layout(uint64_t *off, uint32_t *len, uint32_t *cap, uint32_t n, uint64_t stride,
                    uint32_t vlen, uint32_t capv, void *stream);
/* mismatches[0] += number of values whose bytes differ between a and b (device). */
int pmc_compare_values(const uint8_t *a, const uint64_t *a_off, const uint8_t *b, const uint64_t *b_off,
                       const uint32_t *len, const uint32_t *len_b, uint32_t n, uint32_t *mismatches,
                       void *stream);
/* shard routing: gpu[i] = MurmurHash3_x64_128("key"+(first+i), seed 0)[0]
 * % num_shards % n_gpus  (hash.cpp:4-9 routing, server.cpp:113,121,132). */
int pmc_route_keys(uint64_t first, uint32_t n, uint32_t num_shards, uint32_t n_gpus, uint8_t *gpu,
                   void *stream);

/* Diagnostics: in a library built with -DPMC_STAMPS, the kernels add per-phase cycle sums
 * into dev_buf (32 x uint64, device memory: [0,16) deflate, [16,32) inflate); NULL disables.
 * No effect otherwise. */
int pmc_debug_stamps(pmc_ctx *ctx, uint64_t *dev_buf);

/* Per-kernel launch timing (roofline diagnostics, bench.py): while enabled, every kernel the
 * batched calls enqueue is bracketed by HIP events on its stream.  pmc_ctx_kernel_times
 * synchronizes the context's work, adds each kind's summed milliseconds and launch count
 * to ms[kind] / launches[kind] (kind < nkinds, indices PMC_K_*) and clears the record. */
#define PMC_K_DEFLATE_FRONT 0 /* split pipeline: stage, hash sort, lazy parse, histograms */
#define PMC_K_DEFLATE_TREES 1 /* split pipeline: lane-parallel Huffman trees + block plan */
#define PMC_K_DEFLATE_BACK 2  /* split pipeline: CRC, codes, emission, framing           */
#define PMC_K_DEFLATE_MONO 3  /* single-kernel small-value deflate (PMC_DEFLATE_MONO=1)  */
#define PMC_K_DEFLATE_HBM 4   /* values > 16382 B                                       */
#define PMC_K_INFLATE_LDS 5
#define PMC_K_INFLATE_HBM 6
#define PMC_K_INFLATE_LANE 7   /* lane-per-member decode fast path                     */
#define PMC_K_INFLATE_VERIFY 8 /* CRC-32 check of the fast path's output               */
#define PMC_K_ORDER 9          /* lane visit-order counting sorts (trees, lane inflate)  */
#define PMC_K_INFLATE_REC 10   /* two-phase record decode of members up to 4 KiB output */
#define PMC_K_DEFLATE_LARGE 11 /* large values: hash sort, segment parses, stitching     */
#define PMC_K_DEFLATE_LARGE_EMIT 12 /* large values: blocks of the stitched tokens      */
#define PMC_K_COUNT 13
int pmc_ctx_profile(pmc_ctx *ctx, int enable);
int pmc_ctx_kernel_times(pmc_ctx *ctx, double *ms, uint32_t *launches, int nkinds);

/* Lane-order guards (build-owned; no reference counterpart).  The throughput compressor's hash
 * sort and canonical-code ranks take a lane's rank from a returning LDS atomic, relying on the
 * lanes of one ds_add_rtn_u32 that hit the same word getting their old values in lane order
 * (measured on gfx950, not documented).  Every value is checked where the data already is; a value
 * that fails is recompressed by the HBM kernel, which does not rely on it, so output stays
 * bit-exact.  Synchronizes the device and copies out the context's counters: counts[0] values
 * whose sort failed the check, counts[1] values whose code ranks failed it, counts[2] violations
 * in pmc_ctx_create's self-test (nonzero: the context compresses through the single-kernel path),
 * counts[3] values the other paths handed to the HBM kernel (31.8 KB-class values of several
 * DEFLATE blocks; large values whose segment parses did not stitch), counts[4] members the
 * decompress fast paths (record / lane kernels) handed to the wave-per-member kernels (stored or
 * unusual blocks, and every error verdict). */
int pmc_ctx_guard_counts(pmc_ctx *ctx, uint32_t counts[5]);

/* Host-call routing counters (build-owned; no reference counterpart).  Every host-memory call
 * (pmc_gzip_*_batch_host and the single-value pmc_gzip_compress / pmc_gzip_decompress on top of it)
 * takes one of two routes: the latency path (one wave-per-value kernel reading and writing coherent
 * host memory in place; compress: <= 1,024 values of <= 4 KiB; decompress: <= 4,096 members of
 * <= 48 KiB output, at most 16 MiB in all) or the throughput pipeline (pinned staging, H2D, the
 * kernel pipeline, D2H).  counts[0] / counts[1]: compress / decompress calls on the latency path;
 * counts[2] / counts[3]: on the pipeline.  Host-side, no device synchronization.  (The
 * device-resident pmc_gzip_*_batch calls route batches within the same limits -- and decompress
 * batches of at most 4 members per CU of any size -- to the same one-kernel paths; they are not
 * counted here.) */
int pmc_ctx_path_counts(pmc_ctx *ctx, uint64_t counts[4]);

/* Latency-path compress calls whose declined values were redone (build-owned).  The latency path's
 * one kernel has no retry pass of its own: a value it declines (a lane-order guard fired, see
 * pmc_ctx_guard_counts) is compressed again, alone with the call's other declined values, by a
 * throughput-pipeline call into the caller's buffers (which also counts in counts[2] above).
 * *n = the number of latency-path calls that needed that.  Host-side, no device synchronization. */
int pmc_ctx_latency_redone(pmc_ctx *ctx, uint64_t *n);

#ifdef __cplusplus
}
#endif
#endif
