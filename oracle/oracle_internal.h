/* oracle_internal.h -- shared internals of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 * Constants are zlib 1.2.11's for deflateInit2(9, Z_DEFLATED, 31, 8, 0), the call the
 * reference makes at /root/reference/src/compressor/gzip_compressor.cpp:12. */
#ifndef PMC_ORACLE_INTERNAL_H
#define PMC_ORACLE_INTERNAL_H
#include <stdint.h>
#include <stddef.h>

#define MIN_MATCH 3
#define MAX_MATCH 258
#define MIN_LOOKAHEAD (MAX_MATCH + MIN_MATCH + 1) /* 262 */
#define W_SIZE 32768u
#define W_MASK (W_SIZE - 1)
#define MAX_DIST (W_SIZE - MIN_LOOKAHEAD) /* 32506 */
#define HASH_SIZE 32768u
#define HASH_MASK (HASH_SIZE - 1)
#define HASH_SHIFT 5
#define LIT_BUFSIZE 16384u /* 1 << (memLevel + 6) */
#define TOO_FAR 4096
#define GOOD_LENGTH 32
#define MAX_LAZY 258
#define NICE_LENGTH 258
#define MAX_CHAIN 4096
#define WIN_INIT MAX_MATCH

#define LENGTH_CODES 29
#define LITERALS 256
#define L_CODES (LITERALS + 1 + LENGTH_CODES) /* 286 */
#define D_CODES 30
#define BL_CODES 19
#define HEAP_SIZE (2 * L_CODES + 1) /* 573 */
#define MAX_BITS 15
#define MAX_BL_BITS 7
#define END_BLOCK 256
#define REP_3_6 16
#define REPZ_3_10 17
#define REPZ_11_138 18
#define SMALLEST 1

/* zlib's ct_data: Freq/Code share one field and Dad/Len share another (trees.c relies on
 * the aliasing, e.g. gen_bitlen overwrites Dad with Len), so the restatement keeps it. */
typedef struct { uint16_t fc, dl; } ct_data;
#define Freq fc
#define Code fc
#define Dad dl
#define Len dl

typedef struct {
    const ct_data *static_tree;
    const int *extra_bits;
    int extra_base, elems, max_length;
} static_tree_desc;

typedef struct {
    ct_data *dyn_tree;
    int max_code;
    const static_tree_desc *stat_desc;
} tree_desc;

/* Per-stream trees.c state (the subset of deflate_state the encoder back end touches). */
typedef struct {
    ct_data dyn_ltree[HEAP_SIZE];
    ct_data dyn_dtree[2 * D_CODES + 1];
    ct_data bl_tree[2 * BL_CODES + 1];
    tree_desc l_desc, d_desc, bl_desc;
    uint16_t bl_count[MAX_BITS + 1];
    int heap[2 * L_CODES + 1];
    int heap_len, heap_max;
    uint8_t depth[2 * L_CODES + 1];
    uint64_t opt_len, static_len;
    /* symbol buffer: l_buf = literal or (length - 3); d_buf = distance or 0 */
    uint8_t l_buf[LIT_BUFSIZE];
    uint16_t d_buf[LIT_BUFSIZE];
    unsigned last_lit;
    /* bit writer (LSB first) */
    uint8_t *out;
    size_t pending;
    uint64_t bi_buf;
    int bi_valid;
    /* stats */
    uint64_t n_stored, n_fixed, n_dynamic;
} tstate;

/* trees.c restatement */
void tr_init(tstate *s, uint8_t *out);
/* returns 1 when the symbol buffer is full (block must be flushed) -- _tr_tally */
int tr_tally_lit(tstate *s, unsigned c);
int tr_tally_dist(tstate *s, unsigned dist, unsigned lc);
/* _tr_flush_block: buf may be NULL (block start slid out of the window) */
void tr_flush_block(tstate *s, const uint8_t *buf, uint64_t stored_len, int last);
void tr_put_byte(tstate *s, uint8_t b);

extern uint8_t pmc_length_code[256];
void tr_static_init(void);
extern uint8_t pmc_dist_code[512];

/* write the 10-byte gzip header zlib emits for level 9 (deflate.c, gzip wrapper) */
void gz_header(uint8_t *out);

#endif
