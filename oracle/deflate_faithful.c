/* deflate_faithful.c -- CPU ORACLE (test infrastructure only).
 *
 * Streaming restatement of zlib 1.2.11 deflate.c for the exact configuration the
 * reference uses: deflateInit2(Z_BEST_COMPRESSION=9, Z_DEFLATED, 15+16, 8,
 * Z_DEFAULT_STRATEGY) followed by deflate(Z_FINISH) (/root/reference/src/compressor/
 * gzip_compressor.cpp:12,35-40).  The whole input is available on the first call, and
 * the reference's 16 KiB output chunking does not change the bit stream, so the output
 * goes straight into one buffer.
 *
 * Restated: fill_window (incl. slide_hash and the WIN_INIT high-water zeroing),
 * read_buf (+CRC-32), INSERT_STRING/UPDATE_HASH, longest_match (level-9 parameters
 * good=32 lazy=258 nice=258 chain=4096), deflate_slow (lazy evaluation, TOO_FAR=4096),
 * FLUSH_BLOCK, and the gzip header/trailer.  Kept deliberately zlib-shaped: it is the
 * reference semantics the data-parallel restatement (deflate_dp.c) and the HIP kernels
 * are diffed against. */
#include <stdlib.h>
#include <string.h>
#include "oracle_internal.h"
#include "pmc_oracle.h"

typedef struct {
    tstate t;
    uint8_t window[2 * W_SIZE];
    uint64_t window_size;
    uint16_t prev[W_SIZE];
    uint16_t head[HASH_SIZE];
    unsigned ins_h;
    long block_start;
    unsigned strstart, match_start, lookahead, prev_length, match_length, prev_match;
    int match_available;
    unsigned insert;
    uint64_t high_water;
    const uint8_t *next_in;
    size_t avail_in;
    uint32_t crc;
    uint64_t total_in;
} dstate;

#define UPDATE_HASH(h, c) (h = (((h) << HASH_SHIFT) ^ (c)) & HASH_MASK)
#define INSERT_STRING(s, str, match_head)                                  \
    (UPDATE_HASH((s)->ins_h, (s)->window[(str) + (MIN_MATCH - 1)]),          \
     match_head = (s)->prev[(str) & W_MASK] = (s)->head[(s)->ins_h],        \
     (s)->head[(s)->ins_h] = (uint16_t)(str))

static unsigned read_buf(dstate *s, uint8_t *buf, unsigned size) {
    unsigned len = s->avail_in < size ? (unsigned)s->avail_in : size;
    if (len == 0) return 0;
    memcpy(buf, s->next_in, len);
    s->crc = oracle_crc32(s->crc, buf, len);
    s->next_in += len;
    s->avail_in -= len;
    s->total_in += len;
    return len;
}

static void slide_hash(dstate *s) {
    unsigned n, m;
    for (n = 0; n < HASH_SIZE; n++) {
        m = s->head[n];
        s->head[n] = (uint16_t)(m >= W_SIZE ? m - W_SIZE : 0);
    }
    for (n = 0; n < W_SIZE; n++) {
        m = s->prev[n];
        s->prev[n] = (uint16_t)(m >= W_SIZE ? m - W_SIZE : 0);
    }
}

static void fill_window(dstate *s) {
    unsigned n, more;
    do {
        more = (unsigned)(s->window_size - (uint64_t)s->lookahead - (uint64_t)s->strstart);
        if (s->strstart >= W_SIZE + MAX_DIST) {
            memcpy(s->window, s->window + W_SIZE, (unsigned)W_SIZE - more);
            s->match_start -= W_SIZE;
            s->strstart -= W_SIZE;
            s->block_start -= (long)W_SIZE;
            slide_hash(s);
            more += W_SIZE;
        }
        if (s->avail_in == 0) break;
        n = read_buf(s, s->window + s->strstart + s->lookahead, more);
        s->lookahead += n;
        if (s->lookahead + s->insert >= MIN_MATCH) {
            unsigned str = s->strstart - s->insert;
            s->ins_h = s->window[str];
            UPDATE_HASH(s->ins_h, s->window[str + 1]);
            while (s->insert) {
                UPDATE_HASH(s->ins_h, s->window[str + MIN_MATCH - 1]);
                s->prev[str & W_MASK] = s->head[s->ins_h];
                s->head[s->ins_h] = (uint16_t)str;
                str++;
                s->insert--;
                if (s->lookahead + s->insert < MIN_MATCH) break;
            }
        }
    } while (s->lookahead < MIN_LOOKAHEAD && s->avail_in != 0);

    if (s->high_water < s->window_size) {
        uint64_t curr = s->strstart + (uint64_t)s->lookahead, init;
        if (s->high_water < curr) {
            init = s->window_size - curr;
            if (init > WIN_INIT) init = WIN_INIT;
            memset(s->window + curr, 0, (unsigned)init);
            s->high_water = curr + init;
        } else if (s->high_water < curr + WIN_INIT) {
            init = curr + WIN_INIT - s->high_water;
            if (init > s->window_size - s->high_water) init = s->window_size - s->high_water;
            memset(s->window + s->high_water, 0, (unsigned)init);
            s->high_water += init;
        }
    }
}

/* longest_match (deflate.c, non-UNALIGNED_OK variant) */
static unsigned longest_match(dstate *s, unsigned cur_match) {
    unsigned chain_length = MAX_CHAIN;
    uint8_t *scan = s->window + s->strstart, *match;
    int len;
    int best_len = (int)s->prev_length;
    int nice_match = NICE_LENGTH;
    unsigned limit = s->strstart > (unsigned)MAX_DIST ? s->strstart - (unsigned)MAX_DIST : 0;
    uint8_t *strend = s->window + s->strstart + MAX_MATCH;
    uint8_t scan_end1 = scan[best_len - 1];
    uint8_t scan_end = scan[best_len];

    if (s->prev_length >= GOOD_LENGTH) chain_length >>= 2;
    if ((unsigned)nice_match > s->lookahead) nice_match = (int)s->lookahead;
    do {
        match = s->window + cur_match;
        if (match[best_len] != scan_end || match[best_len - 1] != scan_end1 || *match != *scan ||
            *++match != scan[1])
            continue;
        scan += 2, match++;
        do {
        } while (*++scan == *++match && *++scan == *++match && *++scan == *++match &&
                 *++scan == *++match && *++scan == *++match && *++scan == *++match &&
                 *++scan == *++match && *++scan == *++match && scan < strend);
        len = MAX_MATCH - (int)(strend - scan);
        scan = strend - MAX_MATCH;
        if (len > best_len) {
            s->match_start = cur_match;
            best_len = len;
            if (len >= nice_match) break;
            scan_end1 = scan[best_len - 1];
            scan_end = scan[best_len];
        }
    } while ((cur_match = s->prev[cur_match & W_MASK]) > limit && --chain_length != 0);

    if ((unsigned)best_len <= s->lookahead) return (unsigned)best_len;
    return s->lookahead;
}

#define FLUSH_BLOCK_ONLY(s, last)                                                          \
    tr_flush_block(&(s)->t,                                                                \
                   (s)->block_start >= 0L ? (s)->window + (unsigned)(s)->block_start : 0, \
                   (uint64_t)((long)(s)->strstart - (s)->block_start), (last)),           \
        (s)->block_start = (long)(s)->strstart

/* deflate_slow (deflate.c) with flush == Z_FINISH throughout */
static void deflate_slow(dstate *s) {
    unsigned hash_head;
    int bflush;
    for (;;) {
        if (s->lookahead < MIN_LOOKAHEAD) {
            fill_window(s);
            if (s->lookahead == 0) break;
        }
        hash_head = 0;
        if (s->lookahead >= MIN_MATCH) INSERT_STRING(s, s->strstart, hash_head);

        s->prev_length = s->match_length, s->prev_match = s->match_start;
        s->match_length = MIN_MATCH - 1;

        if (hash_head != 0 && s->prev_length < MAX_LAZY && s->strstart - hash_head <= MAX_DIST) {
            s->match_length = longest_match(s, hash_head);
            if (s->match_length <= 5 &&
                (s->match_length == MIN_MATCH && s->strstart - s->match_start > TOO_FAR))
                s->match_length = MIN_MATCH - 1;
        }
        if (s->prev_length >= MIN_MATCH && s->match_length <= s->prev_length) {
            unsigned max_insert = s->strstart + s->lookahead - MIN_MATCH;
            bflush = tr_tally_dist(&s->t, s->strstart - 1 - s->prev_match, s->prev_length - MIN_MATCH);
            s->lookahead -= s->prev_length - 1;
            s->prev_length -= 2;
            do {
                if (++s->strstart <= max_insert) INSERT_STRING(s, s->strstart, hash_head);
            } while (--s->prev_length != 0);
            s->match_available = 0;
            s->match_length = MIN_MATCH - 1;
            s->strstart++;
            if (bflush) FLUSH_BLOCK_ONLY(s, 0);
        } else if (s->match_available) {
            bflush = tr_tally_lit(&s->t, s->window[s->strstart - 1]);
            if (bflush) FLUSH_BLOCK_ONLY(s, 0);
            s->strstart++;
            s->lookahead--;
        } else {
            s->match_available = 1;
            s->strstart++;
            s->lookahead--;
        }
    }
    if (s->match_available) {
        tr_tally_lit(&s->t, s->window[s->strstart - 1]);
        s->match_available = 0;
    }
    s->insert = s->strstart < MIN_MATCH - 1 ? s->strstart : MIN_MATCH - 1;
    FLUSH_BLOCK_ONLY(s, 1);
}

size_t oracle_gzip_bound(size_t len) {
    /* stored fallback: 5 B per 16383-symbol block; fixed/dynamic after a slide: <= 9/8 */
    return len + (len >> 3) + 6 * (len / 16383 + 1) + 32;
}

size_t oracle_gzip_compress(const uint8_t *in, size_t len, uint8_t *out) {
    dstate *s = (dstate *)calloc(1, sizeof(dstate));
    size_t n;
    gz_header(out);
    tr_init(&s->t, out);
    s->t.pending = 10;
    s->window_size = 2 * (uint64_t)W_SIZE;
    s->match_length = s->prev_length = MIN_MATCH - 1;
    s->next_in = in;
    s->avail_in = len;
    s->crc = 0;
    deflate_slow(s);
    n = s->t.pending;
    for (int k = 0; k < 4; k++) out[n++] = (uint8_t)(s->crc >> (8 * k));
    for (int k = 0; k < 4; k++) out[n++] = (uint8_t)(s->total_in >> (8 * k));
    free(s);
    return n;
}
