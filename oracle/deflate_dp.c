/* deflate_dp.c -- CPU ORACLE (test infrastructure only).
 *
 * Data-parallel-shaped restatement of the same zlib 1.2.11 level-9 encoder as
 * deflate_faithful.c, written in the decomposition the HIP kernels use, so each GPU
 * stage has a CPU twin to be diffed against:
 *
 *  1. h(p) = ((b[p]<<10) ^ (b[p+1]<<5) ^ b[p+2]) & 0x7fff for p <= len-3.  With
 *     HASH_SHIFT 5 and 15 hash bits, zlib's rolling UPDATE_HASH depends only on these
 *     three bytes, and every p <= len-3 is inserted (deflate_slow's INSERT_STRING and the
 *     max_insert bound), so the head/prev chain of p is exactly the list of earlier
 *     positions with the same hash, nearest first.
 *  2. A STABLE sort of positions by h turns every chain into a contiguous run walked
 *     backwards: chain(i) = S[rank(i)-1], S[rank(i)-2], ... while the hash matches.
 *  3. longest_match(i, prev_length) (deflate.c) == over the first C candidates
 *     (C = 4096, or 1024 when prev_length >= good_length 32) the NEAREST candidate with the
 *     largest min(LCP, nice), nice = min(258, len-i); it wins only if that exceeds
 *     prev_length.  The first candidate may sit at distance <= MAX_DIST, later ones at
 *     < MAX_DIST (the caller's `strstart - hash_head <= MAX_DIST` vs the loop's
 *     `> limit`), and a candidate at the current window base is NIL (slide_hash).
 *  4. deflate_slow's lazy decision is a cheap serial scan over those search results.
 *  5. Blocks of 16383 symbols go through the trees.c restatement.
 * Window slides (inputs > 65274 B) are tracked as bookkeeping only: they move the NIL
 * position and make a block's bytes unavailable for a stored block. */
#include <stdlib.h>
#include <string.h>
#include "oracle_internal.h"
#include "pmc_oracle.h"

static oracle_stats g_stats;
void oracle_get_stats(oracle_stats *s) { *s = g_stats; }

typedef struct {
    const uint8_t *b;
    size_t len;
    const uint32_t *S;    /* positions sorted stably by hash */
    const uint32_t *rank; /* rank[p] = index of p in S */
    const uint16_t *h;
} dp_ctx;

static unsigned lcp_capped(const dp_ctx *c, size_t i, size_t q, unsigned cap) {
    unsigned l = 0;
    while (l < cap && c->b[i + l] == c->b[q + l]) l++;
    return l;
}

/* Search result for position i: returns the best length (> b0) or 0 if none beats b0. */
static unsigned dp_search(const dp_ctx *c, size_t i, unsigned b0, size_t B, size_t *qbest) {
    unsigned C = b0 >= GOOD_LENGTH ? MAX_CHAIN >> 2 : MAX_CHAIN;
    size_t rk = c->rank[i];
    unsigned nice = (unsigned)((c->len - i) < NICE_LENGTH ? (c->len - i) : NICE_LENGTH);
    unsigned best = 0, nexam = 0;
    for (size_t k = rk; k-- > 0;) {
        size_t q = c->S[k];
        if (c->h[q] != c->h[i]) break;
        size_t d = i - q;
        if (q <= B) break;
        if (nexam == 0 ? d > MAX_DIST : d >= MAX_DIST) break;
        nexam++;
        unsigned l = lcp_capped(c, i, q, nice);
        if (l > best) { /* strictly longer: nearest wins ties */
            best = l;
            *qbest = q;
            if (l >= nice) break;
        }
        if (nexam == C) break;
    }
    g_stats.searches++;
    g_stats.candidates += nexam;
    return best > b0 ? best : 0;
}

size_t oracle_gzip_compress_dp(const uint8_t *in, size_t len, uint8_t *out) {
    tstate *t = (tstate *)malloc(sizeof(tstate));
    size_t npos = len >= MIN_MATCH ? len - (MIN_MATCH - 1) : 0;
    uint16_t *h = (uint16_t *)malloc((npos + 1) * sizeof(uint16_t));
    uint32_t *S = (uint32_t *)malloc((npos + 1) * sizeof(uint32_t));
    uint32_t *rank = (uint32_t *)malloc((npos + 1) * sizeof(uint32_t));
    uint32_t *cnt = (uint32_t *)calloc(HASH_SIZE + 1, sizeof(uint32_t));
    size_t p, n;
    memset(&g_stats, 0, sizeof(g_stats));
    g_stats.positions = len;

    /* stage 1+2: hashes and a stable counting sort by hash */
    for (p = 0; p < npos; p++) {
        h[p] = (uint16_t)(((in[p] << 10) ^ (in[p + 1] << 5) ^ in[p + 2]) & HASH_MASK);
        cnt[h[p] + 1]++;
    }
    for (unsigned k = 0; k < HASH_SIZE; k++) cnt[k + 1] += cnt[k];
    for (p = 0; p < npos; p++) {
        uint32_t r = cnt[h[p]]++;
        S[r] = (uint32_t)p;
        rank[p] = r;
    }
    dp_ctx c = {in, len, S, rank, h};

    gz_header(out);
    tr_init(t, out);
    t->pending = 10;

    /* stage 3+4: serial lazy parse (deflate_slow) over search results */
    size_t i = 0, B = 0, wend = 0, block_start = 0;
    unsigned match_length = MIN_MATCH - 1, prev_length, match_start = 0, prev_match;
    int match_available = 0, bflush;
#define FLUSH(end, last)                                                             \
    do {                                                                             \
        tr_flush_block(t, block_start >= B ? in + block_start : 0,                   \
                       (uint64_t)((end) - block_start), (last));                     \
        block_start = (end);                                                         \
    } while (0)
    for (;;) {
        if (wend - i < MIN_LOOKAHEAD) { /* fill_window bookkeeping */
            do {
                if (i - B >= W_SIZE + MAX_DIST) B += W_SIZE;
                if (wend == len) break;
                wend = len < B + 2 * W_SIZE ? len : B + 2 * W_SIZE;
            } while (wend - i < MIN_LOOKAHEAD && wend < len);
            if (wend == i) break;
        }
        prev_length = match_length, prev_match = match_start;
        match_length = MIN_MATCH - 1;
        if (i + MIN_MATCH <= len && prev_length < MAX_LAZY) {
            size_t q = 0;
            unsigned m = dp_search(&c, i, prev_length, B, &q);
            if (m) {
                match_length = m;
                match_start = (unsigned)q;
                if (m == MIN_MATCH && i - q > TOO_FAR) match_length = MIN_MATCH - 1;
            }
        }
        if (prev_length >= MIN_MATCH && match_length <= prev_length) {
            bflush = tr_tally_dist(t, (unsigned)(i - 1 - prev_match), prev_length - MIN_MATCH);
            g_stats.matches++;
            i += prev_length - 1;
            match_available = 0;
            match_length = MIN_MATCH - 1;
            if (bflush) FLUSH(i, 0);
        } else if (match_available) {
            bflush = tr_tally_lit(t, in[i - 1]);
            g_stats.literals++;
            if (bflush) FLUSH(i, 0);
            i++;
        } else {
            match_available = 1;
            i++;
        }
    }
    if (match_available) {
        tr_tally_lit(t, in[i - 1]);
        g_stats.literals++;
    }
    FLUSH(i, 1);
#undef FLUSH
    g_stats.stored_blocks = t->n_stored;
    g_stats.fixed_blocks = t->n_fixed;
    g_stats.dynamic_blocks = t->n_dynamic;
    g_stats.blocks = t->n_stored + t->n_fixed + t->n_dynamic;
    n = t->pending;
    uint32_t crc = oracle_crc32(0, in, len);
    for (int k = 0; k < 4; k++) out[n++] = (uint8_t)(crc >> (8 * k));
    for (int k = 0; k < 4; k++) out[n++] = (uint8_t)((uint64_t)len >> (8 * k));
    free(t), free(h), free(S), free(rank), free(cnt);
    return n;
}
