/* trees.c -- CPU ORACLE (test infrastructure only): restatement of zlib 1.2.11 trees.c,
 * the Huffman back end behind the reference's deflate(Z_FINISH) call
 * (/root/reference/src/compressor/gzip_compressor.cpp:38).
 *
 * Restated functions (zlib 1.2.11 trees.c): tr_static_init, init_block, pqdownheap,
 * gen_bitlen, gen_codes, build_tree, scan_tree, send_tree, build_bl_tree,
 * send_all_trees, _tr_stored_block, _tr_flush_block, _tr_tally, compress_block,
 * bi_windup.  Heap tie-breaking (`smaller` on freq then depth) and the Dad/Len field
 * aliasing are kept exactly, because they decide which of two equal-frequency symbols
 * gets the longer code. */
#include <string.h>
#include "oracle_internal.h"

static const int extra_lbits[LENGTH_CODES] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                              2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const int extra_dbits[D_CODES] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                         6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const int extra_blbits[BL_CODES] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
static const uint8_t bl_order[BL_CODES] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static ct_data static_ltree[L_CODES + 2];
static ct_data static_dtree[D_CODES];
uint8_t pmc_dist_code[512];
uint8_t pmc_length_code[256];
static int base_length[LENGTH_CODES];
static int base_dist[D_CODES];
static int static_done;

static const static_tree_desc static_l_desc = {static_ltree, extra_lbits, LITERALS + 1, L_CODES, MAX_BITS};
static const static_tree_desc static_d_desc = {static_dtree, extra_dbits, 0, D_CODES, MAX_BITS};
static const static_tree_desc static_bl_desc = {0, extra_blbits, 0, BL_CODES, MAX_BL_BITS};

static unsigned bi_reverse(unsigned code, int len) {
    unsigned res = 0;
    do {
        res |= code & 1;
        code >>= 1, res <<= 1;
    } while (--len > 0);
    return res >> 1;
}

/* gen_codes (trees.c): canonical codes from bit lengths, stored bit-reversed */
static void gen_codes(ct_data *tree, int max_code, const uint16_t *bl_count) {
    uint16_t next_code[MAX_BITS + 1];
    unsigned code = 0;
    for (int bits = 1; bits <= MAX_BITS; bits++) {
        code = (code + bl_count[bits - 1]) << 1;
        next_code[bits] = (uint16_t)code;
    }
    for (int n = 0; n <= max_code; n++) {
        int len = tree[n].Len;
        if (len == 0) continue;
        tree[n].Code = (uint16_t)bi_reverse(next_code[len]++, len);
    }
}

/* tr_static_init (trees.c) */
void tr_static_init(void) {
    if (static_done) return;
    int n, code, length = 0, dist = 0, bits;
    uint16_t bl_count[MAX_BITS + 1];
    for (code = 0; code < LENGTH_CODES - 1; code++) {
        base_length[code] = length;
        for (n = 0; n < (1 << extra_lbits[code]); n++) pmc_length_code[length++] = (uint8_t)code;
    }
    /* length 258 (lc 255) is sent as code 285, overwrite */
    pmc_length_code[length - 1] = (uint8_t)code;
    base_length[LENGTH_CODES - 1] = 0; /* unused: code 28 has no extra bits */
    for (code = 0; code < 16; code++) {
        base_dist[code] = dist;
        for (n = 0; n < (1 << extra_dbits[code]); n++) pmc_dist_code[dist++] = (uint8_t)code;
    }
    dist >>= 7;
    for (; code < D_CODES; code++) {
        base_dist[code] = dist << 7;
        for (n = 0; n < (1 << (extra_dbits[code] - 7)); n++) pmc_dist_code[256 + dist++] = (uint8_t)code;
    }
    for (bits = 0; bits <= MAX_BITS; bits++) bl_count[bits] = 0;
    n = 0;
    while (n <= 143) static_ltree[n++].Len = 8, bl_count[8]++;
    while (n <= 255) static_ltree[n++].Len = 9, bl_count[9]++;
    while (n <= 279) static_ltree[n++].Len = 7, bl_count[7]++;
    while (n <= 287) static_ltree[n++].Len = 8, bl_count[8]++;
    gen_codes(static_ltree, L_CODES + 1, bl_count);
    for (n = 0; n < D_CODES; n++) {
        static_dtree[n].Len = 5;
        static_dtree[n].Code = (uint16_t)bi_reverse((unsigned)n, 5);
    }
    static_done = 1;
}

#define d_code(dist) ((dist) < 256 ? pmc_dist_code[dist] : pmc_dist_code[256 + ((dist) >> 7)])

/* ---- bit writer: LSB-first, identical byte stream to zlib's 16-bit bi_buf ---- */
void tr_put_byte(tstate *s, uint8_t b) { s->out[s->pending++] = b; }

static void send_bits(tstate *s, unsigned value, int length) {
    s->bi_buf |= (uint64_t)value << s->bi_valid;
    s->bi_valid += length;
    while (s->bi_valid >= 8) {
        s->out[s->pending++] = (uint8_t)s->bi_buf;
        s->bi_buf >>= 8;
        s->bi_valid -= 8;
    }
}
#define send_code(s, c, tree) send_bits(s, (tree)[c].Code, (tree)[c].Len)

static void bi_windup(tstate *s) {
    if (s->bi_valid > 0) s->out[s->pending++] = (uint8_t)s->bi_buf;
    s->bi_buf = 0;
    s->bi_valid = 0;
}

/* init_block (trees.c) */
static void init_block(tstate *s) {
    int n;
    for (n = 0; n < L_CODES; n++) s->dyn_ltree[n].Freq = 0;
    for (n = 0; n < D_CODES; n++) s->dyn_dtree[n].Freq = 0;
    for (n = 0; n < BL_CODES; n++) s->bl_tree[n].Freq = 0;
    s->dyn_ltree[END_BLOCK].Freq = 1;
    s->opt_len = s->static_len = 0;
    s->last_lit = 0;
}

void tr_init(tstate *s, uint8_t *out) {
    tr_static_init();
    memset(s, 0, sizeof(*s));
    s->l_desc.dyn_tree = s->dyn_ltree;
    s->l_desc.stat_desc = &static_l_desc;
    s->d_desc.dyn_tree = s->dyn_dtree;
    s->d_desc.stat_desc = &static_d_desc;
    s->bl_desc.dyn_tree = s->bl_tree;
    s->bl_desc.stat_desc = &static_bl_desc;
    s->out = out;
    init_block(s);
}

/* smaller / pqdownheap (trees.c) */
#define smaller(tree, n, m, depth) \
    (tree[n].Freq < tree[m].Freq || (tree[n].Freq == tree[m].Freq && depth[n] <= depth[m]))

static void pqdownheap(tstate *s, ct_data *tree, int k) {
    int v = s->heap[k];
    int j = k << 1;
    while (j <= s->heap_len) {
        if (j < s->heap_len && smaller(tree, s->heap[j + 1], s->heap[j], s->depth)) j++;
        if (smaller(tree, v, s->heap[j], s->depth)) break;
        s->heap[k] = s->heap[j];
        k = j;
        j <<= 1;
    }
    s->heap[k] = v;
}

/* gen_bitlen (trees.c), including the bit-length overflow redistribution */
static void gen_bitlen(tstate *s, tree_desc *desc) {
    ct_data *tree = desc->dyn_tree;
    int max_code = desc->max_code;
    const ct_data *stree = desc->stat_desc->static_tree;
    const int *extra = desc->stat_desc->extra_bits;
    int base = desc->stat_desc->extra_base;
    int max_length = desc->stat_desc->max_length;
    int h, n, m, bits, xbits, overflow = 0;
    uint16_t f;

    for (bits = 0; bits <= MAX_BITS; bits++) s->bl_count[bits] = 0;
    tree[s->heap[s->heap_max]].Len = 0; /* root */
    for (h = s->heap_max + 1; h < HEAP_SIZE; h++) {
        n = s->heap[h];
        bits = tree[tree[n].Dad].Len + 1;
        if (bits > max_length) bits = max_length, overflow++;
        tree[n].Len = (uint16_t)bits;
        if (n > max_code) continue; /* not a leaf */
        s->bl_count[bits]++;
        xbits = 0;
        if (n >= base) xbits = extra[n - base];
        f = tree[n].Freq;
        s->opt_len += (uint64_t)f * (unsigned)(bits + xbits);
        if (stree) s->static_len += (uint64_t)f * (unsigned)(stree[n].Len + xbits);
    }
    if (overflow == 0) return;
    do {
        bits = max_length - 1;
        while (s->bl_count[bits] == 0) bits--;
        s->bl_count[bits]--;
        s->bl_count[bits + 1] += 2;
        s->bl_count[max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    for (bits = max_length; bits != 0; bits--) {
        n = s->bl_count[bits];
        while (n != 0) {
            m = s->heap[--h];
            if (m > max_code) continue;
            if ((unsigned)tree[m].Len != (unsigned)bits) {
                s->opt_len += ((uint64_t)bits - tree[m].Len) * tree[m].Freq;
                tree[m].Len = (uint16_t)bits;
            }
            n--;
        }
    }
}

/* build_tree (trees.c) */
static void build_tree(tstate *s, tree_desc *desc) {
    ct_data *tree = desc->dyn_tree;
    const ct_data *stree = desc->stat_desc->static_tree;
    int elems = desc->stat_desc->elems;
    int n, m, max_code = -1, node;

    s->heap_len = 0, s->heap_max = HEAP_SIZE;
    for (n = 0; n < elems; n++) {
        if (tree[n].Freq != 0) {
            s->heap[++(s->heap_len)] = max_code = n;
            s->depth[n] = 0;
        } else {
            tree[n].Len = 0;
        }
    }
    while (s->heap_len < 2) {
        node = s->heap[++(s->heap_len)] = (max_code < 2 ? ++max_code : 0);
        tree[node].Freq = 1;
        s->depth[node] = 0;
        s->opt_len--;
        if (stree) s->static_len -= stree[node].Len;
    }
    desc->max_code = max_code;
    for (n = s->heap_len / 2; n >= 1; n--) pqdownheap(s, tree, n);
    node = elems;
    do {
        n = s->heap[SMALLEST]; /* pqremove */
        s->heap[SMALLEST] = s->heap[s->heap_len--];
        pqdownheap(s, tree, SMALLEST);
        m = s->heap[SMALLEST];
        s->heap[--(s->heap_max)] = n;
        s->heap[--(s->heap_max)] = m;
        tree[node].Freq = tree[n].Freq + tree[m].Freq;
        s->depth[node] = (uint8_t)((s->depth[n] >= s->depth[m] ? s->depth[n] : s->depth[m]) + 1);
        tree[n].Dad = tree[m].Dad = (uint16_t)node;
        s->heap[SMALLEST] = node++;
        pqdownheap(s, tree, SMALLEST);
    } while (s->heap_len >= 2);
    s->heap[--(s->heap_max)] = s->heap[SMALLEST];
    gen_bitlen(s, desc);
    gen_codes(tree, max_code, s->bl_count);
}

/* scan_tree (trees.c) */
static void scan_tree(tstate *s, ct_data *tree, int max_code) {
    int n, prevlen = -1, curlen, nextlen = tree[0].Len, count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    tree[max_code + 1].Len = (uint16_t)0xffff; /* guard */
    for (n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[n + 1].Len;
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            s->bl_tree[curlen].Freq += count;
        } else if (curlen != 0) {
            if (curlen != prevlen) s->bl_tree[curlen].Freq++;
            s->bl_tree[REP_3_6].Freq++;
        } else if (count <= 10) {
            s->bl_tree[REPZ_3_10].Freq++;
        } else {
            s->bl_tree[REPZ_11_138].Freq++;
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

/* send_tree (trees.c) */
static void send_tree(tstate *s, ct_data *tree, int max_code) {
    int n, prevlen = -1, curlen, nextlen = tree[0].Len, count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    for (n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[n + 1].Len;
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            do { send_code(s, curlen, s->bl_tree); } while (--count != 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) {
                send_code(s, curlen, s->bl_tree);
                count--;
            }
            send_code(s, REP_3_6, s->bl_tree);
            send_bits(s, count - 3, 2);
        } else if (count <= 10) {
            send_code(s, REPZ_3_10, s->bl_tree);
            send_bits(s, count - 3, 3);
        } else {
            send_code(s, REPZ_11_138, s->bl_tree);
            send_bits(s, count - 11, 7);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

/* build_bl_tree (trees.c) */
static int build_bl_tree(tstate *s) {
    int max_blindex;
    scan_tree(s, s->dyn_ltree, s->l_desc.max_code);
    scan_tree(s, s->dyn_dtree, s->d_desc.max_code);
    build_tree(s, &s->bl_desc);
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
        if (s->bl_tree[bl_order[max_blindex]].Len != 0) break;
    s->opt_len += 3 * ((uint64_t)max_blindex + 1) + 5 + 5 + 4;
    return max_blindex;
}

static void send_all_trees(tstate *s, int lcodes, int dcodes, int blcodes) {
    send_bits(s, lcodes - 257, 5);
    send_bits(s, dcodes - 1, 5);
    send_bits(s, blcodes - 4, 4);
    for (int rank = 0; rank < blcodes; rank++) send_bits(s, s->bl_tree[bl_order[rank]].Len, 3);
    send_tree(s, s->dyn_ltree, lcodes - 1);
    send_tree(s, s->dyn_dtree, dcodes - 1);
}

/* compress_block (trees.c) */
static void compress_block(tstate *s, const ct_data *ltree, const ct_data *dtree) {
    unsigned dist, lx = 0, code;
    int lc, extra;
    if (s->last_lit != 0) do {
            dist = s->d_buf[lx];
            lc = s->l_buf[lx++];
            if (dist == 0) {
                send_code(s, lc, ltree);
            } else {
                code = pmc_length_code[lc];
                send_code(s, code + LITERALS + 1, ltree);
                extra = extra_lbits[code];
                if (extra != 0) {
                    lc -= base_length[code];
                    send_bits(s, lc, extra);
                }
                dist--;
                code = d_code(dist);
                send_code(s, code, dtree);
                extra = extra_dbits[code];
                if (extra != 0) {
                    dist -= (unsigned)base_dist[code];
                    send_bits(s, dist, extra);
                }
            }
        } while (lx < s->last_lit);
    send_code(s, END_BLOCK, ltree);
}

/* _tr_stored_block (trees.c) */
static void tr_stored_block(tstate *s, const uint8_t *buf, uint64_t stored_len, int last) {
    send_bits(s, (0 << 1) + last, 3);
    bi_windup(s);
    tr_put_byte(s, (uint8_t)(stored_len & 0xff));
    tr_put_byte(s, (uint8_t)((stored_len >> 8) & 0xff));
    tr_put_byte(s, (uint8_t)(~stored_len & 0xff));
    tr_put_byte(s, (uint8_t)((~stored_len >> 8) & 0xff));
    memcpy(s->out + s->pending, buf, stored_len);
    s->pending += stored_len;
}

/* _tr_flush_block (trees.c), level > 0, strategy Z_DEFAULT_STRATEGY */
void tr_flush_block(tstate *s, const uint8_t *buf, uint64_t stored_len, int last) {
    uint64_t opt_lenb, static_lenb;
    int max_blindex;
    build_tree(s, &s->l_desc);
    build_tree(s, &s->d_desc);
    max_blindex = build_bl_tree(s);
    opt_lenb = (s->opt_len + 3 + 7) >> 3;
    static_lenb = (s->static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    if (stored_len + 4 <= opt_lenb && buf != 0) {
        tr_stored_block(s, buf, stored_len, last);
        s->n_stored++;
    } else if (static_lenb == opt_lenb) {
        send_bits(s, (1 << 1) + last, 3);
        compress_block(s, static_ltree, static_dtree);
        s->n_fixed++;
    } else {
        send_bits(s, (2 << 1) + last, 3);
        send_all_trees(s, s->l_desc.max_code + 1, s->d_desc.max_code + 1, max_blindex + 1);
        compress_block(s, s->dyn_ltree, s->dyn_dtree);
        s->n_dynamic++;
    }
    init_block(s);
    if (last) bi_windup(s);
}

/* _tr_tally (trees.c): flush when the buffer holds lit_bufsize-1 = 16383 symbols */
int tr_tally_lit(tstate *s, unsigned c) {
    s->d_buf[s->last_lit] = 0;
    s->l_buf[s->last_lit++] = (uint8_t)c;
    s->dyn_ltree[c].Freq++;
    return s->last_lit == LIT_BUFSIZE - 1;
}

int tr_tally_dist(tstate *s, unsigned dist, unsigned lc) {
    s->d_buf[s->last_lit] = (uint16_t)dist;
    s->l_buf[s->last_lit++] = (uint8_t)lc;
    dist--;
    s->dyn_ltree[pmc_length_code[lc] + LITERALS + 1].Freq++;
    s->dyn_dtree[d_code(dist)].Freq++;
    return s->last_lit == LIT_BUFSIZE - 1;
}

/* gzip header as deflate() writes it with no gzhead: FLG 0, MTIME 0,
 * XFL 2 (level 9), OS_CODE 3 (Unix) */
void gz_header(uint8_t *out) {
    static const uint8_t h[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 2, 3};
    memcpy(out, h, 10);
}
