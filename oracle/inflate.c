/* inflate.c -- CPU ORACLE (test infrastructure only).
 *
 * gzip-only inflate restating zlib 1.2.11 inflate.c / inftrees.c semantics as driven by
 * the reference's Decompress (inflateInit2(15+16) + inflate(Z_NO_FLUSH) loop,
 * /root/reference/src/compressor/gzip_compressor.cpp:52-111):
 *   - header: magic 1f 8b else "incorrect header check"; CM must be 8; FLG bits 5-7 must
 *     be 0; FEXTRA/FNAME/FCOMMENT skipped; FHCRC verified (wrap & 4)   -> -3 on failure
 *   - blocks: stored (LEN/NLEN check), fixed (codes 286/287, dist 30/31 invalid), dynamic
 *     (HLIT<=286, HDIST<=30, code-length code must be complete, lit/dist codes may be
 *     incomplete only when their longest code is 1 bit, EOB must have a code, repeat-16
 *     needs a previous length, repeats may not overrun)                  -> -3
 *   - distance beyond the bytes produced so far ("too far back")         -> -3
 *   - trailer: CRC-32 then ISIZE                                           -> -3
 *   - running out of input anywhere                                        -> -5
 *     (the reference loops forever on Z_BUF_ERROR; returning -5 is the documented
 *     divergence)
 * Bits are consumed in the same order zlib consumes them, so the truncated-vs-corrupt
 * verdict matches zlib's on every prefix. */
#include <string.h>
#include "pmc_oracle.h"

#define Z_DATA_ERROR (-3)
#define Z_BUF_ERROR (-5)

typedef struct {
    const uint8_t *in;
    size_t in_len;
    uint64_t bitpos; /* next unread bit */
    uint8_t *out;
    size_t out_cap;
    uint64_t out_n;
    uint32_t crc_run; /* crc of bytes we stored (only valid while out_n <= out_cap) */
} ist;

typedef struct {
    uint16_t count[16];
    uint16_t symbol[320];
    int max; /* longest code length (0: no codes) */
} huff;

static int need(ist *s, unsigned n) { return s->bitpos + n <= (uint64_t)s->in_len * 8; }

static unsigned getbits(ist *s, unsigned n) {
    unsigned v = 0;
    for (unsigned k = 0; k < n; k++) {
        uint64_t b = s->bitpos + k;
        v |= (unsigned)((s->in[b >> 3] >> (b & 7)) & 1) << k;
    }
    s->bitpos += n;
    return v;
}

/* inftrees.c check: 0 ok, -1 over-subscribed / incomplete (incomplete allowed only for
 * type != CODES with max code length 1). */
static int build(huff *h, const uint16_t *lens, int n, int is_codes) {
    int left = 1, len, sym;
    uint16_t offs[16];
    memset(h->count, 0, sizeof(h->count));
    for (sym = 0; sym < n; sym++) h->count[lens[sym]]++;
    h->max = 0;
    for (len = 15; len >= 1; len--)
        if (h->count[len]) { h->max = len; break; }
    if (h->max == 0) return 0; /* all zero: table of invalid codes (1 bit each) */
    for (len = 1; len <= 15; len++) {
        left <<= 1;
        left -= h->count[len];
        if (left < 0) return -1;
    }
    if (left > 0 && (is_codes || h->max != 1)) return -1;
    offs[1] = 0;
    for (len = 1; len < 15; len++) offs[len + 1] = offs[len] + h->count[len];
    for (sym = 0; sym < n; sym++)
        if (lens[sym]) h->symbol[offs[lens[sym]]++] = (uint16_t)sym;
    return 0;
}

/* decode one symbol: >=0 symbol, -1 invalid code, -2 out of input */
static int decode(ist *s, const huff *h) {
    int code = 0, first = 0, index = 0;
    if (h->max == 0) { /* zlib's max==0 table: every 1-bit pattern is the invalid marker */
        if (!need(s, 1)) return -2;
        getbits(s, 1);
        return -1;
    }
    for (int len = 1; len <= h->max; len++) {
        if (!need(s, 1)) return -2;
        code |= (int)getbits(s, 1);
        int count = h->count[len];
        if (code - count < first) return h->symbol[index + (code - first)];
        index += count;
        first += count;
        first <<= 1;
        code <<= 1;
    }
    return -1; /* only reachable for an incomplete (max==1) code */
}

static void put(ist *s, uint8_t b) {
    if (s->out_n < s->out_cap) s->out[s->out_n] = b;
    s->out_n++;
}

static const uint16_t lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint16_t lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
                                   257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint16_t dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

static int codes(ist *s, const huff *lh, const huff *dh) {
    for (;;) {
        int sym = decode(s, lh);
        if (sym == -2) return Z_BUF_ERROR;
        if (sym < 0) return Z_DATA_ERROR;
        if (sym < 256) {
            put(s, (uint8_t)sym);
        } else if (sym == 256) {
            return 0;
        } else {
            sym -= 257;
            if (sym >= 29) return Z_DATA_ERROR; /* 286/287 in fixed code */
            if (!need(s, lext[sym])) return Z_BUF_ERROR;
            unsigned len = lbase[sym] + getbits(s, lext[sym]);
            int ds = decode(s, dh);
            if (ds == -2) return Z_BUF_ERROR;
            if (ds < 0 || ds >= 30) return Z_DATA_ERROR;
            if (!need(s, dext[ds])) return Z_BUF_ERROR;
            unsigned dist = dbase[ds] + getbits(s, dext[ds]);
            if (dist > s->out_n) return Z_DATA_ERROR; /* invalid distance too far back */
            for (unsigned k = 0; k < len; k++) {
                uint64_t src = s->out_n - dist;
                put(s, src < s->out_cap ? s->out[src] : 0);
            }
        }
    }
}

static const uint8_t cl_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

int oracle_gzip_decompress(const uint8_t *in, size_t in_len, uint8_t *out, size_t out_cap,
                           size_t *out_len) {
    ist st = {in, in_len, 0, out, out_cap, 0, 0};
    ist *s = &st;
    size_t p;
    *out_len = 0;
    /* ---- header (inflate.c HEAD..HCRC) ---- */
    if (in_len < 2) return Z_BUF_ERROR;
    if (in[0] != 0x1f || in[1] != 0x8b) return Z_DATA_ERROR;
    if (in_len < 4) return Z_BUF_ERROR;
    if (in[2] != 8) return Z_DATA_ERROR;
    unsigned flg = in[3];
    if (flg & 0xe0) return Z_DATA_ERROR;
    p = 4;
    if (in_len < p + 4) return Z_BUF_ERROR; /* MTIME */
    p += 4;
    if (in_len < p + 2) return Z_BUF_ERROR; /* XFL, OS */
    p += 2;
    if (flg & 0x04) { /* FEXTRA */
        if (in_len < p + 2) return Z_BUF_ERROR;
        size_t xlen = in[p] | ((size_t)in[p + 1] << 8);
        p += 2;
        if (in_len < p + xlen) return Z_BUF_ERROR;
        p += xlen;
    }
    if (flg & 0x08) { /* FNAME */
        while (p < in_len && in[p] != 0) p++;
        if (p >= in_len) return Z_BUF_ERROR;
        p++;
    }
    if (flg & 0x10) { /* FCOMMENT */
        while (p < in_len && in[p] != 0) p++;
        if (p >= in_len) return Z_BUF_ERROR;
        p++;
    }
    if (flg & 0x02) { /* FHCRC */
        if (in_len < p + 2) return Z_BUF_ERROR;
        unsigned hc = in[p] | ((unsigned)in[p + 1] << 8);
        if (hc != (oracle_crc32(0, in, p) & 0xffff)) return Z_DATA_ERROR;
        p += 2;
    }
    s->bitpos = (uint64_t)p * 8;
    /* ---- blocks ---- */
    int last;
    do {
        if (!need(s, 3)) return Z_BUF_ERROR;
        last = (int)getbits(s, 1);
        unsigned type = getbits(s, 2);
        if (type == 0) {
            s->bitpos = (s->bitpos + 7) & ~(uint64_t)7;
            if (!need(s, 32)) return Z_BUF_ERROR;
            unsigned len = getbits(s, 16), nlen = getbits(s, 16);
            if (len != (nlen ^ 0xffff)) return Z_DATA_ERROR;
            for (unsigned k = 0; k < len; k++) {
                if (!need(s, 8)) return Z_BUF_ERROR;
                put(s, (uint8_t)getbits(s, 8));
            }
        } else if (type == 1) {
            static huff fl, fd;
            static int fixed_ready;
            if (!fixed_ready) {
                uint16_t l[288];
                int k;
                for (k = 0; k < 144; k++) l[k] = 8;
                for (; k < 256; k++) l[k] = 9;
                for (; k < 280; k++) l[k] = 7;
                for (; k < 288; k++) l[k] = 8;
                build(&fl, l, 288, 0);
                for (k = 0; k < 32; k++) l[k] = 5;
                build(&fd, l, 32, 0);
                fixed_ready = 1;
            }
            int rc = codes(s, &fl, &fd);
            if (rc) return rc;
        } else if (type == 2) {
            uint16_t lens[320];
            huff clh, lh, dh;
            if (!need(s, 14)) return Z_BUF_ERROR;
            int nlen = (int)getbits(s, 5) + 257, ndist = (int)getbits(s, 5) + 1, ncode = (int)getbits(s, 4) + 4;
            if (nlen > 286 || ndist > 30) return Z_DATA_ERROR;
            int k;
            for (k = 0; k < ncode; k++) {
                if (!need(s, 3)) return Z_BUF_ERROR;
                lens[cl_order[k]] = (uint16_t)getbits(s, 3);
            }
            for (; k < 19; k++) lens[cl_order[k]] = 0;
            if (build(&clh, lens, 19, 1)) return Z_DATA_ERROR;
            int have = 0;
            while (have < nlen + ndist) {
                int sym;
                if (clh.max == 0) { /* zlib decodes value 0 from its 1-bit invalid marker */
                    if (!need(s, 1)) return Z_BUF_ERROR;
                    getbits(s, 1);
                    sym = 0;
                } else {
                    sym = decode(s, &clh);
                    if (sym == -2) return Z_BUF_ERROR;
                    if (sym < 0) return Z_DATA_ERROR;
                }
                if (sym < 16) {
                    lens[have++] = (uint16_t)sym;
                } else {
                    unsigned len = 0, copy;
                    if (sym == 16) {
                        if (!need(s, 2)) return Z_BUF_ERROR;
                        if (have == 0) return Z_DATA_ERROR;
                        len = lens[have - 1];
                        copy = 3 + getbits(s, 2);
                    } else if (sym == 17) {
                        if (!need(s, 3)) return Z_BUF_ERROR;
                        copy = 3 + getbits(s, 3);
                    } else {
                        if (!need(s, 7)) return Z_BUF_ERROR;
                        copy = 11 + getbits(s, 7);
                    }
                    if (have + (int)copy > nlen + ndist) return Z_DATA_ERROR;
                    while (copy--) lens[have++] = (uint16_t)len;
                }
            }
            if (lens[256] == 0) return Z_DATA_ERROR;
            if (build(&lh, lens, nlen, 0)) return Z_DATA_ERROR;
            if (build(&dh, lens + nlen, ndist, 0)) return Z_DATA_ERROR;
            int rc = codes(s, &lh, &dh);
            if (rc) return rc;
        } else {
            return Z_DATA_ERROR; /* invalid block type */
        }
    } while (!last);
    /* ---- trailer ---- */
    s->bitpos = (s->bitpos + 7) & ~(uint64_t)7;
    p = (size_t)(s->bitpos >> 3);
    if (in_len < p + 4) return Z_BUF_ERROR;
    uint32_t crc = in[p] | ((uint32_t)in[p + 1] << 8) | ((uint32_t)in[p + 2] << 16) | ((uint32_t)in[p + 3] << 24);
    if (s->out_n > s->out_cap) { /* decoded past the buffer: report the size, no verdict yet */
        *out_len = s->out_n;
        return ORACLE_E_CAPACITY;
    }
    if (crc != oracle_crc32(0, out, s->out_n)) return Z_DATA_ERROR;
    p += 4;
    if (in_len < p + 4) return Z_BUF_ERROR;
    uint32_t isz = in[p] | ((uint32_t)in[p + 1] << 8) | ((uint32_t)in[p + 2] << 16) | ((uint32_t)in[p + 3] << 24);
    if (isz != (uint32_t)s->out_n) return Z_DATA_ERROR;
    *out_len = s->out_n;
    return 0;
}
