/* util.c -- CPU ORACLE (test infrastructure only): CRC-32 (zlib crc32.c: reflected
 * polynomial 0xEDB88320, the gzip trailer checksum) and the seeded synthetic-value
 * generator of SURVEY.md §8d shared with the GPU generator kernel. */
#include "pmc_oracle.h"

static uint32_t crc_table[256];
static int crc_ready;

static void crc_init(void) {
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_table[n] = c;
    }
    crc_ready = 1;
}

uint32_t oracle_crc32(uint32_t crc, const uint8_t *p, size_t n) {
    if (!crc_ready) crc_init();
    crc = ~crc;
    while (n--) crc = crc_table[(crc ^ *p++) & 0xff] ^ (crc >> 8);
    return ~crc;
}

uint64_t oracle_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* MurmurHash3_x64_128(key, len, seed)[0] -- restates the reference's hashFunc
 * (/root/reference/src/hash/hash.cpp:4-9, MurmurHash3.cpp:255-332) for shard routing. */
static uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}
uint64_t oracle_murmur3_x64_128_h1(const uint8_t *data, int len, uint32_t seed) {
    const int nblocks = len / 16;
    uint64_t h1 = seed, h2 = seed, k1, k2;
    const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
    for (int i = 0; i < nblocks; i++) {
        k1 = k2 = 0;
        for (int b = 0; b < 8; b++) k1 |= (uint64_t)data[16 * i + b] << (8 * b);
        for (int b = 0; b < 8; b++) k2 |= (uint64_t)data[16 * i + 8 + b] << (8 * b);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint8_t *tail = data + nblocks * 16;
    k1 = k2 = 0;
    int t = len & 15;
    for (int b = t - 1; b >= 8; b--) k2 ^= (uint64_t)tail[b] << (8 * (b - 8));
    if (t > 8) { k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; }
    for (int b = (t < 8 ? t : 8) - 1; b >= 0; b--) k1 ^= (uint64_t)tail[b] << (8 * b);
    if (t > 0) { k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1; }
    h1 ^= (uint64_t)len; h2 ^= (uint64_t)len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2;
    return h1;
}

static const char ALNUM[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";

static void gen_one(const uint8_t *corpus, size_t corpus_len, uint64_t seed, int kind, uint64_t i, uint32_t vlen,
                    uint8_t *dst) {
    if (kind == 0) {
        uint64_t off = oracle_splitmix64(seed ^ i) % (corpus_len - vlen + 1);
        for (uint32_t b = 0; b < vlen; b++) dst[b] = corpus[off + b];
    } else {
        /* 8-byte group g of value i: st = splitmix64(splitmix64(seed ^ i) + g) */
        uint64_t hi = oracle_splitmix64(seed ^ i), st = 0;
        for (uint32_t b = 0; b < vlen; b++) {
            if ((b & 7) == 0) st = oracle_splitmix64(hi + (b >> 3));
            dst[b] = (uint8_t)ALNUM[((st >> (8 * (b & 7))) & 0xff) % 62];
        }
    }
}

void oracle_gen_values(const uint8_t *corpus, size_t corpus_len, uint64_t seed, int kind,
                       uint64_t first, uint32_t n, uint32_t vlen, uint8_t *out) {
    for (uint32_t k = 0; k < n; k++) gen_one(corpus, corpus_len, seed, kind, first + k, vlen, out + (uint64_t)k * vlen);
}

/* the same values at arbitrary global indices (a rank's routed key subset) */
void oracle_gen_values_idx(const uint8_t *corpus, size_t corpus_len, uint64_t seed, int kind,
                           const uint64_t *index, uint32_t n, uint32_t vlen, uint8_t *out) {
    for (uint32_t k = 0; k < n; k++) gen_one(corpus, corpus_len, seed, kind, index[k], vlen, out + (uint64_t)k * vlen);
}

/* out[i] = hashFunc("key" + (first + i)) % num_shards % n_gpus: the server's shard routing
 * (/root/reference/src/server/server.cpp:113,121,132; hash.cpp:4-9), what pmc_route_keys computes */
void oracle_route_keys(uint64_t first, uint64_t n, uint32_t num_shards, uint32_t n_gpus, uint8_t *out) {
    char key[32];
    for (uint64_t i = 0; i < n; i++) {
        uint64_t v = first + i;
        char digits[24];
        int nd = 0;
        do {
            digits[nd++] = (char)('0' + v % 10);
            v /= 10;
        } while (v);
        key[0] = 'k';
        key[1] = 'e';
        key[2] = 'y';
        for (int d = 0; d < nd; d++) key[3 + d] = digits[nd - 1 - d];
        out[i] = (uint8_t)(oracle_murmur3_x64_128_h1((const uint8_t *)key, 3 + nd, 0) % num_shards % n_gpus);
    }
}
