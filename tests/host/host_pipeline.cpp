// host_pipeline.cpp -- CPU twin of the gfx950 deflate kernel's back end (test only).
//
// Compiles poor-man-s-cache_amd/csrc/pmc_trees.hpp (the Huffman construction the kernel
// runs on lane 0, and token_bits which the kernel's lanes use to emit symbols) with g++
// and drives it the way pmc_deflate.hip does: serial lazy parse over a hash-sorted chain,
// 16383-symbol blocks, stored/fixed/dynamic choice, gzip framing.  tests/test_host_pipeline.py
// diffs the result against the golden vectors, so the device-side Huffman/emit code is
// pinned on a CPU before any GPU run.
//
// usage: host_pipeline <in> <out>   (writes the gzip member of <in> to <out>)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../poor-man-s-cache_amd/csrc/pmc_trees.hpp"

using namespace pmc;

static const Tables T = make_tables();

struct Bitbuf {
    std::vector<uint8_t> &out;
    uint64_t pos;
    void put(unsigned v, int n) {
        for (int k = 0; k < n; k++) {
            uint64_t p = pos + k;
            if ((p >> 3) >= out.size()) out.resize((p >> 3) + 1, 0);
            if ((v >> k) & 1) out[p >> 3] |= (uint8_t)(1u << (p & 7));
        }
        pos += n;
    }
    void put64(uint64_t v, int n) {
        for (int k = 0; k < n; k += 16) put((unsigned)(v >> k) & 0xffff, n - k < 16 ? n - k : 16);
    }
};

static uint32_t crc32(const uint8_t *p, size_t n) {
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) {
        c ^= p[i];
        for (int k = 0; k < 8; k++) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    }
    return ~c;
}

int main(int argc, char **argv) {
    if (argc != 3) return 2;
    FILE *f = fopen(argv[1], "rb");
    std::vector<uint8_t> in;
    int ch;
    while ((ch = fgetc(f)) != EOF) in.push_back((uint8_t)ch);
    fclose(f);
    const uint64_t len = in.size();
    std::vector<uint8_t> b(in);
    b.resize(len + 64, 0);
    // hash + stable sort (the kernel: 3 x 5-bit LSD radix passes)
    const uint64_t npos = len >= 3 ? len - 2 : 0;
    std::vector<uint64_t> S(npos), rank(npos);
    {
        std::vector<uint32_t> cnt(32769, 0);
        std::vector<uint32_t> h(npos);
        for (uint64_t p = 0; p < npos; p++) {
            h[p] = ((uint32_t)b[p] << 10 ^ (uint32_t)b[p + 1] << 5 ^ b[p + 2]) & 0x7fff;
            cnt[h[p] + 1]++;
        }
        for (int k = 0; k < 32768; k++) cnt[k + 1] += cnt[k];
        for (uint64_t p = 0; p < npos; p++) {
            uint32_t r = cnt[h[p]]++;
            S[r] = (uint64_t)h[p] << 32 | p;
            rank[p] = r;
        }
    }
    auto search = [&](uint64_t i, uint32_t b0, uint64_t B, uint64_t *qo) -> uint32_t {
        uint32_t C = b0 >= 32 ? 1024 : 4096;
        uint32_t nice = (uint32_t)((len - i) < 258 ? (len - i) : 258);
        int64_t r = (int64_t)rank[i];
        uint64_t hi = S[r] >> 32;
        uint32_t ex = 0, best = 0;
        for (int64_t k = r - 1; k >= 0; k--) {
            if ((S[k] >> 32) != hi) break;
            uint64_t q = S[k] & 0xffffffffull, d = i - q;
            if (q <= B || (ex == 0 ? d > 32506 : d >= 32506) || ex >= C) break;
            ex++;
            uint32_t l = 0;
            while (l < nice && b[i + l] == b[q + l]) l++;
            if (l > best) {
                best = l;
                *qo = q;
                if (l >= nice) break;
            }
        }
        return best > b0 ? best : 0;
    };
    std::vector<uint8_t> out(10, 0);
    const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 2, 3};
    memcpy(out.data(), hdr, 10);
    Bitbuf bb{out, 80};
    Trees *tr = (Trees *)calloc(1, sizeof(Trees));
    init_block(*tr);
    std::vector<uint32_t> tok;
    uint64_t block_start = 0, B = 0, wend = 0, i = 0;
    auto flush = [&](uint64_t end, bool last) {
        BlockPlan p = plan_block(*tr, T);
        uint64_t stored_len = end - block_start;
        if (stored_len + 4 <= p.opt_lenb && block_start >= B) {
            bb.put((0u << 1) + last, 3);
            bb.pos = (bb.pos + 7) & ~7ull;
            bb.put((unsigned)stored_len & 0xffff, 16);
            bb.put((~(unsigned)stored_len) & 0xffff, 16);
            for (uint64_t k = 0; k < stored_len; k++) bb.put(b[block_start + k], 8);
        } else {
            bool fixed = p.static_lenb == p.opt_lenb;
            const CtData *lt = fixed ? T.static_ltree : tr->ltree;
            const CtData *dt = fixed ? T.static_dtree : tr->dtree;
            bb.put(((fixed ? 1u : 2u) << 1) + last, 3);
            if (!fixed) send_all_trees(*tr, T, bb, p);
            for (uint32_t t : tok) {
                int nb = 0;
                uint64_t v = token_bits(T, lt, dt, t, nb);
                bb.put64(v, nb);
            }
            bb.put(lt[kEndBlock].fc, lt[kEndBlock].dl);
            if (last) bb.pos = (bb.pos + 7) & ~7ull;
        }
        init_block(*tr);
        tok.clear();
        block_start = end;
    };
    auto emit = [&](uint32_t t) {
        tok.push_back(t);
        uint32_t dist = t >> 16, lc = t & 0xff;
        if (!dist) tr->ltree[lc].fc++;
        else {
            tr->ltree[T.length_code[lc] + kLiterals + 1].fc++;
            tr->dtree[d_code(T, dist - 1)].fc++;
        }
    };
    uint32_t match_length = 2, prev_length;
    uint64_t match_start = 0, prev_match;
    bool avail = false;
    for (;;) {
        if (wend - i < 262) {
            do {
                if (i - B >= 32768 + 32506) B += 32768;
                if (wend == len) break;
                wend = len < B + 65536 ? len : B + 65536;
            } while (wend - i < 262 && wend < len);
            if (wend == i) break;
        }
        prev_length = match_length;
        prev_match = match_start;
        match_length = 2;
        if (i + 3 <= len && prev_length < 258) {
            uint64_t q = 0;
            uint32_t m = search(i, prev_length, B, &q);
            if (m) {
                match_length = m;
                match_start = q;
                if (m == 3 && i - q > 4096) match_length = 2;
            }
        }
        if (prev_length >= 3 && match_length <= prev_length) {
            emit((uint32_t)(i - 1 - prev_match) << 16 | (prev_length - 3));
            i += prev_length - 1;
            avail = false;
            match_length = 2;
            if (tok.size() == 16383) flush(i, false);
        } else if (avail) {
            emit(b[i - 1]);
            if (tok.size() == 16383) flush(i, false);
            i++;
        } else {
            avail = true;
            i++;
        }
    }
    if (avail) emit(b[i - 1]);
    flush(i, true);
    out.resize(bb.pos >> 3);
    uint32_t c = crc32(in.data(), len);
    for (int k = 0; k < 4; k++) out.push_back((uint8_t)(c >> (8 * k)));
    for (int k = 0; k < 4; k++) out.push_back((uint8_t)(len >> (8 * k)));
    FILE *g = fopen(argv[2], "wb");
    fwrite(out.data(), 1, out.size(), g);
    fclose(g);
    free(tr);
    return 0;
}
