// batch_codec_test.cpp -- pmc_batch::CompressForSet / DecompressForGet (the codec half of a
// batched server path) against the reference's per-value kvs decisions
// (/root/reference/src/kvs/kvs.cpp:148,182-196,224,233-234) and the reference's bytes.
// usage: batch_codec_test <tests/golden/data dir> <golden gz dir> [<decompress vector dir>]
#include <cstdio>
#include <cstring>
#include <dirent.h>
#include <string>
#include <vector>

#include "batch_codec.hpp"
#include "gzip_compressor.hpp"

static int failures = 0;
#define EXPECT(c)                                                            \
    do {                                                                     \
        if (!(c)) {                                                          \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);     \
            failures++;                                                      \
        }                                                                    \
    } while (0)

static std::string slurp(const std::string &p) {
    FILE *f = fopen(p.c_str(), "rb");
    if (!f) return {};
    std::string s;
    char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    fclose(f);
    return s;
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    std::vector<std::string> names;
    if (DIR *d = opendir(argv[1])) {
        while (dirent *e = readdir(d))
            if (strstr(e->d_name, ".json")) names.push_back(e->d_name);
        closedir(d);
    }
    EXPECT(!names.empty());
    // one SET batch: the reference's JSON files, the 28/29-character threshold, short values,
    // a null value, and slices of every length 1..300 of the first file
    std::vector<std::string> store;
    std::vector<std::string> gz;  // expected member for the data files ("" = none known)
    for (auto &n : names) {
        store.push_back(slurp(std::string(argv[1]) + "/" + n));
        gz.push_back(slurp(std::string(argv[2]) + "/" + n + ".gz"));
    }
    const size_t nfiles = store.size();
    store.push_back(std::string(28, 'a'));  // strlen 28: vSize 29 < 30 -> stored raw
    store.push_back(std::string(29, 'b'));  // strlen 29: vSize 30 -> compressed (expands, still stored)
    store.push_back("x");
    for (size_t l = 1; l <= 300; l++) store.push_back(store[0].substr(l * 7 % 1000, l));
    std::vector<const char *> vals;
    for (auto &s : store) vals.push_back(s.c_str());
    vals.insert(vals.begin() + nfiles + 2, nullptr);
    auto res = pmc_batch::CompressForSet(vals);
    EXPECT(res.size() == vals.size());
    std::vector<pmc_batch::Entry> ents;
    for (size_t i = 0; i < vals.size(); i++) {
        const auto &r = res[i];
        if (!vals[i]) {
            EXPECT(r.data == nullptr && r.rc == INVALID_INPUT);
            ents.push_back({nullptr, 0, false});
            continue;
        }
        const size_t len = strlen(vals[i]);
        const bool want_c = len + 1 >= pmc_batch::kMinCompressSize;
        EXPECT(r.compressed == want_c && r.rc == 0);
        if (want_c) {
            // the same bytes as the single-value drop-in (and, for the data files, the reference's)
            auto one = GzipCompressor::Compress(vals[i]);
            EXPECT(one.operationResult == 0 && one.size == r.size && memcmp(one.data, r.data, r.size) == 0);
            delete[] one.data;
            if (i < nfiles && !gz[i].empty()) EXPECT(gz[i].size() == r.size && memcmp(gz[i].data(), r.data, r.size) == 0);
        } else {
            EXPECT(r.size == len + 1 && memcmp(r.data, vals[i], len + 1) == 0);
        }
        ents.push_back({r.data, r.size, r.compressed});
    }
    // GET batch over what was stored, plus a corrupt member and a compressed entry of size 0
    std::string bad(res[0].data, res[0].size);
    bad[bad.size() - 6] ^= 0x5a;  // CRC flip -> Z_DATA_ERROR -> nullptr
    ents.push_back({bad.data(), bad.size(), true});
    ents.push_back({bad.data(), 0, true});
    std::vector<bool> owned;
    auto got = pmc_batch::DecompressForGet(ents, &owned);
    EXPECT(got.size() == ents.size());
    for (size_t i = 0; i < vals.size(); i++) {
        if (!vals[i]) continue;
        EXPECT(got[i] != nullptr && strcmp(got[i], vals[i]) == 0);
        EXPECT(owned[i] == res[i].compressed);
        if (!res[i].compressed) EXPECT(got[i] == res[i].data);  // raw entries hand out the stored pointer
    }
    EXPECT(got[vals.size()] == nullptr && !owned[vals.size()]);
    EXPECT(got[vals.size() + 1] == nullptr && !owned[vals.size() + 1]);
    for (size_t i = 0; i < got.size(); i++)
        if (owned[i]) delete[] got[i];
    for (auto &r : res) delete[] r.data;
    // GET batch of tests/golden's decompress vectors (argv[3], as dropin_test): the reference's bytes
    // (nullptr for its error verdicts), members followed by ignored bytes included
    if (argc >= 4) {
        std::string vdir = argv[3];
        FILE *ix = fopen((vdir + "/dec_index.txt").c_str(), "r");
        int k = 0, want_rc = 0;
        std::vector<std::string> ins, wants;
        std::vector<int> rcs;
        while (ix && fscanf(ix, "%d %d", &k, &want_rc) == 2) {
            if (want_rc == -5) continue;  // truncated: the drop-in's documented -5, nullptr here too
            ins.push_back(slurp(vdir + "/dec_" + std::to_string(k) + ".gz"));
            wants.push_back(want_rc == 0 ? slurp(vdir + "/dec_" + std::to_string(k) + ".out") : "");
            rcs.push_back(want_rc);
        }
        if (ix) fclose(ix);
        EXPECT(!ins.empty());
        std::vector<pmc_batch::Entry> dents;
        for (auto &x : ins) dents.push_back({x.data(), x.size(), true});
        std::vector<bool> down;
        auto dgot = pmc_batch::DecompressForGet(dents, &down);
        for (size_t i = 0; i < ins.size(); i++) {
            if (rcs[i] == 0) {
                EXPECT(dgot[i] && strlen(dgot[i]) == wants[i].size() && memcmp(dgot[i], wants[i].data(), wants[i].size()) == 0);
            } else {
                EXPECT(dgot[i] == nullptr);
            }
            if (down[i]) delete[] dgot[i];
        }
    }
    // compression disabled: everything stored raw
    auto raw = pmc_batch::CompressForSet({vals[0], vals[1]}, false);
    EXPECT(!raw[0].compressed && raw[0].size == strlen(vals[0]) + 1);
    for (auto &r : raw) delete[] r.data;
    printf("%s: %zu values, %d failures\n", failures ? "FAILED" : "ok", vals.size(), failures);
    return failures ? 1 : 0;
}
