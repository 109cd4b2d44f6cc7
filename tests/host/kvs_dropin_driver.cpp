// kvs_dropin_driver.cpp -- the reference's own KeyValueStore over the drop-in codec.
//
// Built by `make -C oracle kvs` from the UNMODIFIED reference sources where they lie
// (/root/reference/src/kvs/kvs.cpp, hash/hash.cpp, hash/MurmurHash3.cpp, primegen/primegen.cpp,
// compiled against the reference's own headers) and linked with libgzip_dropin.so in place of
// src/compressor/gzip_compressor.cpp: the link-time substitution of INTEGRATION.md §2.  Nothing of
// the reference is copied; the binary lands in oracle/_ref/ and travels to the GPU box prebuilt.
//
// Checks:
//   1. KeyValueStoreTest.LargeJSONFiles (kvs_test.cpp:36-65): set every tests/data JSON under its
//      stem, get it back equal;
//   2. the compression gate (kvs.cpp:148,182: strlen + 1 >= 30) at 28/29 characters, overwrite and
//      del (the old value's buffer is released by MemoryPool::deallocate's delete[], kvs.hpp:87-98);
//   3. N JSON-slice values of 29..5000 B under keys "key"+i: set all, get all, compare;
//   4. with a device: GzipCompressor::Compress of each JSON file equals the reference's bytes
//      (<gz_dir>/<name>.gz), i.e. the store above ran on the bit-exact GPU codec.
// Without a device the drop-in returns PMC_E_NO_DEVICE and kvs.cpp:188-192 stores values raw:
// the store must still round-trip everything.
//
// usage: kvs_dropin_driver <data_dir> <gz_dir|-> <n_synthetic>
#include <dirent.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "kvs.hpp"  // the reference's header (-I /root/reference/src/kvs)

extern "C" void *pmc_default_ctx(void);  // include/pmc_codec.h (reports whether a device is in use)

static std::string slurp(const std::string &p) {
    std::ifstream f(p, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

static uint64_t splitmix64(uint64_t x) {  // SURVEY.md §8d generator (oracle/util.c)
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

#define CHECK(c, ...)                                 \
    do {                                              \
        if (!(c)) {                                   \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);             \
            fprintf(stderr, "\n");                    \
            return 1;                                 \
        }                                             \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <data_dir> <gz_dir|-> <n_synthetic>\n", argv[0]);
        return 2;
    }
    const std::string data = argv[1], gz = argv[2];
    const long nsyn = atol(argv[3]);
    const bool device = pmc_default_ctx() != nullptr;
    std::vector<std::string> names;
    if (DIR *d = opendir(data.c_str())) {
        while (dirent *e = readdir(d)) {
            std::string n = e->d_name;
            if (n.size() > 5 && n.substr(n.size() - 5) == ".json") names.push_back(n);
        }
        closedir(d);
    }
    std::sort(names.begin(), names.end());
    CHECK(names.size() == 6, "expected the reference's 6 tests/data JSON files, found %zu", names.size());

    kvs::KeyValueStore store;
    // 1. LargeJSONFiles
    std::string corpus;
    for (auto &n : names) {
        const std::string content = slurp(data + "/" + n);
        corpus += content;
        const std::string key = n.substr(0, n.size() - 5);
        CHECK(store.set(key.c_str(), content.c_str()), "set %s", key.c_str());
    }
    for (auto &n : names) {
        const std::string content = slurp(data + "/" + n);
        const std::string key = n.substr(0, n.size() - 5);
        const char *v = store.get(key.c_str());
        CHECK(v != nullptr, "get %s returned nullptr", key.c_str());
        CHECK(strcmp(v, content.c_str()) == 0, "get %s differs", key.c_str());
    }
    // 2. gate, overwrite, del
    const std::string v28(28, 'a'), v29(29, 'b');
    CHECK(store.set("k28", v28.c_str()) && store.set("k29", v29.c_str()), "set k28/k29");
    CHECK(strcmp(store.get("k28"), v28.c_str()) == 0, "k28");
    CHECK(strcmp(store.get("k29"), v29.c_str()) == 0, "k29");
    CHECK(store.set("k29", corpus.substr(100, 3000).c_str()), "overwrite k29");
    CHECK(strcmp(store.get("k29"), corpus.substr(100, 3000).c_str()) == 0, "k29 after overwrite");
    CHECK(store.del("k29"), "del k29");
    CHECK(store.get("k29") == nullptr, "k29 after del");
    // 3. synthetic values
    std::vector<std::string> vals(nsyn);
    for (long i = 0; i < nsyn; i++) {
        const uint64_t r = splitmix64(0x5EEDull ^ (uint64_t)i);
        const size_t len = 29 + r % 4972;
        const size_t off = splitmix64(r) % (corpus.size() - len + 1);
        vals[i] = corpus.substr(off, len);
        const std::string key = "key" + std::to_string(i);
        CHECK(store.set(key.c_str(), vals[i].c_str()), "set %s", key.c_str());
    }
    for (long i = 0; i < nsyn; i++) {
        const std::string key = "key" + std::to_string(i);
        const char *v = store.get(key.c_str());
        CHECK(v && strcmp(v, vals[i].c_str()) == 0, "get %s", key.c_str());
    }
    // 4. the codec under the store is the bit-exact one
    int exact = 0;
    if (device && gz != "-") {
        for (auto &n : names) {
            const std::string content = slurp(data + "/" + n), want = slurp(gz + "/" + n + ".gz");
            CompressResult c = GzipCompressor::Compress(content.c_str());
            CHECK(c.operationResult == 0, "Compress %s rc %d", n.c_str(), c.operationResult);
            CHECK(c.size == want.size() && memcmp(c.data, want.data(), c.size) == 0, "%s bytes differ", n.c_str());
            delete[] c.data;
            exact++;
        }
    }
    printf("OK device=%d json=%zu synthetic=%ld entries=%llu bitexact_files=%d\n", device ? 1 : 0, names.size(),
           nsyn, (unsigned long long)store.getNumEntries(), exact);
    return 0;
}
