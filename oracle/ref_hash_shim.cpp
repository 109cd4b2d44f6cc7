// ref_hash_shim.cpp -- TEST INFRASTRUCTURE ONLY (oracle/_ref).
//
// C entry point around the reference's own key hash, compiled straight from
// /root/reference/src/hash/hash.cpp + MurmurHash3.cpp by oracle/Makefile (target _ref hash):
// hashFunc(key) = MurmurHash3_x64_128(key, strlen(key), 0)[0] (hash.cpp:4-9), the value the
// server routes by (server.cpp:113,121,132: hash % numShards).  Used by
// tests/golden/make_route_golden.py to pin the device router (pmc_route_keys) and the oracle's
// restatement (oracle/util.c) to the reference.
#include <cstdint>

#include "hash.hpp"

extern "C" uint64_t ref_hash_func(const char *key) { return (uint64_t)hashFunc(key); }
