"""Route goldens: the reference's own key hash for the keys BASELINE configs[3] routes.

hashFunc(key) = MurmurHash3_x64_128(key, strlen(key), 0)[0] (/root/reference/src/hash/hash.cpp:4-9,
MurmurHash3.cpp:255-332), compiled unmodified into oracle/_ref/libref_hash.so by `make -C oracle hash`.
The server routes a key to shard hash % numShards (server.cpp:113,121,132); the build sends shard s to
GPU s % nGPU.  Keys are "key" + decimal(i) for i in 0..4999, 9,999,000..10,000,999
and 79,999,000..79,999,999 (the end of configs[3]'s 80M key space).

Also keys of every length 0..70 (16 per length: NUL-free random bytes 1..255 -- hashFunc takes a C
string -- and printable ones), covering the 16-byte block loop and every tail length (MurmurHash3.cpp
:270-318) that the "key"+i keys (4..11 bytes) never reach.

Output (data only): tests/golden/route_golden.npz
  index: uint64, hash: uint64                    -- "key"+index
  key_blob: uint8, key_off: uint64 (n+1), key_hash: uint64  -- the variable-length keys
Usage: python tests/golden/make_route_golden.py
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "hash"])
    R = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_hash.so"))
    R.ref_hash_func.restype = ctypes.c_uint64
    R.ref_hash_func.argtypes = [ctypes.c_char_p]
    idx = np.concatenate([np.arange(0, 5000), np.arange(9_999_000, 10_001_000),
                          np.arange(79_999_000, 80_000_000)]).astype(np.uint64)
    h = np.array([R.ref_hash_func(b"key%d" % int(i)) for i in idx], dtype=np.uint64)
    rng = np.random.default_rng(70)
    keys = []
    for ln in range(0, 71):
        for k in range(16):
            if k < 8:
                keys.append(bytes(rng.integers(1, 256, ln, dtype=np.uint8)))
            else:
                keys.append(bytes(rng.integers(32, 127, ln, dtype=np.uint8)))
    key_off = np.cumsum([0] + [len(k) for k in keys]).astype(np.uint64)
    key_hash = np.array([R.ref_hash_func(k) for k in keys], dtype=np.uint64)
    np.savez_compressed(os.path.join(HERE, "route_golden.npz"), index=idx, hash=h,
                        key_blob=np.frombuffer(b"".join(keys), dtype=np.uint8), key_off=key_off, key_hash=key_hash)
    print("keys", len(idx), "shards of key0..3 (%128):", [int(x) % 128 for x in h[:4]])


if __name__ == "__main__":
    main()
