"""Generate the committed golden vectors (run in the build container only).

Source of truth: the reference's own GzipCompressor::Compress / ::Decompress
(/root/reference/src/compressor/gzip_compressor.cpp:3-111), compiled unmodified from
/root/reference by `make -C oracle ref` into oracle/_ref/libref_gzip.so (system zlib
1.2.11).  Binary (NUL-containing) values cannot pass through the reference's strlen
interface, so those few vectors come from Python's zlib module bound to the same
libz 1.2.11 with the reference's parameters (compressobj(9, DEFLATED, 31, 8, 0)) and are
tagged "libz" instead of "reference".

Outputs (data only -- no reference source is copied):
  tests/golden/data/*.json        the reference's own test fixtures (tests/data)
  tests/golden/golden.npz         vectors: raw bytes, gzip bytes, offsets
  tests/golden/golden_index.json  sets, digests and expected decompress codes

Usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import shutil
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle as O  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DATA = "/root/reference/tests/data"


def libz(b):
    c = zlib.compressobj(9, zlib.DEFLATED, 31, 8, 0)
    return c.compress(b) + c.flush()


def main():
    O.build(ref=True)
    assert O.ref_available(), "oracle/_ref/libref_gzip.so missing (needs /root/reference)"
    os.makedirs(os.path.join(HERE, "data"), exist_ok=True)
    names = sorted(f for f in os.listdir(REF_DATA) if f.endswith(".json"))
    for f in names:
        shutil.copyfile(os.path.join(REF_DATA, f), os.path.join(HERE, "data", f))
    corpus = b"".join(open(os.path.join(HERE, "data", f), "rb").read() for f in names)
    assert len(corpus) == 82002

    raws, gzs, tags = [], [], []

    def add(raw, tag):
        if b"\0" in raw or len(raw) == 0:
            gz = libz(raw)
            src = "libz"
        else:
            rc, gz = O.ref_compress(raw)
            assert rc == 0
            assert gz == libz(raw)
            src = "reference"
        raws.append(raw)
        gzs.append(gz)
        tags.append({"tag": tag, "source": src})

    # 1. the reference's own test inputs (gzip_compressor_test.cpp:7,52-54,75; kvs_test.cpp:36-65)
    for f in names:
        add(open(os.path.join(HERE, "data", f), "rb").read(), "tests/data/" + f)
    add(b"Hello, Gzip!", "gzip_compressor_test.cpp:7")
    add(b"This is a long test string. It should be compressed and decompressed properly. "
        b"We are testing to see if gzip can handle long input.", "gzip_compressor_test.cpp:52")
    add(b"A" * 50, "gzip_compressor_test.cpp:75")
    # 2. edge cases: compression gate thresholds (kvs.hpp:26), lazy/tie cases, blocks, window
    add(b"x" * 29, "29 bytes (strlen+1 == 30, first compressed size)")
    add(b"y" * 30, "30 bytes")
    add(b"abcdefgh-abcdefgh", "position 0 is never a match source")
    add(b"XabcdQabcdRabcdS", "nearest candidate wins ties")
    add(b"XabcdeQabcdRabcdeS", "longer farther candidate beats nearer")
    for ln in (1, 2, 3, 4, 5):
        add(b"q" * ln, "tiny %d" % ln)
    add(corpus, "whole corpus 82002 B (window slide, multi-block)")
    add(corpus[:40000], "40000 B (> MAX_DIST)")
    add((corpus[:3000] * 30)[:65300], "65300 B (slide at end of input)")
    add(b"ab" * 20000, "40000 B of 2 symbols (>16383 symbols -> multi-block)")
    rng = np.random.default_rng(12345)
    add(bytes(rng.integers(1, 256, 3000, dtype=np.uint8)), "3000 random non-zero bytes (stored)")
    add(bytes(rng.integers(0, 256, 5000, dtype=np.uint8)), "5000 random bytes incl. NUL (stored)")
    add(bytes(rng.choice([0, 0, 1, 2, 255], 4000).astype(np.uint8)), "binary skewed incl. NUL")
    geo = np.minimum(rng.geometric(0.08, 20000), 255).astype(np.uint8)
    add(bytes(geo), "geometric symbols (long codes, length-limit overflow)")
    # 3. per-size-class sets: JSON slices (kind 0, seed 0x5EED), alnum (kind 1, seed 0xA1B2)
    sets = []
    for vlen, n in ((29, 64), (30, 64), (64, 64), (256, 64), (1024, 64), (4096, 32), (16384, 8), (65536, 4)):
        for kind, seed in ((0, 0x5EED), (1, 0xA1B2)):
            vals = O.gen_values(corpus, seed, kind, 0, n, vlen)
            first = len(raws)
            for k in range(n):
                add(vals[k].tobytes(), "gen kind=%d vlen=%d i=%d" % (kind, vlen, k))
            sets.append({"kind": kind, "seed": seed, "vlen": vlen, "n": n, "first_vector": first})

    raw_off = np.cumsum([0] + [len(r) for r in raws]).astype(np.uint64)
    gz_off = np.cumsum([0] + [len(g) for g in gzs]).astype(np.uint64)
    np.savez_compressed(os.path.join(HERE, "golden.npz"),
                        raw=np.frombuffer(b"".join(raws), dtype=np.uint8), raw_off=raw_off,
                        gz=np.frombuffer(b"".join(gzs), dtype=np.uint8), gz_off=gz_off)

    # 4. large seeded sets: digest of concatenated gzip members + per-value sizes
    digests = []
    for vlen, n, kind, seed in ((256, 4096, 0, 0x5EED), (1024, 4096, 0, 0x5EED), (4096, 1024, 0, 0x5EED),
                                (1024, 2048, 1, 0xA1B2)):
        vals = O.gen_values(corpus, seed, kind, 0, n, vlen)
        h = hashlib.sha256()
        sizes = []
        for k in range(n):
            rc, gz = O.ref_compress(vals[k].tobytes())
            assert rc == 0
            h.update(gz)
            sizes.append(len(gz))
        digests.append({"kind": kind, "seed": seed, "vlen": vlen, "n": n, "sha256": h.hexdigest(),
                        "gz_bytes": int(sum(sizes)), "sizes_sha256": hashlib.sha256(
                            np.asarray(sizes, dtype=np.uint32).tobytes()).hexdigest()})

    # 5. decompress error vectors with the reference's own verdicts (truncated inputs hang
    #    the reference -- SURVEY.md §5 -- so their expectation is the documented -5)
    z = O.ref_compress(b"Hello, Gzip! Hello, Gzip! Hello, Gzip! 1234567890")[1]
    zj = O.ref_compress(corpus[1000:2024])[1]
    errs = []

    def err(name, data, truncated=False):
        out = None
        if truncated:
            rc = -5
        else:
            rc, out = O.ref_decompress(data)
        e = {"name": name, "hex": data.hex(), "expect_rc": rc, "truncated": truncated}
        if rc == 0:
            # the reference returns a NUL-terminated buffer and no size (gzip_compressor.cpp:105-110);
            # every member here decodes to NUL-free text, so its bytes are the C string
            e["expect_hex"] = out.hex()
        errs.append(e)

    err("not a gzip string (gzip_compressor_test.cpp:90)", b"Not a gzip string")
    err("bad magic", b"\x1f\x8c" + z[2:])
    err("bad method", z[:2] + b"\x07" + z[3:])
    err("reserved flag", z[:3] + b"\x20" + z[4:])
    err("crc flip", z[:-8] + bytes([z[-8] ^ 1]) + z[-7:])
    err("isize flip", z[:-4] + bytes([z[-4] ^ 1]) + z[-3:])
    err("trailing garbage", z + b"trailing garbage")
    err("concatenated members", z + zj)
    err("zlib-wrapped stream", zlib.compress(b"Hello, Gzip!", 9))
    err("invalid block type", z[:10] + bytes([z[10] | 0x06]) + z[11:])
    for k in (1, 4, 8, 9, 12, len(zj) // 2, len(zj) - 5, len(zj) - 1):
        err("truncated to %d" % k, zj[:k], truncated=True)
    # bytes after the first member (the reference stops at Z_STREAM_END, gzip_compressor.cpp:96):
    # the input's last 4 bytes no longer hold the member's ISIZE, so any capacity taken from them
    # is wrong -- smaller, zero, misaligned or larger than the output
    z50 = O.ref_compress(corpus[5000:5050])[1]
    zq = O.ref_compress(corpus[20000:20256])[1]
    err("1 KiB member + 50 B member", zj + z50)
    err("1 KiB member + 4 NUL bytes", zj + b"\0\0\0\0")
    for k in (1, 2, 3):
        err("1 KiB member + %d stray byte(s)" % k, zj + bytes(range(1, k + 1)))
    err("1 KiB member + bytes reading as a larger ISIZE", zj + (5000).to_bytes(4, "little"))
    err("1 KiB member + bytes reading as ISIZE 2^32-1", zj + b"\xff\xff\xff\xff")
    err("256 B member + 4 NUL bytes", zq + b"\0\0\0\0")
    err("short member + 4 NUL bytes", z + b"\0\0\0\0")
    err("1 KiB member + truncated member", zj + zj[:40])
    err("CRC-flipped 1 KiB member + 4 NUL bytes", zj[:-8] + bytes([zj[-8] ^ 1]) + zj[-7:] + b"\0\0\0\0")
    err("ISIZE-flipped 1 KiB member + 50 B member", zj[:-4] + bytes([zj[-4] ^ 1]) + zj[-3:] + z50)

    index = {
        "generator": "tests/golden/make_golden.py",
        "reference": "/root/reference/src/compressor/gzip_compressor.cpp (built by oracle/Makefile ref)",
        "zlib_version": O.ref().ref_zlib_version().decode(),
        "corpus": "tests/golden/data/*.json concatenated in sorted filename order (82002 B)",
        "vectors": tags,
        "sets": sets,
        "digests": digests,
        "decompress_errors": errs,
    }
    with open(os.path.join(HERE, "golden_index.json"), "w") as f:
        json.dump(index, f, indent=1)
    print("vectors", len(raws), "raw bytes", int(raw_off[-1]), "gz bytes", int(gz_off[-1]),
          "digests", len(digests), "error vectors", len(errs))


if __name__ == "__main__":
    main()
