"""Reference vectors for values above the 82,002 B corpus (run in the build container only).

Source of truth: the reference's own GzipCompressor::Compress
(/root/reference/src/compressor/gzip_compressor.cpp:3-50), compiled unmodified into
oracle/_ref/libref_gzip.so by `make -C oracle ref` (system zlib 1.2.11).  Values holding a NUL byte
cannot pass the reference's strlen interface (gzip_compressor.cpp:6); those come from Python's zlib
bound to the same libz 1.2.11 with the reference's parameters (compressobj(9, DEFLATED, 31, 8, 0))
and are tagged "libz".

The values are the sets of tests/large_values.py (100 KB .. 4 MiB: tiled JSON, alnum, small
alphabets, random bytes, period-1/2 runs, segment-boundary sizes).  Members of several MiB would
bloat the repository, so per value the fixture keeps the SHA-256 and length of the reference's member
(a byte-exact check: the tests hash the device's member and compare), keyed by the SHA-256 of the
value.

Output (data only): tests/golden/large_golden.json
Usage: python tests/golden/make_large_golden.py
"""
import hashlib
import json
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import pyoracle as O  # noqa: E402
import large_values  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def libz(b):
    c = zlib.compressobj(9, zlib.DEFLATED, 31, 8, 0)
    return c.compress(b) + c.flush()


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    O.build(ref=True)
    assert O.ref_available(), "oracle/_ref/libref_gzip.so missing (needs /root/reference)"
    d = os.path.join(HERE, "data")
    corpus = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))
    vectors, sets = {}, {}
    for name, vals in large_values.all_sets(corpus).items():
        keys = []
        for v in vals:
            k = sha(v)
            keys.append(k)
            if k in vectors:
                continue
            if b"\0" in v:
                gz, src = libz(v), "libz"
            else:
                rc, gz = O.ref_compress(v)
                assert rc == 0, (name, len(v), rc)
                assert gz == libz(v)
                src = "reference"
            vectors[k] = {"len": len(v), "gz_sha256": sha(gz), "gz_len": len(gz), "source": src}
        sets[name] = keys
        print(f"{name}: {len(vals)} values, {sum(map(len, vals))} B", flush=True)
    doc = {
        "generator": "tests/golden/make_large_golden.py",
        "reference": "/root/reference/src/compressor/gzip_compressor.cpp (built by oracle/Makefile ref)",
        "zlib_version": O.ref().ref_zlib_version().decode(),
        "values": "tests/large_values.py (deterministic builders over tests/golden/data)",
        "record": "vectors[sha256(value)] = SHA-256 and length of the reference's gzip member of the value",
        "sets": sets,
        "vectors": vectors,
    }
    with open(os.path.join(HERE, "large_golden.json"), "w") as f:
        json.dump(doc, f, indent=0)
    print("vectors", len(vectors), "reference", sum(v["source"] == "reference" for v in vectors.values()))


if __name__ == "__main__":
    main()
