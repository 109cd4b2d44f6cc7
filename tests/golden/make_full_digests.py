"""Full-size parity digests for the BASELINE workloads (run in the build container only).

The reference's own GzipCompressor::Compress (/root/reference/src/compressor/gzip_compressor.cpp:3-50,
compiled unmodified into oracle/_ref/libref_gzip.so by `make -C oracle ref`) compresses every value of
each workload; value i of size V is the SURVEY.md §8d generator's (oracle_gen_values, the same formula
as the device's pmc_gen_values).  Per member we keep (u32 length, u32 CRC-32 of the member bytes) and
hash those records with SHA-256 (pyoracle.member_records_digest), with the running digest snapshotted
at several prefix counts so shorter runs of the same workload can be checked too.

bench.py recomputes the same records on the device after its timed steps (pmc_crc32_batch over the
compressed members, lengths from the codec) and reports "bitexact"; tests/test_gpu_fullsize.py checks
the 200K prefixes through a multi-chunk compress.

Output (data only): tests/golden/full_digests.json
Usage: python tests/golden/make_full_digests.py [--threads 8]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle as O  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
# (values, value bytes, generator kind, seed): north star 10M x 1 KiB, configs[1] 10M x 256 B,
# the 4 KiB configs[2] value shape, and the alnum stress generator
SETS = [(10_000_000, 1024, 0, 0x5EED), (10_000_000, 256, 0, 0x5EED), (1_000_000, 4096, 0, 0x5EED),
        (1_000_000, 1024, 1, 0xA1B2)]
CHECKPOINTS = (4096, 200_000, 1_000_000, 2_000_000, 5_000_000, 10_000_000)
CHUNK = 250_000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    args = ap.parse_args()
    O.build(ref=True)
    assert O.ref_available(), "oracle/_ref/libref_gzip.so missing (needs /root/reference)"
    d = os.path.join(HERE, "data")
    corpus = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))
    out = []
    for n, vlen, kind, seed in SETS:
        t0 = time.time()
        h = hashlib.sha256()
        gz_bytes = 0
        marks = {}
        for first in range(0, n, CHUNK):
            m = min(CHUNK, n - first)
            vals = O.gen_values(corpus, seed, kind, first, m, vlen)
            lens, crcs = O.ref_member_records(vals, args.threads)
            # split the chunk at checkpoints that fall inside it
            cut = first
            for c in sorted(CHECKPOINTS):
                if first < c <= first + m:
                    a, b = cut - first, c - first
                    O.member_records_digest(lens[a:b], crcs[a:b], h)
                    gz_bytes += int(lens[a:b].astype(np.uint64).sum())
                    marks[str(c)] = {"sha256": h.copy().hexdigest(), "gz_bytes": gz_bytes}
                    cut = c
            a = cut - first
            O.member_records_digest(lens[a:], crcs[a:], h)
            gz_bytes += int(lens[a:].astype(np.uint64).sum())
        marks[str(n)] = {"sha256": h.hexdigest(), "gz_bytes": gz_bytes}
        out.append({"n": n, "vlen": vlen, "kind": kind, "seed": seed, "first": 0, "prefixes": marks})
        print(f"{n} x {vlen} kind {kind}: {gz_bytes} B compressed, {time.time() - t0:.1f} s", flush=True)
    doc = {
        "generator": "tests/golden/make_full_digests.py",
        "reference": "/root/reference/src/compressor/gzip_compressor.cpp (built by oracle/Makefile ref)",
        "zlib_version": O.ref().ref_zlib_version().decode(),
        "record": "per member, in value order: u32 LE compressed length, u32 LE CRC-32 (zlib crc32) of the "
                  "member bytes; sha256 over all records of the first `prefix` values",
        "values": "SURVEY.md §8d generator: kind 0 = corpus slice at splitmix64(seed ^ i) % (82002 - V + 1), "
                  "kind 1 = random [A-Za-z0-9]; value indices 0 .. n-1",
        "sets": out,
    }
    with open(os.path.join(HERE, "full_digests.json"), "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
