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
Usage: python tests/golden/make_full_digests.py [--threads 8] [--ranks | --large]
  --ranks: tests/golden/rank_digests.json, the per-rank digests of bench.py --gpus 2/4/8
  --large: add the large-value bench legs (100K x 30 KB, 40K x 64 KiB, 1000 x 1 MiB JSON slices; values
           longer than the 82 KB corpus are slices of it tiled, as bench.py makes them) to full_digests.json
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
# the large-value bench legs (bench.py --n N --vlen V): the reference's own fixtures' size (tests/data 5_*, 6_*,
# 29-30 KB), 64 KiB and 1 MiB
LARGE_SETS = [(100_000, 30_000, 0, 0x5EED), (40_000, 65_536, 0, 0x5EED), (1_000, 1 << 20, 0, 0x5EED)]
LARGE_CHECKPOINTS = (1_000, 4_096, 10_000)
CHUNK_BYTES = 1 << 30


def bench_corpus(corpus, vlen):  # = bench.py: values longer than the corpus are slices of it tiled
    return corpus * (vlen // len(corpus) + 2) if vlen > len(corpus) else corpus


def digest_set(corpus, n, vlen, kind, seed, checkpoints, threads):
    corpus = bench_corpus(corpus, vlen)
    chunk = max(1, min(CHUNK, CHUNK_BYTES // vlen))
    h = hashlib.sha256()
    gz_bytes = 0
    marks = {}
    for first in range(0, n, chunk):
        m = min(chunk, n - first)
        vals = O.gen_values(corpus, seed, kind, first, m, vlen)
        lens, crcs = O.ref_member_records(vals, threads)
        cut = first
        for c in sorted(checkpoints):  # split the chunk at checkpoints that fall inside it
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
    return {"n": n, "vlen": vlen, "kind": kind, "seed": seed, "first": 0, "prefixes": marks}


# multi-GPU weak scaling (bench.py --gpus N): rank r of N compresses the first RANK_N keys "key"+i whose
# hashFunc("key"+i) % 128 % N == r (server.cpp:113,121,132), among keys 0 .. route_span - 1
RANK_WORLDS = (2, 4, 8)
RANK_N = 10_000_000
RANK_CHECKPOINTS = (200_000, 1_000_000, 10_000_000)


def route_span(n, world):  # = bench.py route_span
    return int(n * world * 1.05) + 4096


def rank_digests(corpus, threads):
    """Per-rank digests of the north-star workload (10M x 1 KiB JSON slices per GPU) for N = 2, 4, 8."""
    out = []
    for world in RANK_WORLDS:
        route = O.route_keys(0, route_span(RANK_N, world), 128, world)
        for rank in range(world):
            t0 = time.time()
            idx = np.nonzero(route == rank)[0][:RANK_N].astype(np.uint64)
            assert len(idx) == RANK_N, (world, rank, len(idx))
            h = hashlib.sha256()
            gz_bytes = 0
            marks = {}
            for first in range(0, RANK_N, CHUNK):
                m = min(CHUNK, RANK_N - first)
                vals = O.gen_values_idx(corpus, 0x5EED, 0, idx[first:first + m], 1024)
                lens, crcs = O.ref_member_records(vals, threads)
                O.member_records_digest(lens, crcs, h)
                gz_bytes += int(lens.astype(np.uint64).sum())
                if first + m in RANK_CHECKPOINTS:
                    marks[str(first + m)] = {"sha256": h.copy().hexdigest(), "gz_bytes": gz_bytes}
            out.append({"world": world, "rank": rank, "n": RANK_N, "vlen": 1024, "kind": 0, "seed": 0x5EED,
                        "index_sha256": hashlib.sha256(idx.astype("<u8").tobytes()).hexdigest(),
                        "prefixes": marks})
            print(f"world {world} rank {rank}: {gz_bytes} B, {time.time() - t0:.1f} s", flush=True)
    doc = {
        "generator": "tests/golden/make_full_digests.py --ranks",
        "reference": "/root/reference/src/compressor/gzip_compressor.cpp (built by oracle/Makefile ref)",
        "zlib_version": O.ref().ref_zlib_version().decode(),
        "record": "as full_digests.json, over the rank's values in routed-index order",
        "routing": "rank r of N keeps the first n keys 'key'+i (i = 0 .. route_span - 1, route_span = "
                   "int(n * N * 1.05) + 4096) with MurmurHash3_x64_128('key'+i, seed 0)[0] % 128 % N == r",
        "sets": out,
    }
    with open(os.path.join(HERE, "rank_digests.json"), "w") as f:
        json.dump(doc, f, indent=1)


def bytes_digests(corpus, threads):
    """--bytes: SHA-256 over the reference's member BYTES, back to back in value order, for the north-star
    workload at N = 1 (full_digests.json) and every rank of N = 2, 4, 8 (rank_digests.json), stored as
    prefixes[n]["bytes_sha256"] beside the record digests.  bench.py compacts its members on the device and
    hashes them on the host: a byte-by-byte check of all 10M members per GPU."""
    n, vlen, kind, seed = SETS[0]
    path = os.path.join(HERE, "full_digests.json")
    with open(path) as f:
        doc = json.load(f)
    t0 = time.time()
    h = hashlib.sha256()
    for first in range(0, n, CHUNK):
        O.ref_members_hash(O.gen_values(corpus, seed, kind, first, min(CHUNK, n - first), vlen), threads, h)
    for st in doc["sets"]:
        if (st["n"], st["vlen"], st["kind"]) == (n, vlen, kind):
            st["prefixes"][str(n)]["bytes_sha256"] = h.hexdigest()
    doc["bytes_record"] = "bytes_sha256: SHA-256 over the members' bytes, back to back in value order"
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"N=1: {time.time() - t0:.1f} s", flush=True)
    path = os.path.join(HERE, "rank_digests.json")
    with open(path) as f:
        rdoc = json.load(f)
    for st in rdoc["sets"]:
        t0 = time.time()
        world, rank = st["world"], st["rank"]
        route = O.route_keys(0, route_span(RANK_N, world), 128, world)
        idx = np.nonzero(route == rank)[0][:RANK_N].astype(np.uint64)
        assert hashlib.sha256(idx.astype("<u8").tobytes()).hexdigest() == st["index_sha256"]
        h = hashlib.sha256()
        for first in range(0, RANK_N, CHUNK):
            O.ref_members_hash(O.gen_values_idx(corpus, 0x5EED, 0, idx[first:first + CHUNK], 1024), threads, h)
        st["prefixes"][str(RANK_N)]["bytes_sha256"] = h.hexdigest()
        print(f"world {world} rank {rank}: {time.time() - t0:.1f} s", flush=True)
        with open(path, "w") as f:  # (after every rank: a long run keeps what it finished)
            json.dump(rdoc, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", action="store_true", help="add byte-level digests (bytes_digests)")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--ranks", action="store_true", help="only the per-rank digests (rank_digests.json)")
    ap.add_argument("--large", action="store_true", help="add the large-value bench legs to full_digests.json")
    args = ap.parse_args()
    if args.bytes:
        O.build(ref=True)
        d = os.path.join(HERE, "data")
        corpus = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))
        return bytes_digests(corpus, args.threads)
    if args.large:
        O.build(ref=True)
        d = os.path.join(HERE, "data")
        corpus = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))
        path = os.path.join(HERE, "full_digests.json")
        with open(path) as f:
            doc = json.load(f)
        keep = [st for st in doc["sets"] if (st["n"], st["vlen"], st["kind"]) not in
                {(n, v, k) for n, v, k, _ in LARGE_SETS}]
        for n, vlen, kind, seed in LARGE_SETS:
            t0 = time.time()
            st = digest_set(corpus, n, vlen, kind, seed, LARGE_CHECKPOINTS, args.threads)
            st["corpus"] = "tiled" if vlen > len(corpus) else "as is"
            keep.append(st)
            print(f"{n} x {vlen}: {st['prefixes'][str(n)]['gz_bytes']} B, {time.time() - t0:.1f} s", flush=True)
        doc["sets"] = keep
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
        return
    if args.ranks:
        O.build(ref=True)
        d = os.path.join(HERE, "data")
        corpus = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))
        rank_digests(corpus, args.threads)
        return
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
