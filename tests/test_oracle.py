"""CPU: pin the oracle (oracle/, test infrastructure) against the reference's goldens.

The goldens (tests/golden/) were produced by the reference's own GzipCompressor built from
/root/reference/src/compressor/gzip_compressor.cpp (tests/golden/make_golden.py).  Both
CPU restatements -- the zlib-shaped one and the data-parallel-shaped one the HIP kernels
mirror -- must reproduce every byte; the oracle inflate must reproduce every verdict.
"""
import hashlib
import os
import zlib

import numpy as np
import pytest

from oracle import pyoracle as O


@pytest.mark.parametrize("dp", [False, True], ids=["faithful", "data_parallel"])
def test_compress_matches_reference_goldens(golden, dp):
    bad = [k for k, (r, g) in enumerate(golden.pairs()) if O.compress(r, dp=dp) != g]
    assert not bad, f"{len(bad)} golden vectors differ, first {bad[:5]}"


def test_inflate_roundtrips_goldens(golden):
    for k, (r, g) in enumerate(golden.pairs()):
        rc, out = O.decompress(g)
        assert rc == 0 and out == r, k


def test_decompress_error_verdicts(golden):
    """The reference's verdict and bytes for every decompress vector: with a roomy buffer, and with
    the ISIZE-sized first guess that members followed by extra bytes overflow (capacity is then
    reported with the decoded size, never as a verdict)."""
    grew = 0
    for e in golden.index["decompress_errors"]:
        v = bytes.fromhex(e["hex"])
        want = bytes.fromhex(e["expect_hex"]) if e["expect_rc"] == 0 else b""
        for cap in (1 << 16, None):
            rc, out = O.decompress(v, cap=cap)
            assert rc == e["expect_rc"], (e["name"], cap, rc)
            assert out == want, (e["name"], cap)
        rc, _ = O.decompress(v, grow=False)
        grew += rc == O.CAPACITY
    assert grew >= 4


def test_generator_pins_golden_sets(golden):
    for s in golden.index["sets"]:
        vals = O.gen_values(golden.corpus, s["seed"], s["kind"], 0, s["n"], s["vlen"])
        for k in range(s["n"]):
            r, _ = golden.pair(s["first_vector"] + k)
            assert vals[k].tobytes() == r


@pytest.mark.parametrize("dp", [False, True], ids=["faithful", "data_parallel"])
def test_digest_sets(golden, dp):
    for d in golden.index["digests"]:
        vals = O.gen_values(golden.corpus, d["seed"], d["kind"], 0, d["n"], d["vlen"])
        h = hashlib.sha256()
        sizes = []
        for k in range(d["n"]):
            gz = O.compress(vals[k].tobytes(), dp=dp)
            h.update(gz)
            sizes.append(len(gz))
        assert h.hexdigest() == d["sha256"], d
        assert hashlib.sha256(np.asarray(sizes, np.uint32).tobytes()).hexdigest() == d["sizes_sha256"]


def test_crc32_matches_zlib():
    rng = np.random.default_rng(3)
    for n in (0, 1, 15, 16, 17, 1000, 65537):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert O.crc32(b) == zlib.crc32(b)


def test_reference_unit_cases():
    """gzip_compressor_test.cpp:6-95 re-expressed against the oracle."""
    s = b"Hello, Gzip!"
    rc, out = O.decompress(O.compress(s))
    assert rc == 0 and out == s
    long = (b"This is a long test string. It should be compressed and decompressed properly. "
            b"We are testing to see if gzip can handle long input.")
    assert len(O.compress(long)) < len(long)
    assert len(O.compress(b"A" * 50)) < 50
    rc, _ = O.decompress(b"Not a gzip string")
    assert rc < 0


def test_bound_covers_worst_case():
    rng = np.random.default_rng(5)
    for n in (1, 29, 1024, 70000):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert len(O.compress(b)) <= O.bound(n)


def test_murmur_restatement_matches_reference_hash():
    """oracle/util.c's MurmurHash3_x64_128 restatement (the checker of pmc_route_keys) equals the
    reference's own hashFunc (hash.cpp:4-9) on every key of tests/golden/route_golden.npz."""
    import ctypes
    L = O.lib()
    L.oracle_murmur3_x64_128_h1.restype = ctypes.c_uint64
    L.oracle_murmur3_x64_128_h1.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32]
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "route_golden.npz"))
    for i, h in zip(z["index"], z["hash"]):
        k = b"key%d" % int(i)
        assert L.oracle_murmur3_x64_128_h1(k, len(k), 0) == int(h), int(i)


def test_oracle_matches_large_reference_vectors(golden, large_golden):
    """The restatement above 82 KB (window slides, block flushes, stored-block window test, 4 MiB runs)
    against the reference's own members (tests/golden/large_golden.json, tests/golden/make_large_golden.py):
    every value of every large set, hashed."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import large_values
    sets = large_values.all_sets(golden.corpus)
    assert set(sets) == set(large_golden.sets)
    n = 0
    for name, vals in sets.items():
        got = [O.compress(v) for v in vals]
        bad = large_golden.mismatches(vals, got)
        assert not bad, (name, [len(vals[k]) for k in bad[:5]])
        n += len(vals)
    assert n == sum(len(v) for v in large_golden.sets.values())
