"""Value sets of the large-value tests (test infrastructure).

One builder per set, shared by tests/test_gpu_large.py, tests/test_gpu_codec.py and the generator of
their reference vectors (tests/golden/make_large_golden.py), so the GPU tests, the oracle test and
the committed fixture describe exactly the same bytes.  Every builder is deterministic (seeded numpy
generators over the reference's tests/data corpus).

The reference accepts values up to 512 MiB (/root/reference/src/server/constants.hpp:8); the
committed golden.npz stops at the whole 82,002 B corpus, so these sets carry parity from 82 KB to
4 MiB: tiled JSON, alphanumeric, small binary alphabets, random bytes, and period-1/2 runs.
"""
import numpy as np

ALNUM = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)


def segment_boundaries_json(corpus):
    """JSON slices around every multiple of the 16 KiB segment and the 32 KiB window slides."""
    tiled = corpus * 40
    rng = np.random.default_rng(5)
    sizes = [31809, 32768, 32769, 49151, 49152, 49153, 65274, 65275, 65536, 65537, 98304 + 7, 131071,
             200000, 262144, 333333]
    return [tiled[int(o):int(o) + s] for s, o in zip(sizes, rng.integers(0, 82002, len(sizes)))]


def binary_and_stored():
    """Small alphabets (long chains, many cut walks), random bytes (stored blocks) and alnum."""
    rng = np.random.default_rng(17)
    vals = []
    for s in (40000, 70001, 140000, 300007):
        vals.append(bytes(rng.integers(0, 4, s, dtype=np.uint8)))
        vals.append(bytes(rng.integers(0, 256, s, dtype=np.uint8)))
        vals.append(bytes(rng.choice(ALNUM, s)))
    return vals


def periodic():
    """Runs of period 2 and 1 (zero bytes): 258-byte matches from the first candidate."""
    vals = []
    for s in (40000, 70001, 140000, 300007):
        vals.append(b"xy" * (s // 2) + b"x" * (s % 2))
        vals.append(bytes(s))
    return vals


def periodic_megabyte():
    return [bytes(1 << 20), b"ab" * (1 << 19)]


def mixed_with_small(corpus):
    """200 large JSON values of ragged sizes beside small ones."""
    tiled = corpus * 4
    rng = np.random.default_rng(23)
    vals = []
    for k in range(200):
        s = int(rng.integers(31809, 160000))
        o = int(rng.integers(0, 82002))
        vals.append(tiled[o:o + s])
        vals.append(corpus[k:k + 1 + int(rng.integers(0, 3000))])
    return vals


def multi_megabyte(corpus):
    """1 MiB of JSON, 2 MiB of a small binary alphabet, 4 MiB of a period-2 pattern, two small values."""
    rng = np.random.default_rng(99)
    tiled = corpus * (1 + (1 << 20) // len(corpus))
    return [tiled[:1 << 20], bytes(rng.integers(0, 4, 2 << 20, dtype=np.uint8)), b"xy" * (2 << 20),
            corpus[:300], corpus[5:1029]]


CLASS_SIZES = (100_000, 333_333, 1 << 20, 4 << 20)


def size_classes(corpus, sizes=CLASS_SIZES):
    """VERDICT r4 item 1's classes: for 100 KB, 333 KB, 1 MiB and 4 MiB, a tiled-JSON slice, random
    alnum, an `xy...` run and an `a...` run (all NUL-free: the reference's own Compress makes them)."""
    rng = np.random.default_rng(0x1A96E)
    tiled = corpus * (2 + max(sizes) // len(corpus))
    vals = []
    for s in sizes:
        o = int(rng.integers(0, len(corpus)))
        vals.append(tiled[o:o + s])
        vals.append(bytes(rng.choice(ALNUM, s)))
        vals.append((b"xy" * (s // 2 + 1))[:s])
        vals.append(b"a" * s)
    return vals


def block_edges():
    """Values whose parse ends exactly on a 16383-symbol block boundary with a literal: zlib's deflate_slow
    tallies the last literal after its loop, where a full symbol buffer does not flush, so the final
    block holds 16383 symbols (found by searching the oracle's parses of prefixes of seeded random
    strings; NUL-free, so the reference makes them).  Plus random bytes around one and two blocks
    (stored blocks, NULs: libz)."""
    alnum = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
    hexd = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
    cuts = {(0, 0): (16929, 33901), (0, 1): (16884, 33875), (0, 2): (16866, 33916), (0, 3): (16888, 33898),
            (1, 0): (40512, 40515)}
    vals = []
    for (a, seed), ns in cuts.items():
        big = bytes(np.random.default_rng(77 + seed).choice(alnum if a == 0 else hexd, 52000))
        vals += [big[:n] for n in ns] + [big[:n + 1] for n in ns] + [big[:n - 1] for n in ns]
    for s in list(range(16380, 16400, 3)) + [32766, 32767, 32768, 32769]:
        vals.append(bytes(np.random.default_rng(s).integers(0, 256, s, dtype=np.uint8)))
    return vals


def all_sets(corpus):
    """{set name: [values]} -- every set the reference vectors cover."""
    return {
        "segment_boundaries_json": segment_boundaries_json(corpus),
        "binary_and_stored": binary_and_stored(),
        "periodic": periodic(),
        "periodic_megabyte": periodic_megabyte(),
        "mixed_with_small": mixed_with_small(corpus),
        "multi_megabyte": multi_megabyte(corpus),
        "size_classes": size_classes(corpus),
        "block_edges": block_edges(),
    }
