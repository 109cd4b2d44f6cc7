"""GPU: the large-value path (pmc_deflate_large.hip) -- values above the split pipeline's large pass
(~31.8 KB; the reference accepts values up to 512 MiB, /root/reference/src/server/constants.hpp:8).

Each value is sorted by hash in HBM, parsed by one wave per 16 KiB segment from a fresh deflate_slow
state, stitched where consecutive parses reach the same state, and emitted block by block.  These
tests check the reference's bytes (the oracle restates zlib 1.2.11, pinned by the goldens made by the
reference's own Compress) across segment boundaries, window slides, multi-block members, stored
blocks (random bytes), long matches and ragged sizes, and that the values were really stitched (the
context's retry counter, pmc_ctx_guard_counts counts[3], stays put: no value fell back to the HBM
kernel)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def sync():
    torch.cuda.synchronize()


@pytest.fixture(scope="module")
def ctx():
    import pmc_codec
    c = pmc_codec.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def D():
    from pmc_codec import device
    return device


def _check(ctx, D, vals, may_fall_back=False):
    from oracle import pyoracle as O
    before = ctx.guard_counts()["retry"]
    out, rc = D.compress(ctx, D.pack(vals))
    sync()
    rc = rc.cpu().numpy()
    got = out.host_items()
    bad = [(k, len(v)) for k, v in enumerate(vals) if rc[k] != 0 or got[k] != O.compress(v)]
    assert not bad, bad[:8]
    if not may_fall_back:
        assert ctx.guard_counts()["retry"] == before, "a large value fell back to the HBM kernel"
    back, brc = D.decompress(ctx, D.pack(got), [len(v) for v in vals])
    sync()
    assert int((brc != 0).sum()) == 0
    assert back.host_items() == vals


def test_segment_boundaries_json(ctx, D, golden):
    """JSON slices around every multiple of the 16 KiB segment and the 32 KiB window slides."""
    corpus = golden.corpus * 40
    rng = np.random.default_rng(5)
    sizes = [31809, 32768, 32769, 49151, 49152, 49153, 65274, 65275, 65536, 65537, 98304 + 7, 131071,
             200000, 262144, 333333]
    vals = [corpus[int(o):int(o) + s] for s, o in zip(sizes, rng.integers(0, 82002, len(sizes)))]
    _check(ctx, D, vals)


def test_binary_and_stored(ctx, D):
    """Small alphabets (long chains, many cut walks), random bytes (stored blocks: the window base
    decides whether a block may be stored) and alnum."""
    rng = np.random.default_rng(17)
    vals = []
    for s in (40000, 70001, 140000, 300007):
        vals.append(bytes(rng.integers(0, 4, s, dtype=np.uint8)))
        vals.append(bytes(rng.integers(0, 256, s, dtype=np.uint8)))
        vals.append(bytes(rng.choice(np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789",
                                                   dtype=np.uint8), s)))
    _check(ctx, D, vals)


def test_periodic_values(ctx, D):
    """Runs of period 1 and 2 (258-byte matches from the first candidate).  Two parses of such a run meet
    at the same loop top only if they are in phase modulo 258, which a 2 KiB overlap rarely sees, so these
    values fall back to the gated HBM kernel (the stitch's failure path, counted in guard[3]); their
    searches end at the first candidate, so that path is short for exactly them.  Bytes must still be
    the reference's, and a 1 MiB run must not hold its batch for long."""
    import time
    vals = []
    for s in (40000, 70001, 140000, 300007):
        vals.append(b"xy" * (s // 2) + b"x" * (s % 2))
        vals.append(bytes(s))
    _check(ctx, D, vals, may_fall_back=True)
    from oracle import pyoracle as O
    for v in (bytes(1 << 20), b"ab" * (1 << 19)):  # each alone: the time one such value holds a batch
        D.compress(ctx, D.pack([v]))
        sync()
        t0 = time.perf_counter()
        out, rc = D.compress(ctx, D.pack([v]))
        sync()
        dt = time.perf_counter() - t0
        assert int((rc != 0).sum()) == 0 and out.host_items() == [O.compress(v)]
        print(f"1 MiB periodic value ({v[:2]!r}...): {dt * 1e3:.1f} ms")
        assert dt < 0.1


def test_many_values_mixed_with_small(ctx, D, golden):
    """A batch of 200 large JSON values of ragged sizes beside small ones (the split pipeline's)."""
    corpus = golden.corpus * 4
    rng = np.random.default_rng(23)
    vals = []
    for k in range(200):
        s = int(rng.integers(31809, 160000))
        o = int(rng.integers(0, 82002))
        vals.append(corpus[o:o + s])
        vals.append(golden.corpus[k:k + 1 + int(rng.integers(0, 3000))])
    _check(ctx, D, vals)
