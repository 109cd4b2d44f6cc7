"""GPU: the large-value path (pmc_deflate_large.hip) -- values above the split pipeline's large pass
(~31.8 KB; the reference accepts values up to 512 MiB, /root/reference/src/server/constants.hpp:8).

Each value is sorted by hash in HBM, parsed by one wave per 16 KiB segment from a fresh deflate_slow
state, stitched where consecutive parses reach the same state, and emitted block by block.  These
tests check the reference's bytes (the oracle restates zlib 1.2.11, pinned by the goldens made by the
reference's own Compress) across segment boundaries, window slides, multi-block members, stored
blocks (random bytes), long matches and ragged sizes, and that the values were really stitched (the
context's retry counter, pmc_ctx_guard_counts counts[3], stays put: no value fell back to the HBM
kernel)."""
import os
import sys
import time

import pytest
import torch

sys.path.insert(0, os.path.dirname(__file__))
import large_values as LV  # noqa: E402

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


def _check(ctx, D, vals, lg, may_fall_back=False):
    """Compress the batch; every member must be the reference's (tests/golden/large_golden.json, made by
    the reference's own Compress) and the oracle's; then the round trip."""
    from oracle import pyoracle as O
    before = ctx.guard_counts()["retry"]
    out, rc = D.compress(ctx, D.pack(vals))
    sync()
    rc = rc.cpu().numpy()
    got = out.host_items()
    bad = [(k, len(v)) for k, v in enumerate(vals) if rc[k] != 0]
    assert not bad, bad[:8]
    bad = lg.mismatches(vals, got)
    assert not bad, [("reference", k, len(vals[k])) for k in bad[:8]]
    bad = [(k, len(v)) for k, v in enumerate(vals) if got[k] != O.compress(v)]
    assert not bad, bad[:8]
    if not may_fall_back:
        assert ctx.guard_counts()["retry"] == before, "a large value fell back to the HBM kernel"
    back, brc = D.decompress(ctx, D.pack(got), [len(v) for v in vals])
    sync()
    assert int((brc != 0).sum()) == 0
    assert back.host_items() == vals


def test_segment_boundaries_json(ctx, D, golden, large_golden):
    """JSON slices around every multiple of the 16 KiB segment and the 32 KiB window slides."""
    _check(ctx, D, LV.segment_boundaries_json(golden.corpus), large_golden)


def test_binary_and_stored(ctx, D, large_golden):
    """Small alphabets (long chains, many cut walks), random bytes (stored blocks: the window base
    decides whether a block may be stored) and alnum."""
    _check(ctx, D, LV.binary_and_stored(), large_golden)


def test_periodic_values(ctx, D, large_golden):
    """Runs of period 1 and 2 (258-byte matches from the first candidate).  Two parses of such a run meet
    at the same loop top only if they are in phase modulo 258, which a 2 KiB overlap rarely sees, so these
    values fall back to the gated HBM kernel (the stitch's failure path, counted in guard[3]); their
    searches end at the first candidate, so that path is short for exactly them.  Bytes must still be
    the reference's, and a 1 MiB run must not hold its batch for long."""
    _check(ctx, D, LV.periodic(), large_golden, may_fall_back=True)
    for v in LV.periodic_megabyte():  # each alone: the time one such value holds a batch
        D.compress(ctx, D.pack([v]))
        sync()
        t0 = time.perf_counter()
        out, rc = D.compress(ctx, D.pack([v]))
        sync()
        dt = time.perf_counter() - t0
        assert int((rc != 0).sum()) == 0 and not large_golden.mismatches([v], out.host_items())
        print(f"1 MiB periodic value ({v[:2]!r}...): {dt * 1e3:.1f} ms")
        assert dt < 0.1


def test_many_values_mixed_with_small(ctx, D, golden, large_golden):
    """A batch of 200 large JSON values of ragged sizes beside small ones (the split pipeline's)."""
    _check(ctx, D, LV.mixed_with_small(golden.corpus), large_golden)


def test_size_classes_100k_to_4m(ctx, D, golden, large_golden):
    """100 KB, 333 KB, 1 MiB and 4 MiB values of tiled JSON, alnum, `xy...` and `a...` in one
    batch, each member the reference's own (period-1/2 runs may take the stitch's fallback)."""
    _check(ctx, D, LV.size_classes(golden.corpus), large_golden, may_fall_back=True)


def test_block_edges(ctx, D, large_golden):
    """A parse ending exactly on a 16383-symbol boundary with a literal (zlib: no flush for the last literal, the
    final block holds 16383 symbols), and random bytes around one and two blocks (stored blocks)."""
    _check(ctx, D, LV.block_edges(), large_golden)


def test_mid_size_small_batches_take_the_large_pass(ctx, D, golden, large_golden):
    """Values of 16,383-32,506 B: a batch of at most 2 values per CU whose values all fit the split pipeline's
    large pass keeps it (a lone 30 KB value: 5 ms there, 10 ms through the large-value pipeline); bigger
    batches take the large-value pipeline (the 100K x 30 KB bench leg, digest-checked).  Every reference
    vector of that size class, in batches of 1, 7 and all of them, against the reference's members.  Values
    of several DEFLATE blocks (random bytes) are redone by the HBM kernel here, so no retry-counter check."""
    vals = [v for sets in LV.all_sets(golden.corpus).values() for v in sets if 16383 <= len(v) <= 32506]
    assert len(vals) >= 15, len(vals)
    for m in (1, 7, len(vals)):
        for k in range(0, len(vals), m):
            _check(ctx, D, vals[k:k + m], large_golden, may_fall_back=True)
