"""GPU: the lane-order guards (include/pmc_codec.h pmc_ctx_guard_counts).

The throughput compressor takes two ranks from returning LDS atomics, relying on the lanes of one
ds_add_rtn_u32 that hit the same word getting their old values in lane order (measured on gfx950,
not documented): the hash sort's scatter (pmc_deflate_small.hip sort_positions2_body) and the
canonical-code ranks (codes_from_lengths_all).  Each value is checked -- (hash, position)
increasing along the sorted array in build_cn; the symbol before each one in canonical order
being smaller -- and a value that fails goes to the HBM kernel.

* the product library: the create-time probe and both guards read 0 over every golden vector;
* libpmc_codec_fault.so (-DPMC_FAULT_LANE_ORDER): the sort's scatter (odd values) and the code ranks take a
  chunk's lanes in reverse, i.e. the atomics misbehave on purpose; the guards must fire and every
  member must still equal the reference's bytes (tests/golden, made by the reference's own
  Compress) -- a batch with large values (the HBM kernel runs anyway) and one of small values only
  (its retry pass is the gated launch; the small batch is kept on the split pipeline with
  PMC_LATENCY_BATCH=0);
* the fault build's one-kernel path (host calls of <= 1,024 small values, which has no retry pass of its
  own) declines every odd value: those are redone by a pipeline call, bit-exact.
Each library runs in a child process of its own (the C-ABI loads one library per process)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "poor-man-s-cache_amd", "pmc_codec")

CHILD = r"""
import json, sys
sys.path[:0] = [sys.argv[1]]
from conftest import Golden
import pmc_codec
from pmc_codec import device as D
import torch
g = Golden()
pairs = g.pairs()
ctx = pmc_codec.Context(0)
res = {}
for name, sel in (("all", pairs), ("small", [p for p in pairs if 0 < len(p[0]) <= 4096])):
    out, rc = D.compress(ctx, D.pack([r for r, _ in sel]))
    torch.cuda.synchronize()
    rc = rc.cpu().numpy()
    got = out.host_items()
    res[name] = {"n": len(sel), "bad": [k for k, (r, z) in enumerate(sel) if rc[k] != 0 or got[k] != z][:8]}
    res[name + "_guards"] = ctx.guard_counts()
ctx.close()
print(json.dumps(res))
"""


def _run(lib, **extra):
    env = dict(os.environ, PMC_LIB=lib, **extra)
    out = subprocess.run([sys.executable, "-c", CHILD, HERE], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    import json
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_guards_silent_on_the_product_library():
    r = _run("libpmc_codec.so")
    assert r["all"]["bad"] == [] and r["small"]["bad"] == [], r
    g = r["small_guards"]
    assert (g["sort"], g["codes"], g["probe"]) == (0, 0, 0), r


@pytest.mark.gpu
def test_forced_lane_order_fault_is_caught_and_retried_bit_exact():
    if not os.path.exists(os.path.join(PKG, "libpmc_codec_fault.so")):
        pytest.fail("libpmc_codec_fault.so missing: run `make -C poor-man-s-cache_amd`")
    # (PMC_LATENCY_BATCH=0: the 721-value small batch goes through the split pipeline, whose atomics the
    # fault build breaks, not the one-kernel path device-resident batches of <= 1,024 small values take)
    r = _run("libpmc_codec_fault.so", PMC_LATENCY_BATCH="0")
    # every member equals the reference's bytes although (almost) every value failed a guard
    assert r["all"]["bad"] == [] and r["small"]["bad"] == [], r
    g1, g2 = r["all_guards"], r["small_guards"]
    assert g1["probe"] == 0, r  # (the hardware itself is fine: the fault is in the kernels)
    assert g1["sort"] > 0 and g1["codes"] > 0, r
    # the small-only batch's retries came from the gated HBM launch
    assert g2["sort"] > g1["sort"], r


CHILD_HOST = r"""
import json, sys
sys.path[:0] = [sys.argv[1]]
from conftest import Golden
import pmc_codec
g = Golden()
small = [p for p in g.pairs() if 0 < len(p[0]) <= 4096]
ctx = pmc_codec.Context(0)
res = {"n": 0, "bad": []}
# host calls of <= 1,024 values of <= 4 KiB take the latency path (one kernel on zero-copy host memory)
for k0 in range(0, len(small), 256):
    sel = small[k0:k0 + 256]
    got = ctx.compress_many([r for r, _ in sel])
    res["bad"] += [k0 + k for k, ((c, z), (_, want)) in enumerate(zip(got, sel)) if c != 0 or z != want][:8]
    res["n"] += len(sel)
res["paths"] = ctx.path_counts()
res["redone"] = ctx.latency_redone()
res["guards"] = ctx.guard_counts()
ctx.close()
print(json.dumps(res))
"""


def _run_host(lib):
    env = dict(os.environ, PMC_LIB=lib)
    out = subprocess.run([sys.executable, "-c", CHILD_HOST, HERE], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    import json
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_latency_path_declined_values_redone_through_the_pipeline():
    """the latency path (host calls, one wave-per-value kernel) has no retry pass; values it
    declines are redone alone by a pipeline call (pmc_capi.hip host_batch_locked).  Under the fault build
    its guards decline values on purpose: every member must still be the reference's, the calls must
    have taken the latency route AND the pipeline route, and the product library must never need it."""
    if not os.path.exists(os.path.join(PKG, "libpmc_codec_fault.so")):
        pytest.fail("libpmc_codec_fault.so missing: run `make -C poor-man-s-cache_amd`")
    f = _run_host("libpmc_codec_fault.so")
    assert f["bad"] == [] and f["n"] > 700, f
    assert f["paths"]["latency_compress"] >= 3 and f["redone"] > 0, f
    assert f["paths"]["pipeline_compress"] == f["redone"], f  # (one pipeline call per redone latency call)
    assert f["guards"]["sort"] > 0 or f["guards"]["codes"] > 0, f
    p = _run_host("libpmc_codec.so")
    assert p["bad"] == [] and p["redone"] == 0 and p["paths"]["pipeline_compress"] == 0, p
