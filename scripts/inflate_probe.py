"""Diagnostic: how many members of each size the decompress fast paths (record / lane kernels) decode
themselves, i.e. do not hand to the wave-per-member kernels (pmc_ctx_guard_counts counts[4]).
usage: python scripts/inflate_probe.py 30000 16000 4096 300000:32
(vlen[:n], n = 4096 by default; values longer than the corpus are slices of it tiled)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd"), os.path.join(ROOT, "tests")]

import pmc_codec  # noqa: E402
from test_gpu_inflate_rec import _lane_pass_counts  # noqa: E402

ctx = pmc_codec.Context(0)
for arg in sys.argv[1:] or ["30000"]:
    vlen, n = (int(x) for x in arg.split(":")) if ":" in arg else (int(arg), 4096)
    same, retried = _lane_pass_counts(ctx, vlen, n)
    print(f"vlen={vlen} n={n} byte-exact={same} handed to the wave kernels={retried}", flush=True)
ctx.close()
