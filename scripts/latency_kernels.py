"""Diagnostic: device-resident compress of ONE value (1 KiB JSON slice) per call -- the throughput
pipeline's launch chain (front, trees, back, ...) against the single wave-per-value kernel
(PMC_DEFLATE_MONO=1, what the latency path runs).  Run under rocprofv3 --kernel-trace --stats for the
per-kernel split.  usage: [PMC_DEFLATE_MONO=1] python scripts/latency_kernels.py [vlen] [calls]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd")]
import torch  # noqa: E402

import pmc_codec  # noqa: E402
from pmc_codec import device as D  # noqa: E402

vlen = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 300
d = os.path.join(ROOT, "tests", "golden", "data")
cb = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))
ctx = pmc_codec.Context(0)
b = D.pack([cb[1000:1000 + vlen]])
out, rc = D.compress(ctx, b)  # warm-up (sizes the scratch)
torch.cuda.synchronize()
ts = []
for _ in range(calls):
    t0 = time.perf_counter()
    out, rc = D.compress(ctx, b)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
ts.sort()
print(f"mono={os.environ.get('PMC_DEFLATE_MONO', '0')} vlen={vlen} median_us={ts[len(ts) // 2] * 1e6:.1f} "
      f"p10_us={ts[len(ts) // 10] * 1e6:.1f} rc={int(rc[0])} clen={int(out.len[0])}", flush=True)
ctx.close()
