"""Host-memory calls of at most 64 values: latency path (one wave-per-value kernel over coherent host memory)
against the throughput pipeline.  Run twice, PMC_LATENCY_MAX_LEN=0 (pipeline for every size) and =4096
(latency path up to 4 KiB); one JSON line per (values, value_bytes), host wall clock, median of 50 calls,
every result checked against the first call's members and the values (a stability check for the timing,
not parity: the reference's bytes for these calls are asserted by
tests/test_gpu_codec.py::test_latency_path_batches_vs_reference and test_device_small_batches_vs_reference).

usage: PMC_LATENCY_MAX_LEN=0 python scripts/few_sweep.py > few_0.jsonl
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd")]

import numpy as np  # noqa: E402

import pmc_codec  # noqa: E402
from values import gen_values  # noqa: E402  (scripts/values.py: the device generator)


def main():
    ctx = pmc_codec.Context(0)
    few = os.environ.get("PMC_LATENCY_MAX_LEN", "default") + "/" + os.environ.get("PMC_LATENCY_BATCH", "default")
    sizes = [int(x) for x in os.environ.get("SWEEP_N", "1,4,16,64").split(",")]
    for vlen in (256, 1024, 4096):
        for n in sizes:
            vals = gen_values(n, vlen)
            ref = ctx.compress_many(vals)
            assert all(r == 0 for r, _ in ref)
            members = [g for _, g in ref]
            for _ in range(5):
                ctx.compress_many(vals)
                ctx.decompress_many(members, [vlen] * n)
            tc, td, bad = [], [], 0
            for _ in range(50):
                t0 = time.perf_counter()
                res = ctx.compress_many(vals)
                t1 = time.perf_counter()
                back = ctx.decompress_many(members, [vlen] * n)
                t2 = time.perf_counter()
                tc.append((t1 - t0) * 1e3)
                td.append((t2 - t1) * 1e3)
                bad += sum(1 for (r, g), m in zip(res, members) if r or g != m)
                bad += sum(1 for (r, v2), v in zip(back, vals) if r or v2 != v)
            print(json.dumps({"latency_max_len": few, "values": n, "value_bytes": vlen, "compress_ms": float(np.median(tc)),
                              "decompress_ms": float(np.median(td)), "mismatches": bad}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
