"""Single-value latency: the drop-in's per-call path vs the reference codec on one core.

The unchanged server calls GzipCompressor::Compress / ::Decompress once per value on its single
request thread (kvs.cpp:183,233; server.cpp:631-643).  The drop-in does each call through
pmc_gzip_compress / pmc_gzip_decompress (pinned staging, H2D, kernels, D2H, synchronize); the
reference does it with zlib on the calling core (oracle/_ref/libref_gzip.so, its own
gzip_compressor.cpp).  Both are timed here per call over the same JSON-slice values (SURVEY.md §8d
generator), through ctypes (the same ~1 us call overhead on both sides).

usage: python scripts/latency_dropin.py [--calls 2000] > profiles/r02/latency_dropin.json
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd")]

import pmc_codec  # noqa: E402
from values import gen_values  # noqa: E402  (scripts/values.py: the device generator)
# (oracle/_ref is loaded only to time the reference codec itself -- this script's CPU baseline, as bench.py's
# cpu_baseline leg does; every drop-in call measured goes through libpmc_codec)
from oracle import pyoracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    args = ap.parse_args()
    L = pmc_codec.lib()
    ctx = L.pmc_default_ctx()
    assert ctx, "no device"
    R = O.ref() if O.ref_available() else None
    out = {"note": __doc__.split("\n\n")[1].replace("\n", " "), "sizes": []}
    for vlen in (32, 256, 1024, 4096, 30000):
        n = args.calls if vlen <= 4096 else max(200, args.calls // 5)
        vals = gen_values(n, vlen)
        cap = pmc_codec.gzip_bound(vlen)
        obuf = ctypes.create_string_buffer(cap)
        dbuf = ctypes.create_string_buffer(vlen + 64)
        olen = ctypes.c_size_t()
        members = []
        for v in vals[:20]:  # warm-up (context, staging buffers, kernels)
            assert L.pmc_gzip_compress(ctx, v, len(v), obuf, cap, ctypes.byref(olen)) == 0
        t0 = time.perf_counter()
        for v in vals:
            L.pmc_gzip_compress(ctx, v, len(v), obuf, cap, ctypes.byref(olen))
            members.append(obuf.raw[:olen.value])
        t1 = time.perf_counter()
        for m in members:
            rc = L.pmc_gzip_decompress(ctx, m, len(m), dbuf, vlen + 64, ctypes.byref(olen))
            assert rc == 0 and olen.value == vlen
        t2 = time.perf_counter()
        row = {"value_bytes": vlen, "calls": n, "dropin_compress_us": (t1 - t0) / n * 1e6,
               "dropin_decompress_us": (t2 - t1) / n * 1e6}
        if R is not None:
            zs = []
            t0 = time.perf_counter()
            for v in vals:
                zs.append(O.ref_compress(v)[1])
            t1 = time.perf_counter()
            for z in zs:
                O.ref_decompress(z)
            t2 = time.perf_counter()
            row.update({"reference_compress_us": (t1 - t0) / n * 1e6, "reference_decompress_us": (t2 - t1) / n * 1e6,
                        "bytes_equal": zs == members})
        out["sizes"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
