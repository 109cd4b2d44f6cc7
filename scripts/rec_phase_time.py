"""inflate_rec_kernel time by phase: with the stop build (PMC_LIB=libpmc_codec_stop.so), PMC_STOP_AFTER=31 ends
each member after its code tables (prepare), 32 after phase A (records), -1 runs everything; the kernel's time
per launch (HIP events around it, pmc_ctx_profile) differences give each phase's share.  Diagnostic only.

usage: PMC_LIB=libpmc_codec_stop.so PMC_STOP_AFTER=32 python scripts/rec_phase_time.py N VLEN
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd")]
import torch  # noqa: E402

import pmc_codec  # noqa: E402
from pmc_codec import device as D  # noqa: E402


def main():
    n, vlen = int(sys.argv[1]), int(sys.argv[2])
    L = pmc_codec.lib()
    ctx = pmc_codec.Context(0)
    d = os.path.join(ROOT, "tests", "golden", "data")
    corpus_b = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)))
    corpus = torch.frombuffer(bytearray(corpus_b), dtype=torch.uint8).cuda()
    data = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
    L.pmc_gen_values(corpus.data_ptr(), len(corpus_b), 0x5EED, 0, 0, None, n, vlen, data.data_ptr(), D.stream_handle())
    off = torch.arange(n, dtype=torch.int64, device="cuda") * vlen
    lens = torch.full((n,), vlen, dtype=torch.int32, device="cuda")
    out, rc = D.compress(ctx, D.Batch(data, off, lens, n, vlen))
    torch.cuda.synchronize()
    D.decompress(ctx, out, [vlen] * n)
    torch.cuda.synchronize()
    res = {}
    for rep in range(3):
        ctx.profile(True)
        D.decompress(ctx, out, [vlen] * n)
        torch.cuda.synchronize()
        kt = ctx.kernel_times()
        ctx.profile(False)
        for k, (ms, c) in kt.items():
            res.setdefault(k, []).append(ms / c)
    print(json.dumps({"stop_after": os.environ.get("PMC_STOP_AFTER", "-1"), "n": n, "vlen": vlen,
                      "ms_per_launch": {k: min(v) for k, v in res.items()}}))
    ctx.close()


if __name__ == "__main__":
    main()
