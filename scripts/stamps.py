"""Diagnostic: per-phase cycle shares of the deflate kernel (PMC_STAMPS build).

PMC_LIB=libpmc_codec_stamps.so python scripts/stamps.py
Prints wave-cycles per value for each phase.  Shares only -- never quoted as timings.
"""
import os
import sys

os.environ.setdefault("PMC_LIB", "libpmc_codec_stamps.so")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd")]

import torch  # noqa: E402

import pmc_codec  # noqa: E402
from pmc_codec import device as D  # noqa: E402

PHASES = ["stage+crc", "hash+sort", "parse", "#evaluated positions", "#consumed positions", "#evals inside prev span",
          "zero+histogram", "#eval lanes used", "#ext iters", "#general steps", "eval", "chain counts", "search", "#groups",
          "#parse steps", "#search calls"]
COUNTS = {3, 4, 5, 7, 8, 9, 13, 14, 15}
IPHASES = ["inf:stage+header", "inf:block hdr+code lens", "inf:table builds", "lane:#decode iters (wave)",
           "lane:#active lane-iters", "lane:prepare", "lane:decode loop", "lane:finish",
           "rec:phase B", "rec:#jump rounds", "rec:#records", "rec:#members"]
ICOUNTS = {3, 4, 9, 10, 11}


def main():
    ctx = pmc_codec.Context(0)
    L = pmc_codec.lib()
    d = os.path.join(ROOT, "tests", "golden", "data")
    corpus_b = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)))
    corpus = torch.frombuffer(bytearray(corpus_b), dtype=torch.uint8).cuda()
    dbg = torch.zeros(32, dtype=torch.int64, device="cuda")
    L.pmc_debug_stamps(ctx.handle, dbg.data_ptr())
    cases = ((1024, 0, 400_000), (256, 0, 400_000), (4096, 0, 100_000), (1024, 1, 200_000))
    if len(sys.argv) > 1:  # e.g. 30000:0:20000
        cases = tuple(tuple(int(x) for x in a.split(":")) for a in sys.argv[1:])
    for vlen, kind, n in cases:
        data = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
        if kind == 0 and vlen > len(corpus_b):  # (as bench.py: the corpus tiled for values longer than it)
            corpus_b = corpus_b * (vlen // len(corpus_b) + 2)
            corpus = torch.frombuffer(bytearray(corpus_b), dtype=torch.uint8).cuda()
        L.pmc_gen_values(corpus.data_ptr(), len(corpus_b), 0x5EED if kind == 0 else 0xA1B2, kind, 0, None, n,
                         vlen, data.data_ptr(), D.stream_handle())
        off = torch.arange(n, dtype=torch.int64, device="cuda") * vlen
        lens = torch.full((n,), vlen, dtype=torch.int32, device="cuda")
        dbg.zero_()
        torch.cuda.synchronize()
        out, rc = D.compress(ctx, D.Batch(data, off, lens, n, vlen))
        torch.cuda.synchronize()
        back, brc = D.decompress(ctx, out, [vlen] * n)
        torch.cuda.synchronize()
        s = dbg.cpu().tolist()
        for lo, names, what in ((0, PHASES, "deflate"), (16, IPHASES, "inflate")):
            cnt = COUNTS if lo == 0 else ICOUNTS
            tot = sum(v for k, v in enumerate(s[lo:lo + 16]) if k not in cnt)
            bad = int((rc != 0).sum()) if lo == 0 else int((brc != 0).sum())
            print(f"vlen={vlen} kind={kind} n={n} {what}: wave-cycles/value total {tot / n:,.0f}  rc!=0: {bad}")
            for k, name in enumerate(names):
                if s[lo + k]:
                    pct = "" if k in cnt else f"{100 * s[lo + k] / max(tot, 1):5.1f}%"
                    print(f"   {name:24s} {s[lo + k] / n:12,.1f}  {pct}")
    ctx.close()


if __name__ == "__main__":
    main()
