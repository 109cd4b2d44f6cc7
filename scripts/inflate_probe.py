"""Diagnostic: which members each inflate stage accepts (PMC_DIAG_INFLATE_STOP=1: after the record / lane
kernels, 2: after the CRC check), by value size.  usage: python scripts/inflate_probe.py 30000 16000 4096 300000:32
(vlen[:n], n = 4096 by default; values longer than the corpus are slices of it tiled)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd")]

if os.environ.get("PMC_DIAG_INFLATE_STOP") is None:  # parent: one child per stop setting (the knob is read once)
    for stop in ("1", "2", "0"):
        r = subprocess.run([sys.executable, __file__] + sys.argv[1:], env=dict(os.environ, PMC_DIAG_INFLATE_STOP=stop))
        if r.returncode:
            sys.exit(r.returncode)
    sys.exit(0)

import torch  # noqa: E402

import pmc_codec  # noqa: E402
from pmc_codec import device as D  # noqa: E402

L = pmc_codec.lib()
ctx = pmc_codec.Context(0)
d = os.path.join(ROOT, "tests", "golden", "data")
cb = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))
corpus = torch.frombuffer(bytearray(cb), dtype=torch.uint8).cuda()
for arg in sys.argv[1:] or ["30000"]:
    vlen, n = (int(x) for x in arg.split(":")) if ":" in arg else (int(arg), 4096)
    if vlen > len(cb):
        cb = cb * (vlen // len(cb) + 2)
        corpus = torch.frombuffer(bytearray(cb), dtype=torch.uint8).cuda()
    data = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
    assert L.pmc_gen_values(corpus.data_ptr(), len(cb), 0x5EED, 0, 0, None, n, vlen, data.data_ptr(),
                            D.stream_handle()) == 0
    off = torch.arange(n, dtype=torch.int64, device="cuda") * vlen
    lens = torch.full((n,), vlen, dtype=torch.int32, device="cuda")
    out, rc = D.compress(ctx, D.Batch(data, off, lens, n, vlen))
    back, brc = D.decompress(ctx, out, [vlen] * n)
    torch.cuda.synchronize()
    vals, cnt = torch.unique(brc.cpu(), return_counts=True)
    ok = int((brc == 0).sum())
    same = 0
    if ok:
        bo = back.host_items()
        src = data.cpu().numpy().tobytes()
        same = sum(1 for i in range(n) if int(brc[i]) == 0 and bo[i] == src[i * vlen:(i + 1) * vlen])
    print(f"stop={os.environ['PMC_DIAG_INFLATE_STOP']} vlen={vlen} compress_rc!=0={int((rc != 0).sum())} "
          f"inflate rc: {dict(zip(vals.tolist(), cnt.tolist()))} rc==0 and bytes equal: {same}", flush=True)
ctx.close()
