"""GPU: byte parity at scale, through the multi-chunk compress path.

tests/golden/full_digests.json holds, per BASELINE workload, SHA-256 digests of the reference's
(member length, member CRC-32) records for value prefixes up to 10M (tests/golden/make_full_digests.py,
the reference's own Compress).  Here the device generates the same values (SURVEY.md §8d generator),
compresses them with the chunk scratch budget (PMC_SPLIT_CHUNK_MB) forced small enough that the batch
runs as >= 3 front/trees/back launch sets with their work counters, and the records of every member
must hash to the reference's digest; then every member must decompress back to its value.  The C-ABI
reads PMC_SPLIT_CHUNK_MB once per process, so each case runs in a child process.
"""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

CHILD = r"""
import hashlib, json, sys
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import numpy as np, torch
import pmc_codec
n, vlen, kind, seed, want = int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]), sys.argv[7]
L = pmc_codec.lib()
ctx = pmc_codec.Context(0)
sh = torch.cuda.current_stream().cuda_stream
d = sys.argv[2] + "/tests/golden/data"
import os
corpus_b = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))
corpus = torch.frombuffer(bytearray(corpus_b), dtype=torch.uint8).cuda()
src = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
assert L.pmc_gen_values(corpus.data_ptr(), len(corpus_b), seed, kind, 0, None, n, vlen, src.data_ptr(), sh) == 0
off = torch.arange(n, dtype=torch.int64, device="cuda") * vlen
lens = torch.full((n,), vlen, dtype=torch.int32, device="cuda")
cap = pmc_codec.gzip_bound(vlen)
stride = (cap + 15) // 16 * 16
comp = torch.empty(n * stride + 16, dtype=torch.uint8, device="cuda")
coff = torch.arange(n, dtype=torch.int64, device="cuda") * stride
ccap = torch.full((n,), cap, dtype=torch.int32, device="cuda")
clen = torch.zeros(n, dtype=torch.int32, device="cuda")
rc = torch.full((n,), 7, dtype=torch.int32, device="cuda")
ctx.profile(True)
ctx.compress_device(src, off, lens, comp, coff, ccap, clen, rc, vlen, sh)
kt = ctx.kernel_times()
ctx.profile(False)
launches = kt["deflate_front"][1]
mcrc = torch.zeros(n, dtype=torch.int32, device="cuda")
assert L.pmc_crc32_batch(ctx.handle, comp.data_ptr(), coff.data_ptr(), clen.data_ptr(), n, mcrc.data_ptr(), sh) == 0
back = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
blen = torch.zeros(n, dtype=torch.int32, device="cuda")
brc = torch.full((n,), 7, dtype=torch.int32, device="cuda")
ctx.decompress_device(comp, coff, clen, back, off, lens, blen, brc, vlen, sh)
mism = torch.zeros(1, dtype=torch.int32, device="cuda")
assert L.pmc_compare_values(src.data_ptr(), off.data_ptr(), back.data_ptr(), off.data_ptr(), lens.data_ptr(),
                            blen.data_ptr(), n, mism.data_ptr(), sh) == 0
torch.cuda.synchronize()
rec = torch.stack([clen, mcrc], dim=1).cpu().numpy().astype("<u4")
got = hashlib.sha256(rec.tobytes()).hexdigest()
res = {"launches": launches, "rc_bad": int((rc != 0).sum()), "brc_bad": int((brc != 0).sum()),
       "mismatches": int(mism.item()), "digest_ok": got == want}
print(json.dumps(res))
ctx.close()
"""


def _digest(n, vlen, kind):
    with open(os.path.join(HERE, "golden", "full_digests.json")) as f:
        doc = json.load(f)
    for st in doc["sets"]:
        if st["vlen"] == vlen and st["kind"] == kind:
            return st["seed"], st["prefixes"][str(n)]["sha256"]
    raise KeyError((n, vlen, kind))


def test_full_digests_cover_the_bench_workloads():
    """CPU: the committed digests exist for bench.py's default workload and the other BASELINE sizes."""
    for n, vlen, kind in ((10_000_000, 1024, 0), (10_000_000, 256, 0), (1_000_000, 4096, 0), (200_000, 1024, 0)):
        seed, h = _digest(n, vlen, kind)
        assert len(h) == 64 and seed == 0x5EED


# (values, value bytes, kind, chunk budget MiB): split_value_bytes(cap) is ~7.4 KB per 1 KiB value,
# ~4.3 KB per 256 B value and ~20 KB per 4 KiB value, so each budget cuts the batch into >= 3 chunks
@pytest.mark.gpu
@pytest.mark.parametrize("n,vlen,kind,chunk_mb", [(200_000, 1024, 0, 400), (200_000, 256, 0, 200),
                                                  (200_000, 4096, 0, 1000), (1_000_000, 1024, 1, 1500),
                                                  (200_000, 1024, 0, 16384)])
def test_multichunk_compress_matches_reference_digest(n, vlen, kind, chunk_mb):
    seed, want = _digest(n, vlen, kind)
    env = dict(os.environ, PMC_SPLIT_CHUNK_MB=str(chunk_mb))
    out = subprocess.run([sys.executable, "-c", CHILD,
                          os.path.join(ROOT, "poor-man-s-cache_amd"), ROOT, str(n), str(vlen), str(kind), str(seed),
                          want], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    if chunk_mb < 16384:
        assert res["launches"] >= 3, res
    assert res["rc_bad"] == 0 and res["brc_bad"] == 0 and res["mismatches"] == 0, res
    assert res["digest_ok"], res
