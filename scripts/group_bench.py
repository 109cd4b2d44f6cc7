"""Host-to-host rate of the single-process multi-GPU dispatcher (pmc_group_*).

The reference server is one process routing key k to shard hashFunc(k) % NUM_SHARDS
(server.cpp:113,121,132); a pmc_group sends shard s to member s % n, runs each member's share through
its own context's pinned pipelined call on a host thread of its own, and gathers / scatters between the
caller's (unpinned) host buffers and the members' pinned staging on several host threads.  On the
one-GPU box the members are contexts on device 0 (what n GPUs would do, sharing one card).

Workload: N x V-byte JSON-slice values (SURVEY §8d generator on the device, copied to host memory),
keys "key"+i.  Times one group compress and one group decompress (host wall clock, best of 3) for 1 and
2 members, and checks the round trip.
usage: python scripts/group_bench.py [--n 1000000] [--vlen 1024] > profiles/r03/group.json
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pmc_codec  # noqa: E402
from pmc_codec import device as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--vlen", type=int, default=1024)
    ap.add_argument("--members", default="1,2")
    args = ap.parse_args()
    n, vlen = args.n, args.vlen
    L = pmc_codec.lib()
    d = os.path.join(ROOT, "tests", "golden", "data")
    corpus_b = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))
    corpus = torch.frombuffer(bytearray(corpus_b), dtype=torch.uint8).cuda()
    dev = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
    assert L.pmc_gen_values(corpus.data_ptr(), len(corpus_b), 0x5EED, 0, 0, None, n, vlen, dev.data_ptr(),
                            D.stream_handle()) == 0
    src = dev.cpu().numpy()
    del dev
    soff = np.arange(n, dtype=np.uint64) * np.uint64(vlen)
    slen = np.full(n, vlen, dtype=np.uint32)
    cap = np.full(n, pmc_codec.gzip_bound(vlen), dtype=np.uint32)
    doff = np.arange(n, dtype=np.uint64) * np.uint64(int(cap[0]))
    kh = np.array([L.pmc_key_hash(b"key%d" % i, len(b"key%d" % i)) for i in range(n)], dtype=np.uint64)
    gib = n * vlen / 2 ** 30
    out = {"note": __doc__.split("\n\n")[1].replace("\n", " "), "n": n, "vlen": vlen, "rows": []}
    for m in [int(x) for x in args.members.split(",")]:
        g = ctypes.c_void_p()
        devs = (ctypes.c_int * m)(*([0] * m))
        assert L.pmc_group_create(devs, m, ctypes.byref(g)) == 0
        comp = np.zeros(int(doff[-1]) + int(cap[0]) + 64, dtype=np.uint8)
        clen = np.zeros(n, dtype=np.uint32)
        crc = np.zeros(n, dtype=np.int32)
        back = np.zeros(n * vlen + 64, dtype=np.uint8)
        blen = np.zeros(n, dtype=np.uint32)
        brc = np.zeros(n, dtype=np.int32)
        tc, td = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            assert L.pmc_group_compress_batch(g, src.ctypes.data, soff.ctypes.data, slen.ctypes.data, kh.ctypes.data,
                                              128, n, comp.ctypes.data, doff.ctypes.data, cap.ctypes.data,
                                              clen.ctypes.data, crc.ctypes.data, vlen) == 0
            t1 = time.perf_counter()
            assert L.pmc_group_decompress_batch(g, comp.ctypes.data, doff.ctypes.data, clen.ctypes.data,
                                                kh.ctypes.data, 128, n, back.ctypes.data, soff.ctypes.data,
                                                slen.ctypes.data, blen.ctypes.data, brc.ctypes.data, vlen) == 0
            t2 = time.perf_counter()
            tc.append(t1 - t0)
            td.append(t2 - t1)
        L.pmc_group_destroy(g)
        bad = int((crc != 0).sum()) + int((brc != 0).sum()) + int((blen != slen).sum())
        bad += int(not np.array_equal(back[:n * vlen], src[:n * vlen]))
        row = {"members": m, "devices": [0] * m, "compress_gib_s": gib / min(tc), "decompress_gib_s": gib / min(td),
               "roundtrip_gib_s": gib / (min(tc) + min(td)), "compressed_bytes": int(clen.sum()), "mismatches": bad}
        out["rows"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
