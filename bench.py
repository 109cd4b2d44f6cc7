#!/usr/bin/env python
"""bench.py -- device-resident gzip-9 compress+decompress throughput on MI355X.

Metric (BASELINE.json): "device-resident value compress+decompress GiB/s at 1/2/4/8 MI355X".
One step = compress every value of this rank's batch, then decompress every member back,
inputs already resident in HBM.  value = (all ranks' uncompressed bytes) / (max over ranks
of the step time), in GiB/s.  Workload (north star / BASELINE configs[3] per GPU):
10M x 1 KiB JSON-slice values per GPU, routed to GPUs by MurmurHash3("key"+i) % 128 % N
(NUM_SHARDS=128 as deployed) -- weak scaling, no collective on the data path.

Single GPU:  python bench.py [--steps K --warmup W]
Multi GPU :  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "poor-man-s-cache_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "device-resident value compress+decompress GiB/s at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
META_BYTES = 12        # +12 B offset/len per value per direction


NUM_SHARDS = 128       # .env:4 as deployed; server.cpp:113 routes hash % NUM_SHARDS


def route_span(n, world):
    """Keys "key"+0 .. span-1 are routed; every rank finds >= n of its own among them."""
    return int(n * world * 1.05) + 4096


def select_rank_keys(route, rank, n):
    """Global indices of the first n keys whose routed GPU (route[i], any torch device) is
    `rank` -- the rank's weak-scaling share of the key space."""
    import torch
    idx = torch.nonzero(route == rank).flatten()[:n].to(torch.int64).contiguous()
    if idx.numel() != n:
        raise RuntimeError(f"rank {rank}: only {idx.numel()} of {n} keys routed in the span")
    return idx


def landing_keys(route, world, n):
    """bench.py --landing scatter: the batch that lands on one GPU holds every rank's keys (the first n routed to
    each rank, select_rank_keys), in key order."""
    import torch
    return torch.sort(torch.cat([select_rank_keys(route, r, n) for r in range(world)])).values


def reduce_over_ranks(times, sums, world, device):
    """Max over ranks of the step times, sum over ranks of the byte / error counters."""
    import torch
    t = torch.tensor(times, dtype=torch.float64, device=device)
    a = torch.tensor(sums, dtype=torch.float64, device=device)
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(a, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.tolist()], [float(x) for x in a.tolist()]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=10_000_000, help="values per GPU")
    ap.add_argument("--vlen", type=int, default=1024)
    ap.add_argument("--kind", type=int, default=0, help="0 JSON slices, 1 random alnum")
    ap.add_argument("--cpu-sample", type=int, default=300_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--h2h", action="store_true", help="also time pinned H2D+kernel+D2H (host-to-host)")
    ap.add_argument("--h2h-chunk", type=int, default=0, help="values per chunk of the pipelined h2h leg (0 = n/16)")
    ap.add_argument("--mix", action="store_true",
                    help="BASELINE configs[2]: SET/GET mix over a device-resident compressed store instead")
    ap.add_argument("--batch-vlen", type=int, default=4096, help="--batches: value bytes (default 4 KiB)")
    ap.add_argument("--batches", action="store_true",
                    help="server-shaped batches (256 / 1,024 / 4,096 / 400 values, default 4 KiB): ms per batch")
    ap.add_argument("--mix-keys", type=int, default=1_000_000)
    ap.add_argument("--emulate", default="", metavar="RANK/WORLD",
                    help="one GPU runs rank RANK's share of a WORLD-GPU run (its routed keys, checked against that "
                         "rank's reference digests): rehearses the N > 1 parity path on a one-GPU box")
    ap.add_argument("--landing", choices=["host", "scatter"], default="host",
                    help="scatter: the whole batch lands in rank 0's HBM and is scattered to its owner GPUs by one "
                         "RCCL all-to-all before the timed steps (SURVEY §8e); host (default): each rank generates "
                         "its own share, no collective")
    ap.add_argument("--mix-serial", action="store_true", help="SETs and GETs of a batch on one stream")
    ap.add_argument("--mix-ops", type=int, default=1_048_576)
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r06", "traffic.json"),
                    help="PMC-derived HBM bytes and issue counters per launch (scripts/pmc_traffic.py); used "
                         "only if its source_id matches the library's sources")
    ap.add_argument("--cpu-threads", type=int, default=0, help="threads of the all-core CPU baseline "
                    "(0 = every core this process may run on)")
    return ap.parse_args()


def load_corpus():
    d = os.path.join(ROOT, "tests", "golden", "data")
    return b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))


def fullsize_parity(L, ctx, comp, coff, clen, n, vlen, kind, world, rank, sh):
    """Parity of ALL n members of this rank's run with the reference (tests/golden/full_digests.json at
    N = 1, tests/golden/rank_digests.json for rank r of N = 2/4/8; both made by
    tests/golden/make_full_digests.py from the reference's own Compress): the device takes the CRC-32 of
    every member (pmc_crc32_batch), the host hashes the (u32 length, u32 CRC-32) records with SHA-256.
    That is a length + CRC-32 digest of the bytes, not a byte comparison.  Returns {"match": bool, ...},
    or None when no digest covers this workload."""
    import hashlib
    import torch
    fname = "full_digests.json" if world == 1 else "rank_digests.json"
    try:
        with open(os.path.join(ROOT, "tests", "golden", fname)) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None
    want = None
    for st in doc["sets"]:
        if (st["vlen"] == vlen and st["kind"] == kind and str(n) in st["prefixes"]
                and (world == 1 or (st.get("world") == world and st.get("rank") == rank))):
            want = st["prefixes"][str(n)]
    if want is None:
        return None
    mcrc = torch.zeros(n, dtype=torch.int32, device=comp.device)
    assert L.pmc_crc32_batch(ctx.handle, comp.data_ptr(), coff.data_ptr(), clen.data_ptr(), n, mcrc.data_ptr(),
                             sh) == 0
    rec = torch.stack([clen, mcrc], dim=1).cpu().numpy().astype("<u4")
    got = hashlib.sha256(rec.tobytes()).hexdigest()
    out = {"match": got == want["sha256"], "members": n, "sha256": got,
           "method": "sha256 over the (u32 len, u32 CRC-32) record of every member, vs the reference's "
                     "(a length + CRC-32 digest of the member bytes, not a byte-by-byte comparison; the "
                     "byte-by-byte comparisons are the goldens, tests/test_gpu_codec.py)"}
    if "bytes_sha256" in want:  # every member's bytes: compacted on the device, hashed on the host
        t0 = time.perf_counter()
        hb = hashlib.sha256()
        stride = int(coff[1].item() - coff[0].item()) if n > 1 else int(clen[0].item())
        if n > 1 and not bool((coff[1:] - coff[:-1] == stride).all()):
            raise RuntimeError("members are not at a fixed stride")
        rows = comp[int(coff[0].item()):int(coff[0].item()) + n * stride].view(n, stride)
        col = torch.arange(stride, device=comp.device)[None, :]
        for a in range(0, n, 1 << 20):
            b = min(n, a + (1 << 20))
            hb.update(rows[a:b][col < clen[a:b, None]].cpu().numpy().tobytes())
        gotb = hb.hexdigest()
        out.update(match=out["match"] and gotb == want["bytes_sha256"], bytes_sha256=gotb,
                   bytes_match=gotb == want["bytes_sha256"], bytes_s=round(time.perf_counter() - t0, 2),
                   method="sha256 over every member's BYTES back to back, and over the (u32 len, u32 CRC-32) "
                          "records, each vs the reference's own Compress of the same values: a byte-by-byte "
                          "check of every member")
    return {**out,
            "reference": f"tests/golden/{fname} (reference GzipCompressor::Compress, zlib "
                         f"{doc.get('zlib_version')})"}


def cpu_baseline(corpus, args, index0):
    """The reference GzipCompressor timed on the host cores (oracle/_ref), or the oracle
    port if the reference build is absent.  Bounded sample of the same workload."""
    from oracle import pyoracle as O
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    quota = None  # a cgroup CPU quota caps what the threads can get (cpu.max: "<quota> <period>")
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        quota = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    # one thread per CPU this process may use: the affinity set, capped by the cgroup quota (the GPU
    # box runs each GPU's job in a 16-CPU share of a 2 x 64-core host; more threads would only
    # time-slice the same share)
    cores = args.cpu_threads or max(1, min(cores, int(quota) if quota else cores))
    seed = 0x5EED if args.kind == 0 else 0xA1B2
    n = args.cpu_sample
    vals = O.gen_values(corpus, seed, args.kind, index0, n, args.vlen)
    single = None
    if O.ref_available():
        r = O.ref_bench(vals, cores)
        assert r["bad"] == 0
        t = r["t_compress"] + r["t_decompress"]
        kind, zv = "reference", O.ref().ref_zlib_version().decode()
        # one core, the server's single request-handler thread (server.cpp:631-643)
        n1 = min(n, 30_000)
        r1 = O.ref_bench(vals[:n1], 1)
        assert r1["bad"] == 0
        g1 = n1 * args.vlen / 2 ** 30
        single = {"value": g1 / (r1["t_compress"] + r1["t_decompress"]), "cores": 1,
                  "compress_gib_s": g1 / r1["t_compress"], "decompress_gib_s": g1 / r1["t_decompress"],
                  "sample": f"{n1} x {args.vlen} B values (indices {index0}..{index0 + n1 - 1})"}
    else:
        import time as _t
        n = min(n, 20_000)
        t0 = _t.perf_counter()
        gz = [O.compress(vals[k].tobytes()) for k in range(n)]
        t1 = _t.perf_counter()
        for g in gz:
            O.decompress(g)
        t = _t.perf_counter() - t0
        cores, kind, zv = 1, "port", "oracle restatement of zlib 1.2.11"
        r = {"t_compress": t1 - t0, "t_decompress": t - (t1 - t0)}
    gib = n * args.vlen / 2 ** 30
    cpu = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    host_cores = None  # physical cores of the host (lscpu's Core(s) per socket x Socket(s))
    try:
        phys = set()
        with open("/proc/cpuinfo") as f:
            pid = core = None
            for line in f:
                if line.startswith("physical id"):
                    pid = line.split(":")[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":")[1].strip()
                    phys.add((pid, core))
        host_cores = len(phys) or None
    except OSError:
        pass
    all_core = None
    if single and host_cores:
        # linear upper bound: every physical core of the host running the reference at the one-core rate
        all_core = {"value": single["value"] * host_cores, "cores": host_cores,
                    "note": "estimate = single-core rate x physical cores (no shared-resource losses); the "
                            "measured figure above is what the job's CPU share delivers"}
    return {"value": gib / t, "unit": "GiB/s", "cores": cores, "kind": kind, "cgroup_cpu_quota": quota,
            "host_physical_cores": host_cores, "all_host_cores_estimate": all_core,
            "sample": f"{n} x {args.vlen} B values of the same workload (indices {index0}..{index0 + n - 1}), "
                      f"one GzipCompressor::Compress then Decompress per value, {cores} std::threads",
            "compress_gib_s": gib / r["t_compress"], "decompress_gib_s": gib / r["t_decompress"],
            "cpu": cpu, "zlib": zv, "single_core": single}


def mix_bench(args):
    """BASELINE.json configs[2] / SURVEY.md §8d cfg 3: 1M x 4 KiB JSON-slice values, batches of 65,536
    ops, 50 % SET (compress a fresh value into the key's slot of a device-resident compressed store)
    and 50 % GET (decompress a previously stored value), seed 7.

    The store is the library's fixed-slot device slab (pmc_slab_*: pmc_gzip_bound(vlen) bytes per key
    plus a length per key, SURVEY §8f2's device-resident store).  Per batch, a random permutation of the key space
    gives 32,768 SET keys and 32,768 disjoint GET keys, so op order inside a batch cannot change any
    GET's answer.  The store is prefilled (untimed) with value index k for key k; SET j of batch b
    stores fresh value index K + b*32768 + j.  Every GET is verified afterwards against the value
    its key held (device-side compare against regenerated values)."""
    import torch

    import pmc_codec

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    L = pmc_codec.lib()
    ctx = pmc_codec.Context(0)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    corpus_b = load_corpus()
    corpus = torch.frombuffer(bytearray(corpus_b), dtype=torch.uint8).to(dev)
    K, vlen, seed, bsz = args.mix_keys, args.vlen, 0x5EED, 65536
    half = bsz // 2
    nb = args.mix_ops // bsz
    cap = pmc_codec.gzip_bound(vlen)

    def gen(index, n, dst):
        assert L.pmc_gen_values(corpus.data_ptr(), len(corpus_b), seed, 0, 0, index.data_ptr(), n, vlen,
                                dst.data_ptr(), sh) == 0

    # ---- prefill the store: key k holds value index k ----------------------------------------
    slab = pmc_codec.Slab(ctx, K, vlen)
    ver = torch.arange(K, dtype=torch.int64, device=dev)
    src = torch.empty(K * vlen + 16, dtype=torch.uint8, device=dev)
    gen(ver, K, src)
    rc = torch.zeros(K, dtype=torch.int32, device=dev)
    slab.set(src, torch.arange(K, dtype=torch.int64, device=dev) * vlen,
             torch.full((K,), vlen, dtype=torch.int32, device=dev), torch.arange(K, dtype=torch.int32, device=dev), rc,
             sh)
    torch.cuda.synchronize()
    assert int((rc != 0).sum()) == 0
    del src

    # ---- per-batch inputs (untimed): keys, fresh SET values ---------------------------------
    g = torch.Generator(device="cpu").manual_seed(7)
    perms = [torch.randperm(K, generator=g)[:bsz].to(dev).to(torch.int32) for _ in range(nb)]
    set_keys = [p[:half].contiguous() for p in perms]
    get_keys = [p[half:].contiguous() for p in perms]
    set_idx = [K + b * half + torch.arange(half, dtype=torch.int64, device=dev) for b in range(nb)]
    set_vals = torch.empty(nb * half * vlen + 16, dtype=torch.uint8, device=dev)
    for b in range(nb):
        gen(set_idx[b], half, set_vals[b * half * vlen:])
    v_off = torch.arange(half, dtype=torch.int64, device=dev) * vlen
    v_len = torch.full((half,), vlen, dtype=torch.int32, device=dev)
    s_rc = torch.zeros(nb, half, dtype=torch.int32, device=dev)
    outs = torch.empty(nb * half * vlen + 16, dtype=torch.uint8, device=dev)
    o_len = torch.zeros(nb, half, dtype=torch.int32, device=dev)
    g_rc = torch.zeros(nb, half, dtype=torch.int32, device=dev)
    g_ver = torch.zeros(nb, half, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    # SETs of batch b run on stream A and its GETs on stream B: their keys are disjoint, so they may
    # overlap (the GETs fill the CUs the front kernel's tail leaves idle).  B_b waits for A_(b-1)
    # (a GET sees every earlier batch's SETs); A_(b+1) waits for B_b (no SET overwrites a slot a
    # GET of an earlier batch still reads).  --mix-serial runs both on one stream.
    sA = stream
    sB = torch.cuda.Stream() if not args.mix_serial else stream
    evA = [torch.cuda.Event() for _ in range(nb)]
    evB = [torch.cuda.Event() for _ in range(nb)]

    def batch(b):
        sk, gk = set_keys[b], get_keys[b]
        if b > 0:
            sA.wait_event(evB[b - 1])
        with torch.cuda.stream(sA):
            # SET: compress the fresh values straight into their keys' slab slots
            slab.set(set_vals[b * half * vlen:], v_off, v_len, sk, s_rc[b], sA.cuda_stream)
            ver[sk.long()] = set_idx[b]
            evA[b].record(sA)
        if b > 0:
            sB.wait_event(evA[b - 1])
        with torch.cuda.stream(sB):
            # GET: decompress the stored members of the GET keys
            g_ver[b] = ver[gk.long()]
            slab.get(gk, outs[b * half * vlen:], v_off, v_len, o_len[b], g_rc[b], sB.cuda_stream)
            evB[b].record(sB)

    # warm-up GET (untimed): sizes the decompress scratch; its outputs are overwritten by batch 0
    slab.get(get_keys[0], outs, v_off, v_len, o_len[0], g_rc[0], sh)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    sB.wait_event(e0)
    for b in range(nb):
        batch(b)
    sA.wait_event(evB[nb - 1])
    e1.record(stream)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3

    # ---- verify every GET against the value its key held --------------------------------------
    bad = int((s_rc != 0).sum()) + int((g_rc != 0).sum()) + int((o_len != vlen).sum())
    want = torch.empty(half * vlen + 16, dtype=torch.uint8, device=dev)
    mism = torch.zeros(1, dtype=torch.int32, device=dev)
    for b in range(nb):
        gen(g_ver[b].contiguous(), half, want)
        assert L.pmc_compare_values(want.data_ptr(), v_off.data_ptr(), outs[b * half * vlen:].data_ptr(),
                                    v_off.data_ptr(), v_len.data_ptr(), o_len[b].data_ptr(), half,
                                    mism.data_ptr(), sh) == 0
    torch.cuda.synchronize()
    bad += int(mism.item())
    ops = nb * bsz
    gib = ops * vlen / 2 ** 30
    print(json.dumps({
        "metric": "SET/GET mix throughput over a device-resident compressed store (BASELINE configs[2])",
        "value": gib / t, "unit": "GiB/s", "ops_per_s": ops / t, "n_gpus": 1, "ops": ops, "batches": nb,
        "ms_per_batch": t / nb * 1e3, "higher_is_better": True, "dtype": "u8",
        "data": f"synthetic: JSON slices of the reference's tests/data corpus (seed {seed:#x}), keys seed 7",
        "config": {"workload": f"{K} keys x {vlen} B values, batches of {bsz} ops: 50% SET (compress into the "
                               "key's slot of the device slab, pmc_slab_set) / 50% GET (pmc_slab_get), disjoint "
                               "keys per batch",
                   "keys": K, "value_bytes": vlen, "batch_ops": bsz,
                   "streams": 1 if args.mix_serial else 2},
        "mismatches": bad}), flush=True)
    slab.close()
    ctx.close()


def batch_bench(args):
    """Server-shaped batches (BASELINE configs[4]): what one epoll iteration of a
    batched server hands the codec.  Batches of 256 / 1,024 / 4,096 JSON-slice values (default 4 KiB), timed
    per batch: device-resident (pmc_gzip_*_batch, HIP events around each call on its stream) and host-resident
    (pmc_gzip_*_batch_host: pinned staging, H2D, kernels, D2H, host wall clock), compress and decompress
    separately, every member checked against the value it came from."""
    import numpy as np
    import torch

    import pmc_codec
    from pmc_codec import device as D

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    L = pmc_codec.lib()
    ctx = pmc_codec.Context(0)
    sh = torch.cuda.current_stream().cuda_stream
    corpus_b = load_corpus()
    vlen, reps = args.vlen, 20
    out = []
    corpus = torch.frombuffer(bytearray(corpus_b), dtype=torch.uint8).to(dev)
    for n in (1, 16, 64, 256, 1024, 4096, 400):
        raw = torch.empty(n * vlen + 16, dtype=torch.uint8, device=dev)
        assert L.pmc_gen_values(corpus.data_ptr(), len(corpus_b), 0x5EED, 0, 0, None, n, vlen, raw.data_ptr(), sh) == 0
        rh = raw.cpu().numpy().tobytes()
        vals = [rh[i * vlen:(i + 1) * vlen] for i in range(n)]
        b = D.pack(vals, dev)
        D.compress(ctx, b)  # (untimed: sizes the scratch)
        torch.cuda.synchronize()
        # (each call timed by events around it on the stream; output slots allocated outside)
        tc = []
        for r in range(reps):
            caps = [pmc_codec.gzip_bound(vlen)] * n
            dst, doff, dcap = D.slots_for(caps, dev)
            dlen = torch.zeros(n, dtype=torch.int32, device=dev)
            rcc = torch.zeros(n, dtype=torch.int32, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ctx.compress_device(b.data, b.off, b.len, dst, doff, dcap, dlen, rcc, vlen, sh)
            e1.record()
            torch.cuda.synchronize()
            tc.append(e0.elapsed_time(e1))
        comp = D.Batch(dst, doff, dlen, n, int(max(caps)))
        assert int((rcc != 0).sum()) == 0
        members = comp.host_items()
        D.decompress(ctx, comp, [vlen] * n)
        torch.cuda.synchronize()
        td = []
        for r in range(reps):
            back_dst, boff, bcap = D.slots_for([vlen] * n, dev)
            blen = torch.zeros(n, dtype=torch.int32, device=dev)
            brc = torch.zeros(n, dtype=torch.int32, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ctx.decompress_device(comp.data, comp.off, comp.len, back_dst, boff, bcap, blen, brc, vlen, sh)
            e1.record()
            torch.cuda.synchronize()
            td.append(e0.elapsed_time(e1))
        back = D.Batch(back_dst, boff, blen, n, vlen).host_items()
        bad = int((brc != 0).sum()) + sum(1 for v, w in zip(vals, back) if v != w)
        # host-resident batches through the C-ABI alone (what the server's C++ hook calls: caller arrays
        # prepared once, pmc_gzip_*_batch_host timed), wall clock
        import ctypes
        hsrc = b"".join(vals)
        hoff = np.arange(n, dtype=np.uint64) * vlen
        hlen = np.full(n, vlen, dtype=np.uint32)
        hcap = np.full(n, pmc_codec.gzip_bound(vlen), dtype=np.uint32)
        hdoff = np.concatenate([[0], np.cumsum(hcap[:-1], dtype=np.uint64)]).astype(np.uint64)
        hdst = np.empty(int(hcap.sum()) + 16, dtype=np.uint8)
        hdlen = np.zeros(n, dtype=np.uint32)
        hrc = np.zeros(n, dtype=np.int32)
        p = lambda a: a.ctypes.data  # noqa: E731
        ac, ad = [], []
        for r in range(reps):
            t0 = time.perf_counter()
            assert L.pmc_gzip_compress_batch_host(ctx.handle, hsrc, p(hoff), p(hlen), n, p(hdst), p(hdoff), p(hcap),
                                                  p(hdlen), p(hrc)) == 0
            ac.append((time.perf_counter() - t0) * 1e3)
        bad += int((hrc != 0).sum()) + sum(1 for i in range(n) if hdst[hdoff[i]:hdoff[i] + hdlen[i]].tobytes()
                                           != members[i])
        msrc = hdst.tobytes()
        mlen = hdlen.copy()
        bdst = np.empty(n * vlen + 16, dtype=np.uint8)
        for r in range(reps):
            t0 = time.perf_counter()
            assert L.pmc_gzip_decompress_batch_host(ctx.handle, msrc, p(hdoff), p(mlen), n, p(bdst), p(hoff), p(hlen),
                                                    p(hdlen), p(hrc)) == 0
            ad.append((time.perf_counter() - t0) * 1e3)
        bad += int((hrc != 0).sum()) + int(bdst[:n * vlen].tobytes() != hsrc)
        # host-resident batches through the Python mirror (list of bytes in and out), wall clock
        hc, hd = [], []
        for r in range(reps):
            t0 = time.perf_counter()
            res = ctx.compress_many(vals)
            hc.append((time.perf_counter() - t0) * 1e3)
        hm = [g for _, g in res]
        bad += sum(1 for (r_, g), m in zip(res, members) if r_ != 0 or g != m)
        for r in range(reps):
            t0 = time.perf_counter()
            resd = ctx.decompress_many(hm, [vlen] * n)
            hd.append((time.perf_counter() - t0) * 1e3)
        bad += sum(1 for (r_, v2), v in zip(resd, vals) if r_ != 0 or v2 != v)
        med = lambda x: float(np.median(x))
        out.append({"values": n, "value_bytes": vlen,
                    "device_ms": {"compress": med(tc), "decompress": med(td)},
                    "host_abi_ms": {"compress": med(ac), "decompress": med(ad)},
                    "host_ms": {"compress": med(hc), "decompress": med(hd)},
                    "mismatches": bad})
        print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"metric": "server-shaped batch latency (ms per batch, median of 20)", "unit": "ms",
                      "higher_is_better": False, "dtype": "u8", "data": "synthetic: JSON slices of the "
                      "reference's tests/data corpus (seed 0x5EED)", "batches": out}), flush=True)
    ctx.close()


def main():
    args = parse()
    if args.batches:
        args.vlen = args.batch_vlen
        return batch_bench(args)
    if args.mix:
        if args.vlen == 1024:
            args.vlen = 4096
        return mix_bench(args)
    import numpy as np
    import torch
    import torch.distributed as dist

    import pmc_codec
    from pmc_codec import device as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.landing == "scatter" and world == 1 and "MASTER_ADDR" not in os.environ:
        import socket
        with socket.socket() as so:  # a one-rank RCCL group, so the scatter's collectives run as at N > 1
            so.bind(("127.0.0.1", 0))
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(so.getsockname()[1]), RANK="0", WORLD_SIZE="1")
    distributed = world > 1 or args.landing == "scatter"
    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local)
    L = pmc_codec.lib()
    corpus_b = load_corpus()
    n, vlen = args.n, args.vlen
    if args.kind == 0 and vlen > len(corpus_b):  # values longer than the 82 KB corpus: slices of it tiled
        corpus_b = corpus_b * (vlen // len(corpus_b) + 2)
    seed = 0x5EED if args.kind == 0 else 0xA1B2

    # ---- CPU baseline first (host idle), rank 0 at N=1 only ------------------------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(corpus_b, args, 0)

    ctx = pmc_codec.Context(local)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    # ---- this rank's keys: route "key"+i to GPUs, take the first n routed here -----------
    landing = None
    sel_rank, sel_world = (int(x) for x in args.emulate.split("/")) if args.emulate else (rank, world)
    if args.emulate and (world > 1 or args.landing == "scatter" or not 0 <= sel_rank < sel_world):
        raise SystemExit("--emulate RANK/WORLD: one process, default landing, 0 <= RANK < WORLD")
    if sel_world > 1 or args.landing == "scatter":
        span = route_span(n, sel_world)
        route = torch.empty(span, dtype=torch.uint8, device=dev)
        assert L.pmc_route_keys(0, span, NUM_SHARDS, sel_world, route.data_ptr(), sh) == 0
        index = select_rank_keys(route, sel_rank, n)
        idx_ptr = index.data_ptr()
    else:
        index, idx_ptr = None, None
    corpus = torch.frombuffer(bytearray(corpus_b), dtype=torch.uint8).to(dev)
    src = torch.empty(n * vlen + 16, dtype=torch.uint8, device=dev)
    if args.landing == "scatter":
        landing = scatter_landing(L, args, route, corpus, len(corpus_b), seed, world, rank, n, vlen, dev, sh)
        src[:n * vlen].copy_(landing.pop("rows").view(-1))
        landing["tags_match"] = bool(torch.equal(landing.pop("tags"), index))
        if not landing["tags_match"]:
            raise RuntimeError(f"rank {rank}: the scattered keys are not the ones this rank owns")
    else:
        assert L.pmc_gen_values(corpus.data_ptr(), len(corpus_b), seed, args.kind, 0, idx_ptr, n, vlen,
                                src.data_ptr(), sh) == 0
    if index is not None:
        del route
    off = torch.arange(n, dtype=torch.int64, device=dev) * vlen
    lens = torch.full((n,), vlen, dtype=torch.int32, device=dev)
    cap = pmc_codec.gzip_bound(vlen)
    cstride = (cap + 15) // 16 * 16
    comp = torch.empty(n * cstride + 16, dtype=torch.uint8, device=dev)
    coff = torch.arange(n, dtype=torch.int64, device=dev) * cstride
    ccap = torch.full((n,), cap, dtype=torch.int32, device=dev)
    clen = torch.zeros(n, dtype=torch.int32, device=dev)
    crc = torch.zeros(n, dtype=torch.int32, device=dev)
    back = torch.empty(n * vlen + 16, dtype=torch.uint8, device=dev)
    blen = torch.zeros(n, dtype=torch.int32, device=dev)
    brc = torch.zeros(n, dtype=torch.int32, device=dev)
    del index

    def step(evs=None):
        if evs:
            evs[0].record(stream)
        ctx.compress_device(src, off, lens, comp, coff, ccap, clen, crc, vlen, sh)
        if evs:
            evs[1].record(stream)
        ctx.decompress_device(comp, coff, clen, back, off, lens, blen, brc, vlen, sh)
        if evs:
            evs[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    tc = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps / 1e3  # s per compress launch set
    td = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps / 1e3

    # ---- verification of the last step (device-side compare, all values) ----------------
    mism = torch.zeros(1, dtype=torch.int32, device=dev)
    assert L.pmc_compare_values(src.data_ptr(), off.data_ptr(), back.data_ptr(), off.data_ptr(), lens.data_ptr(),
                                blen.data_ptr(), n, mism.data_ptr(), sh) == 0
    torch.cuda.synchronize()
    bad = int(mism.item()) + int((crc != 0).sum().item()) + int((brc != 0).sum().item())
    comp_bytes = int(clen.to(torch.int64).sum().item())
    parity = fullsize_parity(L, ctx, comp, coff, clen, n, vlen, args.kind, sel_world, sel_rank, sh)
    if args.emulate and parity is not None:
        parity["emulated"] = f"rank {sel_rank} of {sel_world}"

    (t_step_s, tc_max, td_max), (total_bytes, total_comp, total_bad, p_match, p_checked) = reduce_over_ranks(
        [wall / args.steps, tc, td], [float(n * vlen), float(comp_bytes), float(bad),
                                      float(bool(parity and parity["match"])), float(parity is not None)],
        world, dev)
    if world > 1 and parity is not None:  # every rank against its own digest
        parity = {"match": p_match == world and p_checked == world, "ranks_checked": int(p_checked),
                  "ranks_matching": int(p_match), "members": n * world, "method": parity["method"],
                  "reference": parity["reference"]}

    # ---- lane-order guards (DESIGN §4 Guards): over the run, no value may have been rerouted -------
    guards = ctx.guard_counts()

    # ---- per-kernel launch times of one more step (HIP events around every launch) -----------
    ctx.profile(True)
    step()
    ktimes = ctx.kernel_times()
    ctx.profile(False)

    h2h = None
    if args.h2h and world == 1:
        h2h = host_to_host(ctx, src, off, lens, comp, coff, ccap, clen, crc, back, blen, brc, n, vlen, cstride,
                           stream, args.h2h_chunk)

    if rank == 0:
        gib = total_bytes / 2 ** 30
        # roofline of the dominant kernel: algorithmic bytes per launch
        alg_c = n * (vlen + META_BYTES) + comp_bytes
        alg_d = comp_bytes + n * (vlen + META_BYTES)
        # dominant compress kernel: the one with the largest summed launch time in the profiled step
        ckinds = [k for k in ktimes if k.startswith("deflate")]
        dom = max(ckinds, key=lambda k: ktimes[k][0])
        dom_ms, dom_launches = ktimes[dom]
        avg_launch_s = dom_ms / dom_launches / 1e3
        alg_launch = alg_c / dom_launches  # mean over the launches (chunks of the batch; the last one is shorter)
        achieved = alg_launch / avg_launch_s / 1e9
        # measured HBM bytes per launch of that kernel and its issue counters (scripts/pmc_traffic.py),
        # quoted only when measured on these kernel sources and this workload
        traffic, issue, tsrc = None, None, None
        if os.path.exists(args.traffic):
            try:
                with open(args.traffic) as f:
                    tj = json.load(f)
                if (tj.get("n") == n and tj.get("vlen") == vlen and tj.get("kind") == args.kind
                        and tj.get("source_id") == pmc_codec.source_id()):
                    # (a templated kernel is listed per instance, "name<1024u>": the one this workload ran)
                    kn, ks = pmc_codec.KERNEL_NAMES[dom], tj.get("kernels", {})
                    inst = [k for k in ks if k == kn or k.startswith(kn + "<")]
                    kj = max((ks[k] for k in inst), key=lambda e: e.get("launches", 0), default={})
                    traffic = kj.get("hbm_bytes_per_launch")
                    issue = kj.get("issue")
                    tsrc = os.path.relpath(args.traffic, ROOT)
            except (OSError, ValueError):
                traffic = None
        # issue floors of the dominant kernel from its counters (when measured on these sources): a wave64
        # VALU instruction occupies its SIMD 2 cycles (4 SIMDs per CU), a scalar instruction the CU's one
        # scalar unit 1 cycle; the clock is the measured GRBM_GUI_ACTIVE / 8 XCDs over the launch time
        floors = None
        if issue and issue.get("counters_per_launch"):
            cp = issue["counters_per_launch"]
            per_launch_vals = n / dom_launches
            clk_hz = cp["GRBM_GUI_ACTIVE"] / 8.0 / avg_launch_s
            cus = 256
            floors = {"valu_per_value": cp["SQ_INSTS_VALU"] / per_launch_vals,
                      "salu_per_value": cp["SQ_INSTS_SALU"] / per_launch_vals,
                      "clock_ghz": clk_hz / 1e9,
                      "valu_floor_ms": cp["SQ_INSTS_VALU"] * 2.0 / (4 * cus) / clk_hz * 1e3,
                      "salu_floor_ms": cp["SQ_INSTS_SALU"] / cus / clk_hz * 1e3,
                      "note": "per launch; VALU: 2 cycles per wave64 instruction on each of 4 SIMDs per CU, "
                              "SALU: one scalar unit per CU"}
        out = {
            "metric": METRIC, "value": gib / t_step_s, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": t_step_s * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: JSON slices of the reference's tests/data corpus (SURVEY.md §8d generator, "
                    f"seed {seed:#x})" if args.kind == 0 else "synthetic: random [A-Za-z0-9]",
            "config": {"workload": f"{n} x {vlen} B values per GPU ({'JSON-slice' if args.kind == 0 else 'alnum'}), "
                                   "batched gzip level-9 compress + decompress, device-resident; every member "
                                   "checked against the reference by a (length, CRC-32) digest (fullsize_parity)",
                       "values_per_gpu": n, "value_bytes": vlen, "total_values": n * world,
                       "partition": "MurmurHash3_x64_128('key'+i)[0] % 128 % n_gpus (NUM_SHARDS=128)",
                       "parallelism": f"shard-partitioned x{world}, no collective"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
                         "issue": issue, "issue_floors": floors,
                         # the whole step (compress + decompress) against the same peak
                         "path": {"alg_bytes_per_step": alg_c + alg_d,
                                  "achieved": (alg_c + alg_d) / (tc + td) / 1e9,
                                  "frac": (alg_c + alg_d) / (tc + td) / 1e9 / HBM_PEAK_GBS},
                         "kernel": pmc_codec.KERNEL_NAMES[dom],
                         "alg_bytes_per_launch": alg_launch, "avg_launch_ms": avg_launch_s * 1e3,
                         "launches_per_step": dom_launches,
                         "kernel_ms_per_step": {pmc_codec.KERNEL_NAMES.get(k, k): round(v[0], 3)
                                                for k, v in ktimes.items()}},
            "cpu_baseline": cpu,
            "compress_gib_s": gib / world / tc_max, "decompress_gib_s": gib / world / td_max,
            "decompress_roofline_frac": alg_d / td / 1e9 / HBM_PEAK_GBS,
            "ratio": total_comp / total_bytes, "verified_values": int(total_bytes // vlen),
            "mismatches": int(total_bad),
            "fullsize_parity": parity,
            "guard_counts": guards,
        }
        if h2h:
            out["host_to_host"] = h2h
        if landing:
            out["landing"] = landing
            out["config"]["parallelism"] = f"shard-partitioned x{world}; batch landed on rank 0, one all-to-all"
        print(json.dumps(out), flush=True)
        # a guard that fired means values silently took the slow retry kernel: fail the run loudly (the
        # line above still records the counts); large periodic values may legitimately take the stitch's
        # fallback (guard_counts.retry), small ones never
        assert guards["sort"] == 0 and guards["codes"] == 0 and guards["probe"] == 0, guards
        assert vlen > 31808 or guards["retry"] == 0, guards
    if distributed:
        dist.destroy_process_group()


def scatter_landing(L, args, route, corpus, corpus_len, seed, world, rank, n, vlen, dev, sh):
    """--landing scatter: rank 0 generates the batch of every rank's keys (landing_keys: key order) in its HBM,
    packs it by owner GPU on the device and one RCCL all-to-all over xGMI gives each rank its share
    (pmc_codec.scatter).  Timed between barriers; returns the rank's rows and keys and the scatter's figures."""
    import torch
    import torch.distributed as dist
    from pmc_codec import scatter as S
    packed = tags = counts = None
    if rank == 0:
        keys = landing_keys(route, world, n)
        batch = torch.empty(keys.numel() * vlen + 16, dtype=torch.uint8, device=dev)
        assert L.pmc_gen_values(corpus.data_ptr(), corpus_len, seed, args.kind, 0, keys.data_ptr(), keys.numel(),
                                vlen, batch.data_ptr(), sh) == 0
        owner = route[keys]
        packed, order, counts = S.pack_by_owner(batch[:keys.numel() * vlen].view(-1, vlen), owner, world)
        tags = keys[order]
        del batch, owner, order
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rows, got = S.scatter_rows(packed, tags, counts, vlen, device=dev)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    moved = n * world * vlen
    return {"mode": "scatter", "root": 0, "bytes": moved, "ms": t * 1e3, "gib_s": moved / t / 2 ** 30,
            "note": "one all-to-all of the landing batch (uint8 rows) plus its int64 keys; the timed steps then "
                    "run on each rank's received share", "rows": rows, "tags": got}


def host_to_host(ctx, src, off, lens, comp, coff, ccap, clen, crc, back, blen, brc, n, vlen, cstride, stream,
                 chunk=0):
    """PCIe-inclusive rates.

    serial:    pinned H2D of the whole batch -> kernels -> D2H, one stream;
    pipelined: pmc_gzip_{compress,decompress}_batch_pinned, chunks of `chunk` values whose H2D / D2H
               run on the context's copy streams beside the previous / next chunk's kernels.
    Both start and end in pinned host memory; the pipelined leg is verified against the device path
    (compressed lengths) and the source bytes (round trip)."""
    import torch
    sh = stream.cuda_stream
    h_src = torch.empty(src.numel(), dtype=torch.uint8, pin_memory=True)
    h_comp = torch.empty(comp.numel(), dtype=torch.uint8, pin_memory=True)
    h_back = torch.empty(back.numel(), dtype=torch.uint8, pin_memory=True)
    h_src.copy_(src)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    e[0].record(stream)
    src.copy_(h_src, non_blocking=True)
    ctx.compress_device(src, off, lens, comp, coff, ccap, clen, crc, vlen, sh)
    h_comp.copy_(comp, non_blocking=True)
    e[1].record(stream)
    comp.copy_(h_comp, non_blocking=True)
    ctx.decompress_device(comp, coff, clen, back, off, lens, blen, brc, vlen, sh)
    h_back.copy_(back, non_blocking=True)
    e[2].record(stream)
    torch.cuda.synchronize()
    tc = e[0].elapsed_time(e[1]) / 1e3
    td = e[1].elapsed_time(e[2]) / 1e3
    gib = n * vlen / 2 ** 30
    out = {"compress_gib_s": gib / tc, "decompress_gib_s": gib / td, "roundtrip_gib_s": gib / (tc + td),
           "note": "whole batch staged: pinned H2D of inputs, kernel, D2H of fixed-stride output slots"}

    # ---- pipelined leg: the C-ABI's chunked, copy/compute-overlapped pinned batch calls -------------
    pin = lambda t: t.cpu().pin_memory()  # noqa: E731
    h_off, h_lens, h_coff, h_ccap = pin(off), pin(lens), pin(coff), pin(ccap)
    h_clen = torch.zeros(n, dtype=torch.int32, pin_memory=True)
    h_crc = torch.zeros(n, dtype=torch.int32, pin_memory=True)
    h_blen = torch.zeros(n, dtype=torch.int32, pin_memory=True)
    h_brc = torch.zeros(n, dtype=torch.int32, pin_memory=True)
    h_back.zero_()

    h_poff = torch.zeros(n, dtype=torch.int64, pin_memory=True)

    def leg():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # SET side: values in, members out packed back to back (dst_off NULL: only real bytes cross PCIe)
        ctx.compress_pinned(h_src, h_off, h_lens, h_comp, None, h_ccap, h_clen, h_crc, vlen, chunk)
        t1 = time.perf_counter()
        # GET side: the packed members in, at offsets a store would already hold (prefix sum of the
        # lengths, computed outside the timed region)
        h_poff.copy_(torch.cumsum(h_clen.to(torch.int64), 0) - h_clen)
        t1b = time.perf_counter()
        ctx.decompress_pinned(h_comp, h_poff, h_clen, h_back, h_off, h_lens, h_blen, h_brc, vlen, chunk)
        t2 = time.perf_counter()
        return t1 - t0, t2 - t1b

    leg()  # warm-up: allocates the chunk slots and copy streams
    times = [leg() for _ in range(2)]
    pc = min(t[0] for t in times)
    pd = min(t[1] for t in times)
    bad = int((h_crc != 0).sum()) + int((h_brc != 0).sum()) + int((h_blen != h_lens).sum())
    bad += int((h_clen != clen.cpu()).sum())
    if not torch.equal(h_back[:n * vlen], h_src[:n * vlen]):
        bad += 1
    out["pipelined"] = {"compress_gib_s": gib / pc, "decompress_gib_s": gib / pd, "roundtrip_gib_s": gib / (pc + pd),
                        "chunk_values": chunk or max(65536, (n + 15) // 16), "mismatches": bad,
                        "compressed_bytes": int(h_clen.sum()),
                        "note": "pmc_gzip_*_batch_pinned: host wall clock, pinned host buffers in and out; compress "
                                "writes the members packed (device scan + compaction), decompress reads them packed; "
                                "H2D/D2H of neighbouring chunks overlapped with the kernels"}
    return out

if __name__ == "__main__":
    main()
