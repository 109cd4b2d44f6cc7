"""CPU, world_size 2 over gloo: bench.py's multi-GPU partitioning and reduction.

The codec path shards with no collective: each rank owns the keys
"key"+i whose MurmurHash3_x64_128(key, 0)[0] % NUM_SHARDS % world equals its rank
(src/server/server.cpp:113,121,132 routing), takes the first n of them, and the
ranks meet only to take the max step time and the summed byte / error counters.
Here the routing comes from the oracle's MurmurHash3 on the CPU; the GPU routing
kernel is checked against the same oracle in test_gpu_codec.py.
"""
import ctypes
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _route_cpu(span, world):
    import numpy as np
    from oracle import pyoracle as O
    L = O.lib()
    L.oracle_murmur3_x64_128_h1.restype = ctypes.c_uint64
    L.oracle_murmur3_x64_128_h1.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32]
    out = np.empty(span, dtype=np.uint8)
    for i in range(span):
        k = b"key%d" % i
        out[i] = (L.oracle_murmur3_x64_128_h1(k, len(k), 0) % 128) % world
    return out


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd")]
    import torch
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        span = bench.route_span(n, world)
        route = torch.from_numpy(_route_cpu(span, world))
        idx = bench.select_rank_keys(route, rank, n)
        gathered = [torch.empty(n, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, idx)
        times, sums = bench.reduce_over_ranks([1.0 + rank, 10.0 - rank, 0.5], [float(n * 1024), 7.0, float(rank)],
                                              world, torch.device("cpu"))
        if rank == 0:
            q.put(([g.tolist() for g in gathered], route.tolist(), times, sums))
    finally:
        dist.destroy_process_group()


def test_two_rank_partition_and_reduction():
    import torch.multiprocessing as mp
    world, n = 2, 1500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        gathered, route, times, sums = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    # each rank got n keys, all routed to itself, in increasing key order; ranks are disjoint
    for r, keys in enumerate(gathered):
        assert len(keys) == n and keys == sorted(keys)
        assert all(route[k] == r for k in keys)
    assert not set(gathered[0]) & set(gathered[1])
    # the ranks' shares are exactly the first n keys of each shard group
    for r in range(world):
        assert gathered[r] == [k for k in range(len(route)) if route[k] == r][:n]
    # max over ranks for times, sum for counters
    assert times == [2.0, 10.0, 0.5]
    assert sums == [float(world * n * 1024), 14.0, 1.0]


def _rows_of(keys, vlen):
    import torch
    k = torch.as_tensor(keys, dtype=torch.int64).view(-1, 1)
    return ((k * 131 + torch.arange(vlen, dtype=torch.int64).view(1, -1) * 7) % 251).to(torch.uint8)


def _scatter_worker(rank, world, port, n, vlen, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd")]
    import torch
    import torch.distributed as dist
    import bench
    from pmc_codec import scatter as S
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        route = torch.from_numpy(_route_cpu(bench.route_span(n, world), world))
        packed = tags = counts = None
        if rank == 0:  # the landing batch: every rank's keys, in key order, resident on the landing rank
            landing = bench.landing_keys(route, world, n)
            packed, order, counts = S.pack_by_owner(_rows_of(landing, vlen), route[landing], world)
            tags = landing[order]
        rows, got = S.scatter_rows(packed, tags, counts, vlen, device=torch.device("cpu"))
        want = bench.select_rank_keys(route, rank, n)
        q.put((rank, bool(torch.equal(got, want)), bool(torch.equal(rows, _rows_of(want, vlen))), int(got.numel())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_landing_batch_scattered_to_owners(world):
    """A batch resident on rank 0 (bench.py --landing scatter) reaches each owner rank as exactly the keys (and
    value rows) that rank would have selected itself -- the same partition as the no-collective path, so the
    per-rank reference digests still apply -- through pack_by_owner + one all-to-all (gloo here, RCCL on GPUs)."""
    import torch.multiprocessing as mp
    n, vlen = 700, 40
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, n, vlen, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert res == [(r, True, True, n) for r in range(world)]


def test_pack_by_owner_keeps_batch_order():
    import torch
    sys.path[:0] = [os.path.join(ROOT, "poor-man-s-cache_amd")]
    from pmc_codec import scatter as S
    owner = torch.tensor([2, 0, 1, 0, 2, 2, 1, 0], dtype=torch.uint8)
    vals = torch.arange(8, dtype=torch.uint8).view(-1, 1).repeat(1, 3)
    packed, order, counts = S.pack_by_owner(vals, owner, 3)
    assert counts.tolist() == [3, 2, 3]
    assert order.tolist() == [1, 3, 7, 2, 6, 0, 4, 5]
    assert packed[:, 0].tolist() == order.tolist()
    with pytest.raises(ValueError):
        S.pack_by_owner(vals, owner, 2)


def test_route_span_covers_every_world():
    import bench
    for world in (1, 2, 4, 8):
        n = 20000
        route = _route_cpu(bench.route_span(n, world), world)
        for r in range(world):
            assert (route == r).sum() >= n


if __name__ == "__main__":
    sys.exit(pytest.main([__file__, "-q"]))


def test_rank_digests_cover_bench_key_selection():
    """tests/golden/rank_digests.json (the reference's Compress over each rank's routed values,
    make_full_digests.py --ranks) was computed on exactly the key indices bench.py --gpus N selects:
    route "key"+i by MurmurHash3 % 128 % N over route_span keys, first n per rank (select_rank_keys)."""
    import hashlib
    import json
    import numpy as np
    import torch
    sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd")]
    import bench
    from oracle import pyoracle as O
    with open(os.path.join(ROOT, "tests", "golden", "rank_digests.json")) as f:
        doc = json.load(f)
    worlds = sorted({s["world"] for s in doc["sets"]})
    assert worlds == [2, 4, 8]
    z = np.load(os.path.join(ROOT, "tests", "golden", "route_golden.npz"))  # the reference's hashFunc
    for w in worlds:
        got = O.route_keys(0, int(z["index"].max()) + 1, 128, w)
        assert all(int(got[i]) == int(h) % 128 % w for i, h in zip(z["index"], z["hash"]))
        n = doc["sets"][0]["n"]
        route = torch.from_numpy(O.route_keys(0, bench.route_span(n, w), 128, w))
        for s in (s for s in doc["sets"] if s["world"] == w):
            idx = bench.select_rank_keys(route, s["rank"], n).numpy().astype("<u8")
            assert hashlib.sha256(idx.tobytes()).hexdigest() == s["index_sha256"], (w, s["rank"])
            assert set(s["prefixes"]) >= {str(n)}
