"""A batch that lands on ONE GPU, scattered to the GPUs that own its keys (the one collective the
north star names).

The reference routes a key to shard hashFunc(key) % NUM_SHARDS (/root/reference/src/server/server.cpp:113,121,132);
GPU g owns shards {s : s % nGPU == g}.  Normally every GPU receives its share straight from pinned
host memory and there is no collective.  When the batch is already resident in one GPU's HBM (it landed there), the
landing rank packs its values by owner on the device (a stable sort of the owners, then one row gather, so each
owner's values stay in batch order) and one RCCL all-to-all over xGMI hands every owner its contiguous slice; the
owner indices travel the same way.  Values are fixed-size rows here (bench.py's batches: n x V bytes); a row is
never split across ranks.

Only torch.distributed collectives are used, so the same code runs on RCCL (one process per GPU, device tensors)
and on gloo (CPU tensors, tests/test_multirank.py).
"""
import torch
import torch.distributed as dist


def pack_by_owner(values, owner, world):
    """values [N, V] uint8, owner [N] (rank per row) -> (packed [N, V], order [N] int64, counts [world] int64):
    packed rows are grouped by owner rank, in batch order within each group; order[j] is packed row j's batch row."""
    o = owner.to(torch.int64)
    order = torch.argsort(o, stable=True)
    counts = torch.bincount(o, minlength=world)
    if counts.numel() != world:
        raise ValueError(f"owner ranks outside [0, {world})")
    return values.index_select(0, order), order, counts


def scatter_rows(packed, tags, counts, vlen, root=0, device=None):
    """Collective over the default group: the root's packed rows (grouped by owner, counts[r] rows for rank r) and
    their int64 tags go to their owners.  Every rank passes vlen; only the root's packed / tags / counts are read.
    Returns (rows [m, vlen] uint8, tags [m] int64) on `device` (default: the root's tensors' device)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    if device is None:
        device = packed.device
    c = counts.to(device=device, dtype=torch.int64).clone() if rank == root else \
        torch.empty(world, dtype=torch.int64, device=device)
    dist.broadcast(c, root)
    cl = [int(x) for x in c.tolist()]
    m = cl[rank]
    rows = torch.empty((m, vlen), dtype=torch.uint8, device=device)
    got = torch.empty(m, dtype=torch.int64, device=device)
    recv_rows = [0] * world
    recv_rows[root] = m
    if rank == root:
        if packed.shape != (sum(cl), vlen) or tags.shape != (sum(cl),):
            raise ValueError(f"packed {tuple(packed.shape)} / tags {tuple(tags.shape)} do not match counts {cl}")
        send_rows, src_rows, src_tags = cl, packed.reshape(-1), tags.to(torch.int64).contiguous()
    else:
        send_rows = [0] * world
        src_rows = torch.empty(0, dtype=torch.uint8, device=device)
        src_tags = torch.empty(0, dtype=torch.int64, device=device)
    dist.all_to_all_single(rows.view(-1), src_rows, [r * vlen for r in recv_rows], [r * vlen for r in send_rows])
    dist.all_to_all_single(got, src_tags, recv_rows, send_rows)
    return rows, got
