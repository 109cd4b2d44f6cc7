"""Device-batch plumbing for the codec: torch supplies HBM buffers and streams only.

A batch is SoA: one uint8 byte buffer plus per-value offsets (int64 = uint64 bits) and
lengths (int32 = uint32 bits), exactly the layout pmc_gzip_*_batch consume.
"""
from dataclasses import dataclass

import numpy as np
import torch

from . import Context, decompress_capacity, gzip_bound


@dataclass
class Batch:
    data: torch.Tensor  # uint8
    off: torch.Tensor   # int64
    len: torch.Tensor   # int32
    n: int
    max_len: int

    def host_items(self, lens=None):
        lens = (lens if lens is not None else self.len).cpu().numpy().astype(np.int64)
        off = self.off.cpu().numpy()
        data = self.data.cpu().numpy()
        return [data[off[i]:off[i] + lens[i]].tobytes() for i in range(self.n)]


def pack(values, device="cuda", align=4):
    n = len(values)
    lens = np.array([len(v) for v in values], dtype=np.int64)
    slots = (lens + align - 1) // align * align
    off = np.zeros(n, dtype=np.int64)
    if n > 1:
        off[1:] = np.cumsum(slots[:-1])
    buf = np.zeros(int(slots.sum()) + 16, dtype=np.uint8)
    for i, v in enumerate(values):
        buf[off[i]:off[i] + lens[i]] = np.frombuffer(v, dtype=np.uint8)
    return Batch(torch.from_numpy(buf).to(device), torch.from_numpy(off).to(device),
                 torch.from_numpy(lens.astype(np.int32)).to(device), n, int(lens.max()) if n else 0)


def slots_for(caps, device="cuda", align=4):
    caps = np.asarray(caps, dtype=np.int64)
    slots = (caps + align - 1) // align * align
    off = np.zeros(len(caps), dtype=np.int64)
    if len(caps) > 1:
        off[1:] = np.cumsum(slots[:-1])
    total = int(slots.sum()) + 16
    return (torch.empty(total, dtype=torch.uint8, device=device), torch.from_numpy(off).to(device),
            torch.from_numpy(caps.astype(np.int32)).to(device))


def stream_handle():
    return torch.cuda.current_stream().cuda_stream


def compress(ctx: Context, b: Batch):
    caps = [gzip_bound(int(x)) for x in b.len.cpu().numpy()]
    dst, doff, dcap = slots_for(caps, b.data.device)
    dlen = torch.zeros(b.n, dtype=torch.int32, device=b.data.device)
    rc = torch.zeros(b.n, dtype=torch.int32, device=b.data.device)
    ctx.compress_device(b.data, b.off, b.len, dst, doff, dcap, dlen, rc, b.max_len, stream_handle())
    return Batch(dst, doff, dlen, b.n, int(max(caps) if caps else 0)), rc


def decompress(ctx: Context, b: Batch, caps=None):
    if caps is None:
        caps = [decompress_capacity(x) for x in b.host_items()]
    dst, doff, dcap = slots_for(caps, b.data.device)
    dlen = torch.zeros(b.n, dtype=torch.int32, device=b.data.device)
    rc = torch.zeros(b.n, dtype=torch.int32, device=b.data.device)
    ctx.decompress_device(b.data, b.off, b.len, dst, doff, dcap, dlen, rc, int(max(caps) if len(caps) else 0),
                          stream_handle())
    return Batch(dst, doff, dlen, b.n, int(max(caps) if len(caps) else 0)), rc
