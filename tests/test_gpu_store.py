"""GPU: the device-resident compressed value store (pmc_store_*).

Values go in as host bytes and are compressed straight into HBM extents: the members held there
must be the reference's bytes (goldens from its own Compress).  GETs come back decompressed and
framed in the server's wire formats: raw, the custom protocol's value + 0x1F
(/root/reference/src/server/protocol.hpp:17) and RESP bulk strings "$<len>\\r\\n<value>\\r\\n"
(protocol.cpp:466-497).  Freed extents are reused; a full heap fails per value (Z_MEM_ERROR).
"""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch  # noqa: F401
    import pmc_codec
    c = pmc_codec.Context(0)
    yield c
    c.close()


def test_store_put_members_get_framed(ctx, golden):
    import pmc_codec
    pairs = [(r, g) for r, g in golden.pairs() if r][:400]
    st = pmc_codec.Store(ctx, 64 << 20)
    ext, rc = st.put([r for r, _ in pairs])
    assert rc == [0] * len(pairs)
    assert all(ext[i].flags == 1 and ext[i].raw_len == len(pairs[i][0]) for i in range(len(pairs)))
    mem = st.members(ext, len(pairs))
    bad = [i for i, (_, g) in enumerate(pairs) if mem[i] != g]
    assert not bad, bad[:10]
    for frame, wrap in ((pmc_codec.FRAME_RAW, lambda v: v), (pmc_codec.FRAME_CUSTOM, lambda v: v + b"\x1f"),
                        (pmc_codec.FRAME_RESP, lambda v: b"$%d\r\n" % len(v) + v + b"\r\n")):
        got = st.get(ext, len(pairs), frame)
        bad = [i for i, (r, _) in enumerate(pairs) if got[i] != (0, wrap(r))]
        assert not bad, (frame, bad[:10])
    # one batch answering both protocols (pmc_store_get_batch_frames): frames cycle raw / custom / RESP
    wraps = ((lambda v: v), (lambda v: v + b"\x1f"), (lambda v: b"$%d\r\n" % len(v) + v + b"\r\n"))
    frames = [i % 3 for i in range(len(pairs))]
    got = st.get(ext, len(pairs), frames)
    bad = [i for i, (r, _) in enumerate(pairs) if got[i] != (0, wraps[frames[i]](r))]
    assert not bad, bad[:10]
    s0 = st.stats()
    assert s0["used"] == s0["reserved"] > 0


def test_store_free_reuse_and_full_heap(ctx, golden):
    import pmc_codec
    vals = [r for r, _ in golden.pairs() if 0 < len(r) <= 4096][:200]
    st = pmc_codec.Store(ctx, 1 << 20)
    ext, rc = st.put(vals)
    assert rc == [0] * len(vals)
    before = st.stats()
    # free every other extent, then put the same values again: the freed extents are reused
    half = (pmc_codec.Extent * len(vals))()
    for i in range(0, len(vals), 2):
        half[i] = ext[i]
    st.free(half, len(vals))
    mid = st.stats()
    assert mid["used"] < before["used"] and mid["reserved"] == before["reserved"]
    ext2, rc2 = st.put([vals[i] for i in range(0, len(vals), 2)])
    assert rc2 == [0] * len(rc2)
    assert st.stats()["reserved"] == before["reserved"]
    got = st.get(ext2, len(rc2))
    assert [g for _, g in got] == [vals[i] for i in range(0, len(vals), 2)]
    # the odd extents are untouched by the frees and the re-puts
    odd = (pmc_codec.Extent * len(vals))()
    k = 0
    for i in range(1, len(vals), 2):
        odd[k] = ext[i]
        k += 1
    assert [g for _, g in st.get(odd, k)] == [vals[i] for i in range(1, len(vals), 2)]
    # a freed extent is not readable; a heap that cannot hold a value fails that value only
    assert st.get(half, 1)[0][0] == pmc_codec.E_ARG
    import numpy as np
    small = pmc_codec.Store(ctx, 4096)
    noise = bytes(np.random.default_rng(3).integers(0, 256, 6000, dtype=np.uint8))  # stored blocks: > 4 KiB
    e3, rc3 = small.put([b"x" * 100, noise, b"y" * 200])
    assert rc3[0] == 0 and rc3[1] == pmc_codec.Z_MEM_ERROR and rc3[2] == 0
    assert [g for _, g in small.get(e3, 3)][0::2] == [b"x" * 100, b"y" * 200]
    assert small.get(e3, 3)[1][0] == pmc_codec.E_ARG


def test_store_footprint_is_compressed_size(ctx, golden):
    """Extents are sized by the member, not by the uncompressed bound (the reference's Entry holds the
    compressed bytes, kvs.hpp:38-44): used == sum of 16-byte-rounded member sizes.  A put that cannot
    place a value (heap full) leaves `used` unchanged."""
    import pmc_codec
    pairs = [(r, g) for r, g in golden.pairs() if 0 < len(r) <= 4096]
    st = pmc_codec.Store(ctx, 16 << 20)
    ext, rc = st.put([r for r, _ in pairs])
    assert rc == [0] * len(pairs)
    want = sum((len(g) + 15) & ~15 for _, g in pairs)
    assert st.stats()["used"] == want
    bound = sum((pmc_codec.gzip_bound(len(r)) + 15) & ~15 for r, _ in pairs)
    assert want < 0.75 * bound
    assert [ext[i].len for i in range(len(pairs))] == [len(g) for _, g in pairs]
    full = pmc_codec.Store(ctx, 4096)
    e1, r1 = full.put([b"z" * 3000])
    assert r1 == [0]
    u = full.stats()["used"]
    import numpy as np
    noise = bytes(np.random.default_rng(4).integers(0, 256, 8000, dtype=np.uint8))
    e2, r2 = full.put([noise, noise])
    assert r2 == [pmc_codec.Z_MEM_ERROR] * 2 and full.stats()["used"] == u
    assert e2[0].flags == 0 and e2[1].flags == 0


def _d2h(ptr, nbytes):
    """Copy nbytes of device memory at ptr into host bytes (HIP runtime through ctypes)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(nbytes)
    assert hip.hipMemcpy(buf, ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 2) == 0  # hipMemcpyDeviceToHost
    return buf.raw


def test_slab_set_get_overwrite_empty(ctx, golden):
    """pmc_slab_*: values into permuted slots (members = the reference's bytes, read back from the slab),
    get back, overwrite, an empty slot gives INVALID_INPUT."""
    import numpy as np
    import torch
    import pmc_codec
    from pmc_codec import device as D
    pairs = [(r, g) for r, g in golden.pairs() if 0 < len(r) <= 4096][:300]
    n, K = len(pairs), 1000
    slab = pmc_codec.Slab(ctx, K, 4096)
    b = D.pack([r for r, _ in pairs])
    slots = torch.from_numpy(np.random.default_rng(3).permutation(K)[:n].astype(np.int32)).cuda()
    rc = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    slab.set(b.data, b.off, b.len, slots, rc, D.stream_handle())
    torch.cuda.synchronize()
    assert int((rc != 0).sum()) == 0
    lens = np.frombuffer(_d2h(slab.lengths_ptr(), 4 * K), dtype=np.uint32)
    data = _d2h(slab.data_ptr(), slab.stride * K)
    sl = slots.cpu().numpy()
    for i, (_, g) in enumerate(pairs):
        assert lens[sl[i]] == len(g) and data[sl[i] * slab.stride:sl[i] * slab.stride + len(g)] == g, i
    caps = [max(len(r), 1) for r, _ in pairs]
    dst, doff, dcap = D.slots_for(caps)
    dlen = torch.zeros(n, dtype=torch.int32, device="cuda")
    grc = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    slab.get(slots, dst, doff, dcap, dlen, grc, D.stream_handle())
    torch.cuda.synchronize()
    assert int((grc != 0).sum()) == 0
    got = D.Batch(dst, doff, dlen, n, 0).host_items()
    assert got == [r for r, _ in pairs]
    # overwrite the first half with the second half's values
    h = n // 2
    b2 = D.pack([r for r, _ in pairs[h:2 * h]])
    rc2 = torch.full((h,), 7, dtype=torch.int32, device="cuda")
    slab.set(b2.data, b2.off, b2.len, slots[:h].contiguous(), rc2, D.stream_handle())
    dst2, doff2, dcap2 = D.slots_for([max(len(r), 1) for r, _ in pairs[h:2 * h]])
    dlen2 = torch.zeros(h, dtype=torch.int32, device="cuda")
    grc2 = torch.full((h,), 7, dtype=torch.int32, device="cuda")
    slab.get(slots[:h].contiguous(), dst2, doff2, dcap2, dlen2, grc2, D.stream_handle())
    torch.cuda.synchronize()
    assert int((grc2 != 0).sum()) == 0
    assert D.Batch(dst2, doff2, dlen2, h, 0).host_items() == [r for r, _ in pairs[h:2 * h]]
    # an empty slot
    empty = int(np.setdiff1d(np.arange(K), sl)[0])
    e = torch.tensor([empty], dtype=torch.int32, device="cuda")
    erc = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    slab.get(e, dst, doff[:1].contiguous(), dcap[:1].contiguous(), dlen[:1].contiguous(), erc, D.stream_handle())
    torch.cuda.synchronize()
    assert int(erc.item()) == pmc_codec.INVALID_INPUT
    slab.close()


def test_mix_bench_two_streams_small():
    """bench.py --mix (BASELINE configs[2] shape on the slab: SETs and GETs of a batch on two streams,
    cross-batch order by events), small: every GET verified against the value its key held."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--mix", "--mix-keys", "65536", "--mix-ops",
                        "262144"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["mismatches"] == 0 and res["config"]["streams"] == 2 and res["ops"] == 262144, res
