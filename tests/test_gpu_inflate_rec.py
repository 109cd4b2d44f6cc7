"""GPU: the two-phase record inflate (pmc_inflate_rec.hip) on the shapes it special-cases.

Members of <= 4096 output bytes decode in inflate_rec_kernel: <= 256-byte members four at a time in
256-position slices of the image, larger ones one at a time; members of more output go to
inflate_lane_kernel, anything either declines to the wave kernels.  The batch mixes all of these
in one launch (visit order on: n >= 4096), writes into slots at unaligned offsets with guard bytes
around every slot, and checks bytes and verdicts against the oracle (zlib's inflate rules).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import pmc_codec
    c = pmc_codec.Context(0)
    yield c
    c.close()


def _values(golden, rng):
    corpus = golden.corpus * 3
    sizes = [1, 2, 3, 29, 200, 255, 256, 257, 300, 511, 512, 513, 1000, 1023, 1024, 1025, 2047, 2048, 3000, 4095,
             4096, 4097, 5000, 9000]
    vals = []
    for s in sizes:
        o = int(rng.integers(0, len(corpus) - s))
        vals.append(corpus[o:o + s])                                   # JSON slice
        vals.append(b"a" * s)                                          # one long chain of copies
        vals.append(b"abc" * (s // 3) + b"x" * (s % 3))                # period-3 copies
        vals.append(bytes(rng.integers(0, 4, s, dtype=np.uint8)))      # small alphabet, NULs
        vals.append(bytes(rng.integers(0, 256, s, dtype=np.uint8)))    # stored blocks (declined)
    # bulk: small JSON slices, so waves hold mixed small / large members
    for _ in range(5000):
        s = int(rng.integers(1, 700))
        o = int(rng.integers(0, len(corpus) - s))
        vals.append(corpus[o:o + s])
    order = rng.permutation(len(vals))
    return [vals[k] for k in order]


def _unaligned_slots(caps, rng, guard=0xA5):
    import torch
    caps = np.asarray(caps, dtype=np.int64)
    pad = rng.integers(1, 8, len(caps))
    off = np.zeros(len(caps), dtype=np.int64)
    pos = 3
    for i, c in enumerate(caps):
        off[i] = pos
        pos += int(c) + int(pad[i])
    host = np.full(pos + 16, guard, dtype=np.uint8)
    return host, torch.from_numpy(host).cuda(), torch.from_numpy(off).cuda(), torch.from_numpy(caps.astype(np.int32)).cuda(), off


def test_record_inflate_mixed_sizes_unaligned_slots(golden):
    import torch
    import pmc_codec
    from pmc_codec import device as D
    from oracle import pyoracle as O
    rng = np.random.default_rng(2024)
    vals = _values(golden, rng)
    gz = [O.compress(v) for v in vals]
    caps = [max(len(v), 1) for v in vals]
    host0, dst, doff, dcap, off = _unaligned_slots(caps, rng)
    b = D.pack(gz)
    n = len(vals)
    dlen = torch.zeros(n, dtype=torch.int32, device="cuda")
    rc = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    ctx = pmc_codec.Context(0)
    try:
        ctx.decompress_device(b.data, b.off, b.len, dst, doff, dcap, dlen, rc, max(caps), D.stream_handle())
        torch.cuda.synchronize()
    finally:
        ctx.close()
    rc = rc.cpu().numpy()
    dlen = dlen.cpu().numpy()
    out = dst.cpu().numpy()
    bad = [k for k in range(n) if rc[k] != 0 or dlen[k] != len(vals[k]) or
           out[off[k]:off[k] + len(vals[k])].tobytes() != vals[k]]
    assert not bad, [(k, len(vals[k]), int(rc[k])) for k in bad[:8]]
    # every byte outside the members is untouched
    mask = np.ones(len(out), dtype=bool)
    for k in range(n):
        mask[off[k]:off[k] + len(vals[k])] = False
    assert (out[mask] == host0[mask]).all()


def test_record_inflate_capacity_and_corrupt_verdicts(golden):
    """Output capacity one short of ISIZE (PMC_E_CAPACITY + the decoded size), a lying ISIZE, a
    corrupt distance: zlib's verdicts."""
    import torch
    import pmc_codec
    from pmc_codec import device as D
    from oracle import pyoracle as O
    rng = np.random.default_rng(5)
    corpus = golden.corpus * 2
    vecs, caps = [], []
    for s in (10, 100, 256, 257, 1024, 4096, 4097):
        o = int(rng.integers(0, len(corpus) - s))
        z = O.compress(corpus[o:o + s])
        vecs.append(z)
        caps.append(s)            # exact
        vecs.append(z)
        caps.append(s - 1)        # one short
        t = bytearray(z)          # ISIZE + 1
        t[-4:] = (s + 1).to_bytes(4, "little")
        vecs.append(bytes(t))
        caps.append(s + 8)
        t = bytearray(z)          # ISIZE - 1
        t[-4:] = (s - 1).to_bytes(4, "little")
        vecs.append(bytes(t))
        caps.append(s + 8)
        for _ in range(6):        # bit flips in the deflate body
            t = bytearray(z)
            t[int(rng.integers(10, len(z) - 8))] ^= 1 << int(rng.integers(8))
            vecs.append(bytes(t))
            caps.append(s + 8)
    b = D.pack(vecs)
    n = len(vecs)
    dst, doff, dcap = D.slots_for(caps)
    dlen = torch.zeros(n, dtype=torch.int32, device="cuda")
    rc = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    ctx = pmc_codec.Context(0)
    try:
        ctx.decompress_device(b.data, b.off, b.len, dst, doff, dcap, dlen, rc, max(caps), D.stream_handle())
        torch.cuda.synchronize()
    finally:
        ctx.close()
    rc = rc.cpu().numpy()
    dl = dlen.cpu().numpy()
    got = D.Batch(dst, doff, dlen, n, 0).host_items()
    short = 0
    for k, v in enumerate(vecs):
        erc, eout = O.decompress(v, cap=caps[k], grow=False)
        assert rc[k] == erc, (k, caps[k], int(rc[k]), erc)
        if erc == 0:
            assert got[k] == eout, k
        if erc == pmc_codec.E_CAPACITY:
            # no verdict yet: the decoded size comes back, and exactly that much room suffices
            short += 1
            assert dl[k] > caps[k], k
            assert O.decompress(v, cap=int(dl[k]), grow=False)[0] != O.CAPACITY, k
    assert short >= 7  # every "one short" member


def _lane_pass_counts(ctx, vlen, n):
    """Compress + decompress n JSON slices of vlen bytes (the bench generator; values longer than the
    corpus are slices of it tiled); returns (members returned byte-exact, members the record / lane
    fast paths handed to the wave kernels: pmc_ctx_guard_counts counts[4])."""
    import os
    import torch
    import pmc_codec
    from pmc_codec import device as D
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = os.path.join(root, "tests", "golden", "data")
    cb = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))
    if vlen > len(cb):
        cb = cb * (vlen // len(cb) + 2)
    corpus = torch.frombuffer(bytearray(cb), dtype=torch.uint8).cuda()
    data = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
    assert pmc_codec.lib().pmc_gen_values(corpus.data_ptr(), len(cb), 0x5EED, 0, 0, None, n, vlen, data.data_ptr(),
                                          D.stream_handle()) == 0
    off = torch.arange(n, dtype=torch.int64, device="cuda") * vlen
    lens = torch.full((n,), vlen, dtype=torch.int32, device="cuda")
    out, rc = D.compress(ctx, D.Batch(data, off, lens, n, vlen))
    torch.cuda.synchronize()
    assert int((rc != 0).sum()) == 0
    before = ctx.guard_counts()["inflate_retry"]
    back, brc = D.decompress(ctx, out, [vlen] * n)
    torch.cuda.synchronize()
    retried = ctx.guard_counts()["inflate_retry"] - before
    bo = back.host_items()
    src = data.cpu().numpy().tobytes()
    same = sum(1 for i in range(n) if int(brc[i]) == 0 and bo[i] == src[i * vlen:(i + 1) * vlen])
    return same, retried


def test_large_members_decode_on_the_lane_passes(ctx):
    """16-30 KB JSON members (the reference's own 5_*/6_* fixtures are 29-30 KB): a third of them use more
    than 96 lit/len symbols, which the first lane pass declines and the wide pass (128-entry lists) takes.
    At most 1 % of the members may reach the wave-kernel retry (the context's counter), and every member
    must come back byte-exact."""
    for vlen in (30000, 16000):
        same, retried = _lane_pass_counts(ctx, vlen, 4096)
        assert same == 4096 and retried <= 0.01 * 4096, (vlen, same, retried)


@pytest.mark.gpu
def test_multiblock_members_decode_in_the_lane_pass(ctx):
    """Members of several DEFLATE blocks (zlib flushes every 16383 symbols: 100 KB and 300 KB JSON values)
    decode in the multi-block lane pass, block after block, not in the wave-per-member retry kernel: the
    context's retry counter stays put and every member comes back byte-exact."""
    for vlen, n in ((100000, 128), (300000, 24)):
        same, retried = _lane_pass_counts(ctx, vlen, n)
        assert same == n and retried == 0, (vlen, same, retried)
