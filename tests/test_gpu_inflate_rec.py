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


def test_large_members_decode_on_the_lane_passes(tmp_path):
    """16-30 KB JSON members (the reference's own 5_*/6_* fixtures are 29-30 KB): a third of them use more
    than 96 lit/len symbols, which the first lane pass declines and the wide pass (128-entry lists) takes.
    Run in a child with PMC_DIAG_INFLATE_STOP=2 (verdicts after the CRC check, before the wave-kernel
    retry): at least 99 % of the members must come back decoded, byte-exact, from the lane passes alone,
    and the full path (retry included) must return every member."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    probe = os.path.join(root, "scripts", "inflate_probe.py")
    out = {}
    for stop in ("2", "0"):
        r = subprocess.run([sys.executable, probe, "30000", "16000"], capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, PMC_DIAG_INFLATE_STOP=stop))
        assert r.returncode == 0, r.stdout + r.stderr
        for ln in r.stdout.splitlines():
            if ln.startswith("stop="):
                f = dict(x.split("=", 1) for x in ln.split()[:2])
                out[(f["stop"], int(f["vlen"]))] = int(ln.rsplit(":", 1)[1])
    for vlen in (30000, 16000):
        assert out[("2", vlen)] >= 0.99 * 4096, out
        assert out[("0", vlen)] == 4096, out


@pytest.mark.gpu
def test_multiblock_members_decode_in_the_lane_pass():
    """Members of several DEFLATE blocks (zlib flushes every 16383 symbols: 100 KB and 300 KB JSON values)
    decode in the multi-block lane pass, block after block, not in the wave-per-member retry kernel:
    with PMC_DIAG_INFLATE_STOP=2 (verdicts before the retry) every member comes back byte-exact."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    probe = os.path.join(root, "scripts", "inflate_probe.py")
    out = {}
    for stop in ("2", "0"):
        r = subprocess.run([sys.executable, probe, "100000:128", "300000:24"], capture_output=True, text=True,
                           timeout=600, env=dict(os.environ, PMC_DIAG_INFLATE_STOP=stop))
        assert r.returncode == 0, r.stdout + r.stderr
        for ln in r.stdout.splitlines():
            if ln.startswith("stop="):
                f = dict(x.split("=", 1) for x in ln.split()[:2])
                out[(f["stop"], int(f["vlen"]))] = int(ln.rsplit(":", 1)[1])
    for vlen, n in ((100000, 128), (300000, 24)):
        assert out[("2", vlen)] == n and out[("0", vlen)] == n, out
