"""CPU: the C-ABI library loads and exports every entry point include/pmc_codec.h declares,
the drop-in exports the reference's GzipCompressor symbols, and the device code object is
gfx950.  No compute calls (no GPU here)."""
import ctypes
import os
import re
import subprocess

import pmc_codec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "pmc_codec.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pmc_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 15
    L = pmc_codec.lib()
    for n in names:
        assert hasattr(L, n), n
        assert n in pmc_codec.SIGNATURES, n


def test_bound_matches_oracle():
    from oracle import pyoracle as O
    ns = (0, 1, 29, 1024, 16382, 16383, 16384, 65536, 10 ** 6, 2 ** 31)
    for n in ns:
        assert pmc_codec.gzip_bound(n) == O.bound(n)
    assert pmc_codec.gzip_bounds(ns).tolist() == [pmc_codec.gzip_bound(n) for n in ns]


def test_isize_helper():
    L = pmc_codec.lib()
    blob = b"\x1f\x8b" + b"\0" * 12 + (1234).to_bytes(4, "little")
    assert L.pmc_gzip_isize(blob, len(blob)) == 1234
    assert L.pmc_gzip_isize(b"short", 5) == 0


def test_dropin_exports_reference_class():
    out = subprocess.check_output(["nm", "-DC", pmc_codec.DROPIN_PATH]).decode()
    assert "GzipCompressor::Compress(char const*)" in out
    assert "GzipCompressor::Decompress(char const*, unsigned long)" in out


def test_device_code_is_gfx950():
    data = open(pmc_codec.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"gfx942" not in data and b"sm_" not in data[:0]  # single target, no CUDA


def test_no_gpu_fails_loudly_or_works():
    """Without a gfx950 device the context must refuse (never silently fall back)."""
    import torch
    if torch.cuda.is_available():
        return
    h = ctypes.c_void_p()
    rc = pmc_codec.lib().pmc_ctx_create(0, ctypes.byref(h))
    assert rc == pmc_codec.E_NO_DEVICE


def test_pinned_batch_rejects_bad_arguments_without_touching_a_device():
    """pmc_gzip_*_batch_pinned validate before any HIP call: NULL context or arrays -> PMC_E_ARG."""
    L = pmc_codec.lib()
    buf = ctypes.create_string_buffer(64)
    for fn in (L.pmc_gzip_compress_batch_pinned, L.pmc_gzip_decompress_batch_pinned):
        assert fn(None, buf, buf, buf, 1, buf, None, buf, buf, buf, 16, 0) == pmc_codec.E_ARG
        assert fn(None, None, None, None, 0, None, None, None, None, None, 0, 0) == pmc_codec.E_ARG


def test_host_key_hash_matches_reference_hash():
    """pmc_key_hash (host side of the group route) equals the reference's own hashFunc
    (tests/golden/route_golden.npz, from /root/reference/src/hash) -- a host function, no device."""
    import numpy as np
    z = np.load(os.path.join(ROOT, "tests", "golden", "route_golden.npz"))
    L = pmc_codec.lib()
    for i, h in zip(z["index"], z["hash"]):
        k = b"key%d" % int(i)
        assert L.pmc_key_hash(k, len(k)) == int(h), int(i)
    # keys of every length 0..70 -- the 16-byte block loop and every tail length, bytes up to 0xff --
    # against the reference's hashFunc too (make_route_golden.py), and the oracle's restatement
    from oracle import pyoracle as O
    O.lib().oracle_murmur3_x64_128_h1.restype = ctypes.c_uint64
    O.lib().oracle_murmur3_x64_128_h1.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32]
    blob, off, kh = z["key_blob"].tobytes(), z["key_off"], z["key_hash"]
    assert {int(off[i + 1] - off[i]) for i in range(len(kh))} == set(range(71))
    for i in range(len(kh)):
        k = blob[int(off[i]):int(off[i + 1])]
        assert L.pmc_key_hash(k, len(k)) == int(kh[i]), (len(k), k)
        assert O.lib().oracle_murmur3_x64_128_h1(k, len(k), 0) == int(kh[i]), (len(k), k)
