"""ctypes bindings for the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker (never as the thing measured or shipped).

liboracle.so  : CPU restatement of zlib 1.2.11 level-9 gzip (see pmc_oracle.h).
_ref/libref_gzip.so : the reference's own GzipCompressor
                  (/root/reference/src/compressor/gzip_compressor.cpp) built by
                  `make -C oracle ref`; optional (absent if the reference was not
                  present when it was built).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None


def build(ref=True):
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    if ref and os.path.isdir("/root/reference"):
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build(ref=False)
        L = ctypes.CDLL(path)
        L.oracle_gzip_bound.restype = ctypes.c_size_t
        L.oracle_gzip_bound.argtypes = [ctypes.c_size_t]
        for fn in (L.oracle_gzip_compress, L.oracle_gzip_compress_dp):
            fn.restype = ctypes.c_size_t
            fn.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        L.oracle_gzip_decompress.restype = ctypes.c_int
        L.oracle_gzip_decompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p,
                                             ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_crc32.restype = ctypes.c_uint32
        L.oracle_crc32.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_splitmix64.restype = ctypes.c_uint64
        L.oracle_splitmix64.argtypes = [ctypes.c_uint64]
        L.oracle_gen_values.restype = None
        L.oracle_gen_values.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int,
                                        ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_gen_values_idx.restype = None
        L.oracle_gen_values_idx.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_route_keys.restype = None
        L.oracle_route_keys.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_void_p]
        _LIB = L
    return _LIB


def bound(n):
    return lib().oracle_gzip_bound(n)


def compress(data: bytes, dp=False) -> bytes:
    L = lib()
    out = ctypes.create_string_buffer(L.oracle_gzip_bound(len(data)))
    fn = L.oracle_gzip_compress_dp if dp else L.oracle_gzip_compress
    n = fn(data, len(data), out)
    return out.raw[:n]


def isize(gz: bytes) -> int:
    return int.from_bytes(gz[-4:], "little") if len(gz) >= 4 else 0


CAPACITY = -101  # ORACLE_E_CAPACITY: decoded past the buffer (never a verdict of the reference)


def decompress(gz: bytes, cap=None, grow=True):
    """Returns (rc, bytes).  rc: 0, -3 (Z_DATA_ERROR), -5 (truncated).  The first capacity guess
    is the ISIZE trailer (last 4 bytes); a stream that decodes past it is retried with the decoded
    size, as the reference's doubling buffer would hold it (gzip_compressor.cpp:71-77).  With
    grow=False a capacity overflow returns (CAPACITY, b"")."""
    L = lib()
    if cap is None:
        cap = min(max(isize(gz), 1) + 64, 1032 * len(gz) + 64)
    for _ in range(2):
        out = ctypes.create_string_buffer(max(cap, 1))
        n = ctypes.c_size_t(0)
        rc = L.oracle_gzip_decompress(gz, len(gz), out, cap, ctypes.byref(n))
        if rc != CAPACITY or not grow:
            break
        cap = n.value
    return rc, (out.raw[:n.value] if rc == 0 else b"")


def crc32(data: bytes, crc=0) -> int:
    return lib().oracle_crc32(crc, data, len(data))


class _Stats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in (
        "positions", "searches", "candidates", "literals", "matches", "blocks",
        "stored_blocks", "fixed_blocks", "dynamic_blocks")]


def last_stats():
    s = _Stats()
    lib().oracle_get_stats(ctypes.byref(s))
    return {k: getattr(s, k) for k, _ in s._fields_}


def gen_values(corpus: bytes, seed: int, kind: int, first: int, n: int, vlen: int) -> np.ndarray:
    out = np.empty((n, vlen), dtype=np.uint8)
    lib().oracle_gen_values(corpus, len(corpus), seed, kind, first, n, vlen,
                            out.ctypes.data_as(ctypes.c_void_p))
    return out


def gen_values_idx(corpus: bytes, seed: int, kind: int, index: np.ndarray, vlen: int) -> np.ndarray:
    index = np.ascontiguousarray(index, dtype=np.uint64)
    out = np.empty((len(index), vlen), dtype=np.uint8)
    lib().oracle_gen_values_idx(corpus, len(corpus), seed, kind, index.ctypes.data_as(ctypes.c_void_p),
                                len(index), vlen, out.ctypes.data_as(ctypes.c_void_p))
    return out


def route_keys(first: int, n: int, num_shards: int, n_gpus: int) -> np.ndarray:
    """hashFunc("key" + i) % num_shards % n_gpus for i in [first, first + n) (server.cpp:113)."""
    out = np.empty(n, dtype=np.uint8)
    lib().oracle_route_keys(ctypes.c_uint64(first), ctypes.c_uint64(n), num_shards, n_gpus,
                            out.ctypes.data_as(ctypes.c_void_p))
    return out


# ---------------------------------------------------------------- reference (_ref)
def ref_available():
    return os.path.exists(os.path.join(HERE, "_ref", "libref_gzip.so"))


def ref():
    global _REF
    if _REF is None:
        R = ctypes.CDLL(os.path.join(HERE, "_ref", "libref_gzip.so"))
        R.ref_compress.restype = ctypes.c_int
        R.ref_compress.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.POINTER(ctypes.c_size_t)]
        R.ref_decompress.restype = ctypes.c_int
        R.ref_decompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]
        R.ref_free.argtypes = [ctypes.c_void_p]
        R.ref_zlib_version.restype = ctypes.c_char_p
        R.ref_bench.restype = ctypes.c_int
        R.ref_bench.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_uint64)]
        R.ref_members.restype = ctypes.c_int
        R.ref_members.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_uint64, ctypes.c_void_p]
        R.ref_member_records.restype = ctypes.c_int
        R.ref_member_records.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_void_p]
        _REF = R
    return _REF


def ref_compress(s: bytes):
    """The reference GzipCompressor::Compress (strlen semantics).  Returns (rc, bytes)."""
    R = ref()
    p = ctypes.c_void_p()
    n = ctypes.c_size_t()
    rc = R.ref_compress(s, ctypes.byref(p), ctypes.byref(n))
    data = ctypes.string_at(p.value, n.value) if p.value else b""
    if p.value:
        R.ref_free(p)
    return rc, data


def ref_decompress(gz: bytes):
    """The reference GzipCompressor::Decompress.  Never call on truncated input (hangs)."""
    R = ref()
    p = ctypes.c_void_p()
    rc = R.ref_decompress(gz, len(gz), ctypes.byref(p))
    data = ctypes.string_at(p.value) if p.value else None
    if p.value:
        R.ref_free(p)
    return rc, data


def member_records_digest(lens: np.ndarray, crcs: np.ndarray, h=None):
    """Digest of a compressed set (tests/golden/full_digests.json): SHA-256 over the records
    (u32 LE member length, u32 LE CRC-32 of the member bytes), value order.  Pass `h` to feed
    a running hashlib object chunk by chunk."""
    import hashlib
    rec = np.empty((len(lens), 2), dtype="<u4")
    rec[:, 0] = lens
    rec[:, 1] = crcs
    if h is None:
        h = hashlib.sha256()
    h.update(rec.tobytes())
    return h


def ref_members_hash(values: np.ndarray, nthreads: int, h):
    """The reference Compress over every row of `values`: its members' bytes, back to back in row order, go
    into hashlib object h.  Returns the member lengths."""
    R = ref()
    n, vlen = values.shape
    stride = bound(vlen)
    dst = np.zeros((n, stride), np.uint8)
    lens = np.zeros(n, np.uint32)
    bad = R.ref_members(values.ctypes.data_as(ctypes.c_void_p), n, vlen, nthreads,
                        dst.ctypes.data_as(ctypes.c_void_p), stride, lens.ctypes.data_as(ctypes.c_void_p))
    assert bad == 0
    h.update(dst[np.arange(stride)[None, :] < lens[:, None]].tobytes())
    return lens


def ref_member_records(values: np.ndarray, nthreads: int):
    """(lens, crcs) of the reference Compress over every row of `values`."""
    R = ref()
    n, vlen = values.shape
    lens = np.zeros(n, np.uint32)
    crcs = np.zeros(n, np.uint32)
    bad = R.ref_member_records(values.ctypes.data_as(ctypes.c_void_p), n, vlen, nthreads,
                               lens.ctypes.data_as(ctypes.c_void_p), crcs.ctypes.data_as(ctypes.c_void_p))
    assert bad == 0
    return lens, crcs


def ref_bench(values: np.ndarray, nthreads: int):
    R = ref()
    n, vlen = values.shape
    tc, td = ctypes.c_double(), ctypes.c_double()
    cb = ctypes.c_uint64()
    bad = R.ref_bench(values.ctypes.data_as(ctypes.c_void_p), n, vlen, nthreads,
                      ctypes.byref(tc), ctypes.byref(td), ctypes.byref(cb))
    return {"t_compress": tc.value, "t_decompress": td.value, "compressed_bytes": cb.value, "bad": bad}
