"""pmc_codec -- Python host mirror of the MI355X value codec.

Mirrors the reference's codec interface (/root/reference/src/compressor/gzip_compressor.hpp:
CompressResult / DecompressResult / GzipCompressor::Compress / ::Decompress, codes
INVALID_INPUT=-999, OPERATION_SUCCESS=0) on top of the C-ABI in include/pmc_codec.h,
plus the batched device-resident API the GPU hot path is measured through.

The HIP library (libpmc_codec.so, built for gfx950) is REQUIRED: importing works without a
GPU (so the CPU test suite can check exports), but every compute call raises
CodecUnavailable when no gfx950 device/context is available.  There is no CPU fallback.
"""
import ctypes
import os
from dataclasses import dataclass
from typing import Optional

HERE = os.path.dirname(os.path.abspath(__file__))
# PMC_LIB selects a diagnostic build (e.g. libpmc_codec_stamps.so); default is the product
LIB_PATH = os.path.join(HERE, os.environ.get("PMC_LIB", "libpmc_codec.so"))
DROPIN_PATH = os.path.join(HERE, "libgzip_dropin.so")

CHUNK_SIZE = 16384
INVALID_INPUT = -999
OPERATION_SUCCESS = 0
Z_DATA_ERROR = -3
Z_MEM_ERROR = -4
Z_BUF_ERROR = -5
E_NO_DEVICE = -100
E_CAPACITY = -101
E_ARG = -102


class CodecUnavailable(RuntimeError):
    pass


_lib = None

_c = ctypes
_p = ctypes.c_void_p
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64

# name -> (restype, argtypes) for every function in include/pmc_codec.h
SIGNATURES = {
    "pmc_ctx_create": (_c.c_int, [_c.c_int, _c.POINTER(_p)]),
    "pmc_ctx_destroy": (None, [_p]),
    "pmc_default_ctx": (_p, []),
    "pmc_last_error": (_c.c_char_p, []),
    "pmc_version": (_c.c_char_p, []),
    "pmc_gzip_bound": (_c.c_size_t, [_c.c_size_t]),
    "pmc_gzip_compress": (_c.c_int, [_p, _p, _c.c_size_t, _p, _c.c_size_t, _c.POINTER(_c.c_size_t)]),
    "pmc_gzip_decompress": (_c.c_int, [_p, _p, _c.c_size_t, _p, _c.c_size_t, _c.POINTER(_c.c_size_t)]),
    "pmc_gzip_isize": (_u32, [_p, _c.c_size_t]),
    "pmc_gzip_compress_batch": (_c.c_int, [_p, _p, _p, _p, _u32, _p, _p, _p, _p, _p, _u32, _p]),
    "pmc_gzip_decompress_batch": (_c.c_int, [_p, _p, _p, _p, _u32, _p, _p, _p, _p, _p, _u32, _p]),
    "pmc_gzip_isize_batch": (_c.c_int, [_p, _p, _p, _p, _u32, _p, _p]),
    "pmc_crc32_batch": (_c.c_int, [_p, _p, _p, _p, _u32, _p, _p]),
    "pmc_gzip_compress_batch_host": (_c.c_int, [_p, _p, _p, _p, _u32, _p, _p, _p, _p, _p]),
    "pmc_gzip_decompress_batch_host": (_c.c_int, [_p, _p, _p, _p, _u32, _p, _p, _p, _p, _p]),
    "pmc_gzip_compress_batch_pinned": (_c.c_int, [_p, _p, _p, _p, _u32, _p, _p, _p, _p, _p, _u32, _u32]),
    "pmc_gzip_decompress_batch_pinned": (_c.c_int, [_p, _p, _p, _p, _u32, _p, _p, _p, _p, _p, _u32, _u32]),
    "pmc_store_create": (_c.c_int, [_p, _u64, _c.POINTER(_p)]),
    "pmc_store_destroy": (None, [_p]),
    "pmc_store_put_batch": (_c.c_int, [_p, _p, _p, _p, _u32, _p, _p]),
    "pmc_store_get_batch": (_c.c_int, [_p, _p, _u32, _c.c_int, _p, _p, _p]),
    "pmc_store_get_batch_frames": (_c.c_int, [_p, _p, _u32, _p, _p, _p, _p]),
    "pmc_store_read_members": (_c.c_int, [_p, _p, _u32, _p, _p]),
    "pmc_store_free": (_c.c_int, [_p, _p, _u32]),
    "pmc_store_stats": (_c.c_int, [_p, _c.POINTER(_u64), _c.POINTER(_u64), _c.POINTER(_u64)]),
    "pmc_slab_create": (_c.c_int, [_p, _u32, _u32, _c.POINTER(_p)]),
    "pmc_slab_destroy": (None, [_p]),
    "pmc_slab_data": (_p, [_p]),
    "pmc_slab_lengths": (_p, [_p]),
    "pmc_slab_stride": (_u64, [_p]),
    "pmc_slab_set": (_c.c_int, [_p, _p, _p, _p, _p, _u32, _p, _p]),
    "pmc_slab_get": (_c.c_int, [_p, _p, _u32, _p, _p, _p, _p, _p, _p]),
    "pmc_key_hash": (_u64, [_c.c_char_p, _c.c_size_t]),
    "pmc_group_create": (_c.c_int, [_c.POINTER(_c.c_int), _c.c_int, _c.POINTER(_p)]),
    "pmc_group_destroy": (None, [_p]),
    "pmc_group_size": (_c.c_int, [_p]),
    "pmc_group_route": (_c.c_int, [_p, _p, _u32, _u32, _p]),
    "pmc_group_compress_batch": (_c.c_int, [_p, _p, _p, _p, _p, _u32, _u32, _p, _p, _p, _p, _p, _u32]),
    "pmc_group_decompress_batch": (_c.c_int, [_p, _p, _p, _p, _p, _u32, _u32, _p, _p, _p, _p, _p, _u32]),
    "pmc_gen_values": (_c.c_int, [_p, _u32, _u64, _c.c_int, _u64, _p, _u32, _u32, _p, _p]),
    "pmc_fill_layout": (_c.c_int, [_p, _p, _p, _u32, _u64, _u32, _u32, _p]),
    "pmc_compare_values": (_c.c_int, [_p, _p, _p, _p, _p, _p, _u32, _p, _p]),
    "pmc_route_keys": (_c.c_int, [_u64, _u32, _u32, _u32, _p, _p]),
    "pmc_debug_stamps": (_c.c_int, [_p, _p]),
    "pmc_ctx_profile": (_c.c_int, [_p, _c.c_int]),
    "pmc_ctx_kernel_times": (_c.c_int, [_p, _c.POINTER(_c.c_double), _c.POINTER(_u32), _c.c_int]),
    "pmc_ctx_guard_counts": (_c.c_int, [_p, _c.POINTER(_u32)]),
    "pmc_ctx_path_counts": (_c.c_int, [_p, _c.POINTER(_u64)]),
    "pmc_ctx_latency_redone": (_c.c_int, [_p, _c.POINTER(_u64)]),
}

# pmc_ctx_kernel_times kinds (include/pmc_codec.h PMC_K_*)
KERNEL_KINDS = ["deflate_front", "deflate_trees", "deflate_back", "deflate_mono", "deflate_hbm", "inflate_lds",
                "inflate_hbm", "inflate_lane", "inflate_verify", "order", "inflate_rec", "deflate_large",
                "deflate_large_emit"]
KERNEL_NAMES = {"deflate_front": "pmc::deflate_front_kernel", "deflate_trees": "pmc::deflate_trees_kernel",
                "deflate_back": "pmc::deflate_back_kernel", "deflate_mono": "pmc::deflate_small_kernel",
                "deflate_hbm": "pmc::deflate_kernel<true>", "inflate_lds": "pmc::inflate_kernel<false>",
                "inflate_hbm": "pmc::inflate_kernel<true>", "inflate_lane": "pmc::inflate_lane_kernel",
                "inflate_verify": "pmc::inflate_verify_kernel", "order": "pmc::order_{hist,scan,scatter}_kernel",
                "inflate_rec": "pmc::inflate_rec_kernel", "deflate_large": "pmc::lv_*_kernel",
                "deflate_large_emit": "pmc::deflate_lv_emit_kernel"}


def lib():
    """Load libpmc_codec.so (fails loudly if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CodecUnavailable(f"{LIB_PATH} missing: run `make -C poor-man-s-cache_amd` "
                                   "(hipcc --offload-arch=gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if "PMC_LIB" in os.environ and not hasattr(L, name):
                continue  # an older diagnostic build (A/B runs) may predate an entry point
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def source_id() -> str:
    """SHA-256 (16 hex) of the HIP library's sources (csrc/*.hip, csrc/*.hpp, include/pmc_codec.h):
    stamps PMC-derived artifacts (profiles/*/traffic.json) so bench.py only quotes measurements
    taken on the kernels it is running."""
    import hashlib
    pkg = os.path.dirname(HERE)
    csrc = os.path.join(pkg, "csrc")
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".hpp")))
    files.append(os.path.join(os.path.dirname(pkg), "include", "pmc_codec.h"))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def last_error() -> str:
    return lib().pmc_last_error().decode()


def gzip_bound(n: int) -> int:
    return lib().pmc_gzip_bound(n)


def gzip_bounds(lengths):
    """pmc_gzip_bound of every length (numpy): the same closed form (csrc/pmc_kernels.hpp gzip_bound,
    = oracle_gzip_bound; tests/test_abi.py checks them equal), without a C call per value."""
    import numpy as np
    n = np.asarray(lengths, dtype=np.uint64)
    return (n + (n >> np.uint64(3)) + np.uint64(6) * (n // np.uint64(16383) + np.uint64(1)) + np.uint64(32)).astype(np.uint32)


def decompress_capacity(member: bytes) -> int:
    """Output capacity for one gzip member: its ISIZE trailer, clamped to DEFLATE's
    1032:1 maximum expansion (a larger ISIZE cannot belong to a valid member)."""
    isz = int.from_bytes(member[-4:], "little") if len(member) >= 18 else 0
    return min(isz, 1032 * len(member) + 64)


class Context:
    """One device: stream, symbol slabs, HBM working sets, pinned staging."""

    def __init__(self, device: int = 0):
        self.handle = _p()
        rc = lib().pmc_ctx_create(device, ctypes.byref(self.handle))
        if rc != 0:
            raise CodecUnavailable(f"pmc_ctx_create({device}) = {rc}: {last_error()}")
        self.device = device
        import weakref
        self._deps = weakref.WeakSet()  # stores / slabs on this context: closed before it

    def profile(self, enable: bool):
        """Bracket every kernel the batched calls enqueue with HIP events (diagnostics)."""
        lib().pmc_ctx_profile(self.handle, 1 if enable else 0)

    def kernel_times(self):
        """{kind: (total_ms, launches)} of the launches recorded since profile(True)."""
        n = len(KERNEL_KINDS)
        ms = (ctypes.c_double * n)()
        cnt = (_u32 * n)()
        rc = lib().pmc_ctx_kernel_times(self.handle, ms, cnt, n)
        if rc != 0:
            raise CodecUnavailable(f"pmc_ctx_kernel_times failed ({rc}): {last_error()}")
        return {KERNEL_KINDS[k]: (ms[k], cnt[k]) for k in range(n) if cnt[k]}

    def guard_counts(self):
        """Guard counters {sort, codes, probe, retry, inflate_retry} (include/pmc_codec.h pmc_ctx_guard_counts)."""
        c = (_u32 * 5)()
        rc = lib().pmc_ctx_guard_counts(self.handle, c)
        if rc != 0:
            raise CodecUnavailable(f"pmc_ctx_guard_counts failed ({rc}): {last_error()}")
        return {"sort": c[0], "codes": c[1], "probe": c[2], "retry": c[3], "inflate_retry": c[4]}

    def path_counts(self):
        """Host-call routes taken so far {latency_compress, latency_decompress, pipeline_compress,
        pipeline_decompress} (include/pmc_codec.h pmc_ctx_path_counts)."""
        c = (_u64 * 4)()
        rc = lib().pmc_ctx_path_counts(self.handle, c)
        if rc != 0:
            raise CodecUnavailable(f"pmc_ctx_path_counts failed ({rc})")
        return {"latency_compress": c[0], "latency_decompress": c[1], "pipeline_compress": c[2],
                "pipeline_decompress": c[3]}

    def latency_redone(self):
        """Latency-path compress calls whose declined values a pipeline call redid (include/pmc_codec.h
        pmc_ctx_latency_redone)."""
        c = _u64(0)
        rc = lib().pmc_ctx_latency_redone(self.handle, ctypes.byref(c))
        if rc != 0:
            raise CodecUnavailable(f"pmc_ctx_latency_redone failed ({rc})")
        return c.value

    def close(self):
        if self.handle:
            for d in list(getattr(self, "_deps", ())):
                d.close()
            lib().pmc_ctx_destroy(self.handle)
            self.handle = _p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------- host-resident batches (pinned H2D -> GPU -> D2H) --------------
    def compress_many(self, values):
        """values: list of bytes -> list of (rc, gzip bytes)."""
        return self._host_batch(values, True)

    def decompress_many(self, members, caps=None):
        """members: list of gzip bytes -> list of (rc, bytes).  caps default: ISIZE."""
        return self._host_batch(members, False, caps)

    def _host_batch(self, items, compress, caps=None):
        import numpy as np
        n = len(items)
        if n == 0:
            return []
        L = lib()
        src = b"".join(items)
        src_len = np.fromiter(map(len, items), dtype=np.uint32, count=n)
        src_off = np.zeros(n, dtype=np.uint64)
        src_off[1:] = np.cumsum(src_len[:-1], dtype=np.uint64)
        if compress:
            cap = gzip_bounds(src_len)
        elif caps is not None:
            cap = np.asarray(caps, dtype=np.uint32)
        else:
            cap = np.fromiter(map(decompress_capacity, items), dtype=np.uint32, count=n)
        dst_off = np.zeros(n, dtype=np.uint64)
        dst_off[1:] = np.cumsum(cap[:-1], dtype=np.uint64)
        dst = np.empty(int(cap.sum()) + 1, dtype=np.uint8)
        dst_len = np.zeros(n, dtype=np.uint32)
        rc = np.zeros(n, dtype=np.int32)
        fn = L.pmc_gzip_compress_batch_host if compress else L.pmc_gzip_decompress_batch_host
        r = fn(self.handle, src, src_off.ctypes.data, src_len.ctypes.data, n, dst.ctypes.data, dst_off.ctypes.data,
               cap.ctypes.data, dst_len.ctypes.data, rc.ctypes.data)
        if r != 0:
            raise CodecUnavailable(f"batch call failed {r}: {last_error()}")
        mv = memoryview(dst)
        offs, lens, rcs = dst_off.tolist(), dst_len.tolist(), rc.tolist()
        res = [(c, mv[o:o + ln].tobytes() if c == 0 else b"") for c, o, ln in zip(rcs, offs, lens)]
        if not compress and caps is None:
            # bytes after a member misstated its size (the reference ignores them,
            # gzip_compressor.cpp:96): PMC_E_CAPACITY carries the decoded size; decode those again
            again = [i for i in range(n) if rcs[i] == E_CAPACITY and lens[i] > int(cap[i])]
            if again:
                redo = self._host_batch([items[i] for i in again], False, [lens[i] for i in again])
                for i, r in zip(again, redo):
                    res[i] = r
        return res

    # ---------------- device-resident batches (the hot path) ------------------------
    def compress_device(self, src, src_off, src_len, dst, dst_off, dst_cap, dst_len, rc, max_len, stream=0):
        """All tensor arguments are torch CUDA tensors (or raw device pointers as int)."""
        r = lib().pmc_gzip_compress_batch(self.handle, _ptr(src), _ptr(src_off), _ptr(src_len), _n(src_len),
                                          _ptr(dst), _ptr(dst_off), _ptr(dst_cap), _ptr(dst_len), _ptr(rc),
                                          max_len, stream)
        if r != 0:
            raise CodecUnavailable(f"pmc_gzip_compress_batch = {r}: {last_error()}")

    def decompress_device(self, src, src_off, src_len, dst, dst_off, dst_cap, dst_len, rc, max_len, stream=0):
        r = lib().pmc_gzip_decompress_batch(self.handle, _ptr(src), _ptr(src_off), _ptr(src_len), _n(src_len),
                                            _ptr(dst), _ptr(dst_off), _ptr(dst_cap), _ptr(dst_len), _ptr(rc),
                                            max_len, stream)
        if r != 0:
            raise CodecUnavailable(f"pmc_gzip_decompress_batch = {r}: {last_error()}")

    # ---------------- pinned host batches, pipelined over copy streams --------------
    def compress_pinned(self, src, src_off, src_len, dst, dst_off, dst_cap, dst_len, rc, max_len, chunk=0):
        """All tensor arguments are pinned CPU tensors (torch pin_memory=True)."""
        r = lib().pmc_gzip_compress_batch_pinned(self.handle, _ptr(src), _ptr(src_off), _ptr(src_len),
                                                 _n(src_len), _ptr(dst), _ptr(dst_off), _ptr(dst_cap),
                                                 _ptr(dst_len), _ptr(rc), max_len, chunk)
        if r != 0:
            raise CodecUnavailable(f"pmc_gzip_compress_batch_pinned = {r}: {last_error()}")

    def decompress_pinned(self, src, src_off, src_len, dst, dst_off, dst_cap, dst_len, rc, max_len, chunk=0):
        r = lib().pmc_gzip_decompress_batch_pinned(self.handle, _ptr(src), _ptr(src_off), _ptr(src_len),
                                                   _n(src_len), _ptr(dst), _ptr(dst_off), _ptr(dst_cap),
                                                   _ptr(dst_len), _ptr(rc), max_len, chunk)
        if r != 0:
            raise CodecUnavailable(f"pmc_gzip_decompress_batch_pinned = {r}: {last_error()}")


def _ptr(t):
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def _n(t):
    return t.numel() if hasattr(t, "numel") else int(t)


_default: Optional[Context] = None


def default_context() -> Context:
    global _default
    if _default is None:
        _default = Context(0)
    return _default


# ------------------------------------------------------------ device-resident store (f2/f3)
class Extent(ctypes.Structure):
    """pmc_extent (include/pmc_codec.h)."""
    _fields_ = [("off", _u64), ("cap", _u32), ("len", _u32), ("raw_len", _u32), ("flags", _u32)]


FRAME_RAW, FRAME_CUSTOM, FRAME_RESP = 0, 1, 2


class Store:
    """Compressed values kept in an HBM heap: put(values) -> extents, get(extents, frame) -> responses."""

    def __init__(self, ctx: Context, heap_bytes: int = 0):
        self.ctx = ctx
        self.handle = _p()
        rc = lib().pmc_store_create(ctx.handle, heap_bytes, ctypes.byref(self.handle))
        if rc != 0:
            raise CodecUnavailable(f"pmc_store_create = {rc}: {last_error()}")
        ctx._deps.add(self)

    def put(self, values):
        """values: list of bytes -> (Extent array, rc list)."""
        import numpy as np
        n = len(values)
        ext = (Extent * max(n, 1))()
        rc = np.zeros(max(n, 1), dtype=np.int32)
        if n:
            lens = np.array([len(v) for v in values], dtype=np.uint32)
            off = np.zeros(n, dtype=np.uint64)
            off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            r = lib().pmc_store_put_batch(self.handle, b"".join(values), off.ctypes.data, lens.ctypes.data, n,
                                          ext, rc.ctypes.data)
            if r != 0:
                raise CodecUnavailable(f"pmc_store_put_batch = {r}: {last_error()}")
        return ext, [int(x) for x in rc[:n]]

    def get(self, ext, n=None, frame=FRAME_RAW):
        """-> list of (rc, response bytes).  frame: one FRAME_* for the batch, or a sequence of n
        (pmc_store_get_batch_frames)."""
        import numpy as np
        n = len(ext) if n is None else n
        if n == 0:
            return []
        resp = (_p * n)()
        rlen = np.zeros(n, dtype=np.uint32)
        rc = np.zeros(n, dtype=np.int32)
        if isinstance(frame, int):
            r = lib().pmc_store_get_batch(self.handle, ext, n, frame, resp, rlen.ctypes.data, rc.ctypes.data)
        else:
            fr = np.ascontiguousarray(frame, dtype=np.uint8)
            assert fr.shape == (n,), fr.shape
            r = lib().pmc_store_get_batch_frames(self.handle, ext, n, fr.ctypes.data, resp, rlen.ctypes.data,
                                                 rc.ctypes.data)
        if r != 0:
            raise CodecUnavailable(f"pmc_store_get_batch = {r}: {last_error()}")
        return [(int(rc[i]), ctypes.string_at(resp[i], int(rlen[i])) if rc[i] == 0 else b"") for i in range(n)]

    def members(self, ext, n=None):
        import numpy as np
        n = len(ext) if n is None else n
        lens = [ext[i].len for i in range(n)]
        off = np.zeros(max(n, 1), dtype=np.uint64)
        if n > 1:
            off[1:n] = np.cumsum(lens[:-1], dtype=np.uint64)
        buf = ctypes.create_string_buffer(sum(lens) + 1)
        r = lib().pmc_store_read_members(self.handle, ext, n, buf, off.ctypes.data)
        if r != 0:
            raise CodecUnavailable(f"pmc_store_read_members = {r}: {last_error()}")
        raw = buf.raw
        return [raw[int(off[i]):int(off[i]) + lens[i]] for i in range(n)]

    def free(self, ext, n=None):
        lib().pmc_store_free(self.handle, ext, len(ext) if n is None else n)

    def stats(self):
        u, r, h = _u64(), _u64(), _u64()
        lib().pmc_store_stats(self.handle, ctypes.byref(u), ctypes.byref(r), ctypes.byref(h))
        return {"used": u.value, "reserved": r.value, "heap": h.value}

    def close(self):
        if self.handle:
            lib().pmc_store_destroy(self.handle)
            self.handle = _p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Slab:
    """Fixed-slot device slab (pmc_slab_*): set(values -> slots), get(slots -> values), all device
    tensors, enqueue-only on a stream."""

    def __init__(self, ctx: Context, slots: int, max_value_len: int):
        self.ctx = ctx
        self.handle = _p()
        rc = lib().pmc_slab_create(ctx.handle, slots, max_value_len, ctypes.byref(self.handle))
        if rc != 0:
            raise CodecUnavailable(f"pmc_slab_create = {rc}: {last_error()}")
        ctx._deps.add(self)
        self.stride = lib().pmc_slab_stride(self.handle)
        self.slots = slots

    def set(self, src, src_off, src_len, slot, rc, stream=0):
        r = lib().pmc_slab_set(self.handle, _ptr(src), _ptr(src_off), _ptr(src_len), _ptr(slot), _n(slot), _ptr(rc),
                               stream)
        if r != 0:
            raise CodecUnavailable(f"pmc_slab_set = {r}: {last_error()}")

    def get(self, slot, dst, dst_off, dst_cap, dst_len, rc, stream=0):
        r = lib().pmc_slab_get(self.handle, _ptr(slot), _n(slot), _ptr(dst), _ptr(dst_off), _ptr(dst_cap),
                               _ptr(dst_len), _ptr(rc), stream)
        if r != 0:
            raise CodecUnavailable(f"pmc_slab_get = {r}: {last_error()}")

    def data_ptr(self):
        return lib().pmc_slab_data(self.handle)

    def lengths_ptr(self):
        return lib().pmc_slab_lengths(self.handle)

    def close(self):
        if self.handle:
            lib().pmc_slab_destroy(self.handle)
            self.handle = _p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------ reference mirror
@dataclass
class CompressResult:
    """gzip_compressor.hpp:16-23"""
    data: Optional[bytes]
    size: int
    operationResult: int


@dataclass
class DecompressResult:
    """gzip_compressor.hpp:26-31 (data is the NUL-free payload, as a C string would read)"""
    data: Optional[bytes]
    operationResult: int


class GzipCompressor:
    """Static-method mirror of the reference class (gzip_compressor.hpp:33-44)."""

    @staticmethod
    def Compress(input: Optional[bytes]) -> CompressResult:
        # gzip_compressor.cpp:4,6 -- null/empty rejected; the value is a C string (strlen)
        if input is None:
            return CompressResult(None, 0, INVALID_INPUT)
        s = bytes(input).split(b"\0", 1)[0]
        if not s:
            return CompressResult(None, 0, INVALID_INPUT)
        rc, out = default_context().compress_many([s])[0]
        if rc != 0:
            return CompressResult(None, 0, rc)
        return CompressResult(out, len(out), OPERATION_SUCCESS)

    @staticmethod
    def Decompress(input: Optional[bytes], input_size: int) -> DecompressResult:
        # gzip_compressor.cpp:53 -- null or size 0 rejected
        if input is None or input_size == 0:
            return DecompressResult(None, INVALID_INPUT)
        data = bytes(input[:input_size])
        rc, out = default_context().decompress_many([data])[0]
        if rc != 0:
            return DecompressResult(None, rc)
        return DecompressResult(out, OPERATION_SUCCESS)
