"""GPU: one process driving several contexts (pmc_group_*, SURVEY.md §8e deployment shape).

The reference server routes key k to shard hashFunc(k) % NUM_SHARDS (server.cpp:113,121,132);
a group sends shard s to member s % n.  On the one-GPU box the members are several contexts on
device 0, which exercises the split, the per-member threads and pinned pipelines, and the merge
back into the caller's order exactly as n GPUs would.  Outputs must be the reference's bytes.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("members", [1, 2, 3])
def test_group_split_merge_bit_exact(golden, members):
    import torch  # noqa: F401
    import pmc_codec
    L = pmc_codec.lib()
    pairs = [(r, g) for r, g in golden.pairs() if r]
    n = len(pairs)
    keys = [b"key%d" % i for i in range(n)]
    kh = np.array([L.pmc_key_hash(k, len(k)) for k in keys], dtype=np.uint64)
    g = ctypes.c_void_p()
    devs = (ctypes.c_int * members)(*([0] * members))
    assert L.pmc_group_create(devs, members, ctypes.byref(g)) == 0
    try:
        route = np.zeros(n, dtype=np.uint32)
        assert L.pmc_group_route(g, kh.ctypes.data, 128, n, route.ctypes.data) == 0
        assert (route == (kh % np.uint64(128)) % np.uint64(members)).all()
        assert len(set(route.tolist())) == members  # every member gets a share
        src = b"".join(r for r, _ in pairs)
        slen = np.array([len(r) for r, _ in pairs], dtype=np.uint32)
        soff = np.concatenate([[0], np.cumsum(slen[:-1], dtype=np.uint64)]).astype(np.uint64)
        cap = np.array([pmc_codec.gzip_bound(int(x)) for x in slen], dtype=np.uint32)
        # outputs at permuted, gapped offsets of the caller's buffer
        perm = np.random.default_rng(members).permutation(n)
        doff = np.zeros(n, dtype=np.uint64)
        doff[perm] = np.concatenate([[0], np.cumsum(cap[perm][:-1].astype(np.uint64) + 3)])
        dst = ctypes.create_string_buffer(int(doff.max() + cap.max()) + 64)
        dlen = np.zeros(n, dtype=np.uint32)
        rc = np.full(n, 7, dtype=np.int32)
        assert L.pmc_group_compress_batch(g, src, soff.ctypes.data, slen.ctypes.data, kh.ctypes.data, 128, n, dst,
                                          doff.ctypes.data, cap.ctypes.data, dlen.ctypes.data, rc.ctypes.data,
                                          int(slen.max())) == 0
        raw = dst.raw
        assert (rc == 0).all()
        bad = [i for i, (_, gz) in enumerate(pairs) if raw[int(doff[i]):int(doff[i]) + int(dlen[i])] != gz]
        assert not bad, bad[:10]
        # and back: members in index order, values to their own slots
        mem = b"".join(gz for _, gz in pairs)
        mlen = np.array([len(gz) for _, gz in pairs], dtype=np.uint32)
        moff = np.concatenate([[0], np.cumsum(mlen[:-1], dtype=np.uint64)]).astype(np.uint64)
        out = ctypes.create_string_buffer(int(slen.sum()) + 64)
        olen = np.zeros(n, dtype=np.uint32)
        orc = np.full(n, 7, dtype=np.int32)
        assert L.pmc_group_decompress_batch(g, mem, moff.ctypes.data, mlen.ctypes.data, kh.ctypes.data, 128, n, out,
                                            soff.ctypes.data, slen.ctypes.data, olen.ctypes.data, orc.ctypes.data,
                                            int(slen.max())) == 0
        assert (orc == 0).all() and (olen == slen).all()
        assert out.raw[:len(src)] == src
    finally:
        L.pmc_group_destroy(g)
