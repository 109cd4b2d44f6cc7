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
    small = pmc_codec.Store(ctx, 4096)
    e3, rc3 = small.put([b"x" * 100, bytes(range(1, 256)) * 40, b"y" * 200])
    assert rc3[0] == 0 and rc3[1] == pmc_codec.Z_MEM_ERROR and rc3[2] == 0
    assert [g for _, g in small.get(e3, 3)][0::2] == [b"x" * 100, b"y" * 200]
    assert small.get(e3, 3)[1][0] == pmc_codec.E_ARG
