"""CPU: the device Huffman / emit code (pmc_trees.hpp) compiled with g++ and driven the
way the kernel drives it (tests/host/host_pipeline.cpp) reproduces every golden vector."""
import os
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def host_bin():
    d = tempfile.mkdtemp(prefix="pmc_host_")
    exe = os.path.join(d, "host_pipeline")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-o", exe,
                           os.path.join(HERE, "host", "host_pipeline.cpp")])
    return exe, d


@pytest.mark.parametrize("mode", ["v1", "v2"])
def test_host_pipeline_matches_goldens(golden, host_bin, mode):
    """v1: pmc_trees.hpp as the general kernel runs it; v2: the small kernel's formulation
    (packed-key heap, depth lengths, closed-form per-run scan_tree/send_tree)."""
    exe, d = host_bin
    src, dst = os.path.join(d, "in"), os.path.join(d, "out")
    bad = []
    for k, (r, g) in enumerate(golden.pairs()):
        with open(src, "wb") as f:
            f.write(r)
        subprocess.check_call([exe, src, dst] + (["v2"] if mode == "v2" else []))
        with open(dst, "rb") as f:
            if f.read() != g:
                bad.append(k)
    assert not bad, bad[:10]


def test_closed_form_code_tables():
    """The closed forms the kernels use for trees.c's length/distance code tables equal the
    tables zlib builds (tests/host/closed_forms_check.cpp, every entry)."""
    d = tempfile.mkdtemp(prefix="pmc_cf_")
    exe = os.path.join(d, "closed_forms_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-o", exe,
                           os.path.join(HERE, "host", "closed_forms_check.cpp")])
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
