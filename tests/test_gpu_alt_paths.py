"""GPU: the codec's alternate paths stay bit-exact.  The C-ABI reads its path switches once per
process (PMC_DEFLATE_MONO: single-kernel small-value compress; PMC_DEFLATE_V1: the general
kernels for every size; PMC_BIG_PASS=1: the split pipeline's large pass for 16383..31808-byte values
instead of the large-value pipeline; PMC_INFLATE_WAVE: wave-per-member decode only; PMC_INFLATE_REC=0: the
lane kernel for members of every size instead of the record kernel; PMC_TREES_ORDER=0 /
PMC_INFLATE_ORDER=0: lanes in index order), so each switch runs every golden vector through
compress and decompress in a child process of its own, one after the other."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

CHILD = r"""
import sys
sys.path[:0] = [sys.argv[1]]
from conftest import Golden
import pmc_codec
from pmc_codec import device as D
import torch
g = Golden()
pairs = g.pairs()
ctx = pmc_codec.Context(0)
out, rc = D.compress(ctx, D.pack([r for r, _ in pairs]))
torch.cuda.synchronize()
rc = rc.cpu().numpy()
got = out.host_items()
bad = [k for k, (r, z) in enumerate(pairs) if rc[k] != 0 or got[k] != z]
caps = [max(len(r), 1) for r, _ in pairs]
back, brc = D.decompress(ctx, D.pack([z for _, z in pairs]), caps)
torch.cuda.synchronize()
brc = brc.cpu().numpy()
items = back.host_items()
bad += [k for k, (r, _) in enumerate(pairs) if brc[k] != 0 or items[k] != r]
ctx.close()
print("bad", len(bad), bad[:8])
sys.exit(1 if bad else 0)
"""


@pytest.mark.gpu
@pytest.mark.parametrize("switch", ["PMC_DEFLATE_MONO=1", "PMC_DEFLATE_V1=1", "PMC_BIG_PASS=1", "PMC_INFLATE_WAVE=1",
                                    "PMC_INFLATE_REC=0", "PMC_TREES_ORDER=0", "PMC_INFLATE_ORDER=0"])
def test_alternate_path_goldens(switch):
    k, v = switch.split("=")
    env = dict(os.environ, **{k: v})
    out = subprocess.run([sys.executable, "-c", CHILD, HERE], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
