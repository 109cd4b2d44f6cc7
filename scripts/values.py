"""The SURVEY §8d value generator for the measurement scripts, run by the product library on the device
(pmc_gen_values, the generator bench.py uses) and copied back: scripts time the codec on these values and
load nothing from oracle/ to make them."""
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def corpus_bytes():
    d = os.path.join(ROOT, "tests", "golden", "data")
    return b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.endswith(".json"))


def gen_values(n, vlen, seed=0x5EED, kind=0, index0=0):
    """n values of vlen bytes (indices index0 .., generator kind 0 JSON slices / 1 alnum) as bytes objects."""
    import pmc_codec
    from pmc_codec import device as D
    L = pmc_codec.lib()
    cb = corpus_bytes()
    corpus = torch.frombuffer(bytearray(cb), dtype=torch.uint8).cuda()
    out = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
    assert L.pmc_gen_values(corpus.data_ptr(), len(cb), seed, kind, index0, None, n, vlen, out.data_ptr(),
                            D.stream_handle()) == 0
    torch.cuda.synchronize()
    raw = out[:n * vlen].cpu().numpy().tobytes()
    return [raw[i * vlen:(i + 1) * vlen] for i in range(n)]
