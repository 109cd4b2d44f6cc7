"""Driver for scripts/phase_cost.sh: one compress launch over N device-generated values
(PMC_LIB / PMC_STOP_AFTER from the environment)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poor-man-s-cache_amd")]
import torch  # noqa: E402

import pmc_codec  # noqa: E402
from pmc_codec import device as D  # noqa: E402


def main():
    n, vlen, kind = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    L = pmc_codec.lib()
    ctx = pmc_codec.Context(0)
    d = os.path.join(ROOT, "tests", "golden", "data")
    corpus_b = b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)))
    corpus = torch.frombuffer(bytearray(corpus_b), dtype=torch.uint8).cuda()
    data = torch.empty(n * vlen + 16, dtype=torch.uint8, device="cuda")
    L.pmc_gen_values(corpus.data_ptr(), len(corpus_b), 0x5EED if kind == 0 else 0xA1B2, kind, 0, None, n, vlen,
                     data.data_ptr(), D.stream_handle())
    off = torch.arange(n, dtype=torch.int64, device="cuda") * vlen
    lens = torch.full((n,), vlen, dtype=torch.int32, device="cuda")
    out, rc = D.compress(ctx, D.Batch(data, off, lens, n, vlen))
    torch.cuda.synchronize()
    if os.environ.get("PMC_DRIVE_DECOMPRESS"):
        D.decompress(ctx, out, [vlen] * n)
        torch.cuda.synchronize()
    ctx.close()


if __name__ == "__main__":
    main()
