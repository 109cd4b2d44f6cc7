import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "poor-man-s-cache_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the HIP library")


class Golden:
    def __init__(self):
        z = np.load(os.path.join(GOLDEN, "golden.npz"))
        self.raw, self.raw_off, self.gz, self.gz_off = z["raw"], z["raw_off"], z["gz"], z["gz_off"]
        with open(os.path.join(GOLDEN, "golden_index.json")) as f:
            self.index = json.load(f)
        names = sorted(f for f in os.listdir(os.path.join(GOLDEN, "data")) if f.endswith(".json"))
        self.data_files = [(n, open(os.path.join(GOLDEN, "data", n), "rb").read()) for n in names]
        self.corpus = b"".join(d for _, d in self.data_files)

    def __len__(self):
        return len(self.raw_off) - 1

    def pair(self, k):
        r = self.raw[self.raw_off[k]:self.raw_off[k + 1]].tobytes()
        g = self.gz[self.gz_off[k]:self.gz_off[k + 1]].tobytes()
        return r, g

    def pairs(self):
        return [self.pair(k) for k in range(len(self))]


@pytest.fixture(scope="session")
def golden():
    return Golden()
