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


class LargeGolden:
    """tests/golden/large_golden.json (tests/golden/make_large_golden.py): the reference's member of every
    value of tests/large_values.py, as SHA-256 + length, keyed by the value's SHA-256."""

    def __init__(self):
        with open(os.path.join(GOLDEN, "large_golden.json")) as f:
            doc = json.load(f)
        self.vectors, self.sets = doc["vectors"], doc["sets"]

    @staticmethod
    def _sha(b):
        import hashlib
        return hashlib.sha256(b).hexdigest()

    def mismatches(self, values, members):
        """Indices whose member is not the reference's (or whose value has no vector)."""
        bad = []
        for k, (v, m) in enumerate(zip(values, members)):
            want = self.vectors.get(self._sha(v))
            if want is None or len(m) != want["gz_len"] or self._sha(m) != want["gz_sha256"]:
                bad.append(k)
        return bad


@pytest.fixture(scope="session")
def large_golden():
    return LargeGolden()
