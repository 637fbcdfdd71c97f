"""pytest setup: the `gpu` marker, import paths, shared fixtures.

`-m "not gpu"` (the CPU suite) covers: the oracle against the golden fixtures, the host-side
mirror of the reference API, and the C ABI surface of libsrhip.so (load + exported symbols).
`-m gpu` runs the parity tests proper (device vs oracle) through the C ABI on an MI355X.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "symbolicregression.jl_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (ROOT, PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libsrhip.so")


def load_cases(name):
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    n = int(z["ncases"])
    cases = []
    for i in range(n):
        pre = f"c{i}_"
        cases.append({k[len(pre):]: z[k] for k in z.files if k.startswith(pre)})
    extra = {k: z[k] for k in z.files if not k.startswith("c") or k == "ncases"}
    return cases, extra


@pytest.fixture(scope="session")
def oracle():
    import oracle as orc

    orc.load()
    return orc


@pytest.fixture(scope="session")
def ctx():
    import srhip

    return srhip.get_context(0)
