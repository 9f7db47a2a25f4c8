import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsbo.so on cuda:0)")


@pytest.fixture(scope="session")
def gp_cases():
    d = np.load(os.path.join(GOLDEN, "gp_cases.npz"))
    names = sorted({k.split("__")[0] for k in d.files})
    return {n: {k.split("__")[1]: d[k] for k in d.files if k.startswith(n + "__")} for n in names}


@pytest.fixture(scope="session")
def c1_case():
    d = np.load(os.path.join(GOLDEN, "c1.npz"))
    return {k: d[k] for k in d.files}


@pytest.fixture(scope="session")
def contour_cases():
    import json
    with open(os.path.join(GOLDEN, "contours.json")) as f:
        return json.load(f)


def pytest_sessionstart(session):
    # the oracle is test infrastructure: make sure its .so matches its source
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
