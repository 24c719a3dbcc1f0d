import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device and the built HIP library")


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """Print every recorded parity error next to its bound; write them to $PARITY_LOG."""
    try:
        from parity import RESULTS
    except ImportError:
        return
    if not RESULTS:
        return
    tr = terminalreporter
    tr.section("parity: achieved error vs bound")
    for r in RESULTS:
        tr.write_line(f"{r['err']:.3e} < {r['bound']:.1e}  {r['test']}  {r['what']}")
    path = os.environ.get("PARITY_LOG")
    if path:
        import json
        with open(path, "w") as f:
            json.dump(RESULTS, f, indent=1)
