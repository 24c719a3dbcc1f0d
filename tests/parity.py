"""Parity bookkeeping for the -m gpu tests: every error bound a test asserts is
recorded with the error actually achieved, printed at the end of the session and
written to $PARITY_LOG (JSON) when set, so the bounds can be tightened against
measured values (bounds are ~2x the measured error on the GPU box)."""
import os

import numpy as np
import torch

RESULTS = []


def relerr(a, b) -> float:
    """Relative Frobenius error ||a - b|| / ||b|| in float64."""
    a = torch.as_tensor(np.asarray(a.detach().cpu() if torch.is_tensor(a) else a)).double()
    b = torch.as_tensor(np.asarray(b.detach().cpu() if torch.is_tensor(b) else b)).double()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def check(what: str, err: float, bound: float) -> None:
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    RESULTS.append({"test": test, "what": what, "err": float(err), "bound": float(bound)})
    assert err < bound, f"{what}: error {err:.3e} >= bound {bound:.1e}"
