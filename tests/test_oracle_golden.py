"""CPU: the oracle (C + torch-CPU restatement) against the reference's own outputs.

The golden vectors were produced by importing the reference components
(tests/golden/make_goldens.py); these tests are what "pins" the oracle.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref


def test_kshift_rows_bit_exact():
    g = golden("kshift_rows")
    for a, P in enumerate(g["Ps"]):
        rows = ref.kshift_rows(g["ids"], int(P), 32)
        np.testing.assert_array_equal(rows.T, g["rows"][a])


@pytest.mark.parametrize("case", range(6))
def test_kshift_fwd_bwd(case):
    g = golden(f"kshift_fwd_bwd_{case}")
    K, mode = int(g["K"]), (1 if int(g["normalize"]) else 0)
    out = ref.kshift_fwd_c(g["ids"], g["weight"], K, mode)
    if mode == 0:
        np.testing.assert_array_equal(out, g["out"])  # in-order fp32 sum + IEEE divide: bit-exact
    else:
        np.testing.assert_allclose(out, g["out"], rtol=2e-7, atol=1e-7)
    # torch restatement is bit-exact in both modes
    ot = ref.kshift_fwd_torch(torch.from_numpy(g["ids"]), torch.from_numpy(g["weight"]), K, bool(mode))
    np.testing.assert_array_equal(ot.numpy(), g["out"])
    W = torch.from_numpy(g["weight"]).clone().requires_grad_(True)
    y = ref.kshift_fwd_torch(torch.from_numpy(g["ids"]), W, K, bool(mode))
    (y * torch.from_numpy(g["dy"])).sum().backward()
    np.testing.assert_allclose(W.grad.numpy(), g["dweight"], rtol=1e-5, atol=1e-5)
    if mode == 0:
        dw = ref.kshift_bwd_c(g["ids"], g["dy"], int(g["P"]), K, 0)
        np.testing.assert_allclose(dw, g["dweight"], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_flat(seed):
    g = golden(f"flat_{seed}")
    pad = int(g["padding_idx"])
    W = torch.from_numpy(g["weight"]).clone().requires_grad_(True)
    y = ref.flat_fwd(torch.from_numpy(g["ids"]), W, bool(g["normalize"]), None if pad < 0 else pad)
    np.testing.assert_allclose(y.detach().numpy(), g["out"], rtol=1e-6, atol=1e-7)
    (y * torch.from_numpy(g["dy"])).sum().backward()
    np.testing.assert_allclose(W.grad.numpy(), g["dweight"], rtol=1e-5, atol=1e-5)


def test_hot_row_skew_structure():
    """for c >= 1 every negative id lands in the last 2^(c-1) rows."""
    rng = np.random.default_rng(0)
    ids = rng.integers(-(2 ** 63), 2 ** 63 - 1, size=20000, dtype=np.int64)
    P = 1_000_000
    rows = ref.kshift_rows(ids, P, 16)
    neg = ids < 0
    for c in range(1, 16):
        assert (rows[neg, c] >= P - 2 ** (c - 1)).all()
    assert (rows[neg, 1] == P - 1).all()
    assert (ref.kshift_rows(np.zeros(3, dtype=np.int64), P, 16) == 0).all()
