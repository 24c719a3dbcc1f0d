"""CPU checks of the contrastive-loss goldens (tests/golden/contrastive_*.npz, written from
the reference's own wrapper.py:72-245 by tests/golden/make_goldens.py):

  * the fixture inputs rebuild bit for bit here (digest), so the GPU test sees the
    same inputs the reference saw;
  * the oracle restatement (oracle/lthm_ref.py::contrastive_loss) reproduces the
    reference's loss, gradients and per-offset statistics: the oracle is pinned by the
    reference, not only by self-consistency.
"""
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)
from contrastive_inputs import CASES, inputs_digest, make_inputs  # noqa: E402

from oracle.lthm_ref import contrastive_loss  # noqa: E402


@pytest.mark.parametrize("name", [n for n, c in CASES.items() if c["B"] * c["T"] <= 10000])
def test_oracle_vs_reference_goldens(name):
    case = CASES[name]
    fx = golden("contrastive_" + name)
    inp = make_inputs(case)
    assert inputs_digest(inp) == str(fx["digest"])
    B = case["B"]
    whole = case["mode"] == "val" or case["mbs"] < 0
    mbs = B if whole else case["mbs"]
    y = torch.from_numpy(inp["y"]).requires_grad_(True)
    t = torch.from_numpy(inp["tgt"]).requires_grad_(True)
    logq = None if case["beta"] == 0.0 else -case["beta"] * torch.from_numpy(inp["logq"])
    loss, stats = contrastive_loss(y, t, torch.from_numpy(inp["mask"]), fx["offsets"], mbs, case["tau"], case["ks"],
                                   logq=logq)
    ref_loss = float(fx["loss"][0])
    assert abs(float(loss) - ref_loss) <= 1e-5 * abs(ref_loss)
    loss.backward()
    De = y.shape[-1]
    if not np.isfinite(float(fx["dy_norm"])):
        # train_nan: the reference's gradients carry NaN (0 dlogits x the NaN embedding in its matmul
        # backward); the oracle's NaN pattern is the reference's
        ry, rt = torch.from_numpy(fx["dy_rows"]), torch.from_numpy(fx["dt_rows"])
        assert torch.equal(torch.isnan(y.grad.reshape(-1, De)[ry]), torch.isnan(torch.from_numpy(fx["dy_sample"])))
        assert torch.equal(torch.isnan(t.grad.reshape(-1, De)[rt]), torch.isnan(torch.from_numpy(fx["dt_sample"])))
    elif "dy" in fx:
        gy, gt = torch.from_numpy(fx["dy"]), torch.from_numpy(fx["dt"])
        assert float((y.grad - gy).norm() / gy.norm()) < 1e-5
        assert float((t.grad - gt).norm() / gt.norm()) < 1e-5
    else:
        ry, rt = torch.from_numpy(fx["dy_rows"]), torch.from_numpy(fx["dt_rows"])
        gy, gt = torch.from_numpy(fx["dy_sample"]), torch.from_numpy(fx["dt_sample"])
        assert float((y.grad.reshape(-1, De)[ry] - gy).norm() / gy.norm()) < 1e-5
        assert float((t.grad.reshape(-1, De)[rt] - gt).norm() / gt.norm()) < 1e-5
    # per-offset statistics of the first helper call against the reference's keys
    ref = dict(zip([str(k) for k in fx["metric_keys"]], fx["metric_values"].tolist()))
    st = "val" if case["mode"] == "val" else "train"
    if whole:
        for h, s in enumerate(stats[0]):
            if s is None:
                continue
            off = int(fx["offsets"][0, h])
            assert s["used"] == ref[f"{st}_used_tokens_offset_{off}"]
            assert abs(s["loss"] - ref[f"{st}_loss_all_tokens_offset_{off}"]) <= 1e-5 * abs(s["loss"])
            assert abs(s["neg"] - ref[f"{st}_average_negatives_per_token_offset_{off}"]) <= 1e-6 * s["neg"]
