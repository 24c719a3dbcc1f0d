"""The oracle's LTHM composition (oracle/lthm_ref.py) against the reference's OWN forward code.

tests/golden/lthm_step_*.npz hold one training step of the reference's Encoder.forward /
ProductTower.forward / QueryTower.forward and its _mini_batch_mapper loss, run in fp32 on the
CPU with the build-defined stand-ins listed in make_goldens.py::gen_lthm_step (the pieces the
reference cannot construct).  Here the build's parameter tree must hold every tensor of the
reference's under the same name and shape, and the oracle run on those weights must give the
reference's loss and parameter gradients (fp32 on both sides, different op order: 1e-5 on the
loss, 1e-4 relative Frobenius on every gradient)."""
import numpy as np
import pytest
import torch

from lthm_step_case import STEP_CASES, build_wrapper, case_config, load_case


@pytest.mark.parametrize("name", STEP_CASES)
def test_state_dict_names_match_reference(name):
    fx, params, _, _ = load_case(name)
    build_wrapper(fx, params, "cpu")  # asserts every reference tensor name / shape is ours


@pytest.mark.parametrize("name", STEP_CASES)
def test_oracle_step_vs_reference(name):
    from oracle import lthm_ref
    fx, params, grads, batch = load_case(name)
    cfg = case_config(fx)
    sd = {k: (v.clone().float().requires_grad_(k in grads) if v.is_floating_point() else v.clone())
          for k, v in params.items()}
    loss = lthm_ref.lthm_forward_loss(sd, cfg, batch, np.asarray(fx["offsets"]))
    ref = float(fx["loss"][0])
    assert abs(float(loss) - ref) <= 1e-5 * abs(ref), (float(loss), ref)
    loss.backward()
    for k, g in grads.items():
        got = sd[k].grad
        assert got is not None, k
        err = float((got.double() - g.double()).norm() / max(float(g.double().norm()), 1e-30))
        assert err < 1e-4, (k, err)
