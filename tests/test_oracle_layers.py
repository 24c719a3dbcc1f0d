"""Pin the encoder / layer restatements in oracle/ref.py to the reference's own
outputs (tests/golden/*.npz, made by tests/golden/make_goldens.py from the
reference modules).  CPU only: fp32 torch against fp32 torch, so the bounds are
float-rounding tight."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref

T = torch.from_numpy


def close(a, b, tol=2e-5):
    a = a.detach().numpy() if isinstance(a, torch.Tensor) else a
    np.testing.assert_allclose(a, b, rtol=tol, atol=tol)


def _params(g):
    return {k[2:]: T(g[k]).clone().requires_grad_(g[k].dtype.kind == "f") for k in g.files if k.startswith("p_")}


def test_quickgelu():
    g = golden("quickgelu")
    close(ref.quick_gelu(T(g["x"])), g["out"], 1e-6)


def test_mlp_quickgelu():
    g = golden("mlp_quickgelu")
    p = _params(g)
    x = T(g["x"]).clone().requires_grad_(True)
    n = len([k for k in p if k.endswith("weight")])
    y = ref.mlp_quickgelu(x, [p[f"model.{2 * i}.weight"] for i in range(n)], [p[f"model.{2 * i}.bias"] for i in range(n)])
    close(y, g["out"])
    (y * T(g["dy"])).sum().backward()
    close(x.grad, g["dx"])
    for k, v in p.items():
        close(v.grad, g["g_" + k])


def test_cap_gradients():
    g = golden("cap_gradients")
    x = T(g["x"]).clone().requires_grad_(True)
    y = ref.cap_gradients(x)
    close(y, g["out"], 0)
    y.backward(T(g["dy"]))
    close(x.grad, g["dx"], 1e-6)


def test_logq():
    g = golden("logq")
    y = ref.logq_forward(T(g["ids"]), T(g["b"]), int(g["num_buckets"]), [int(o) for o in g["offsets"]])
    close(y, g["out"], 1e-6)


def test_layernorm():
    g = golden("layernorm")
    x, w, b = (T(g[k]).clone().requires_grad_(True) for k in ("x", "w", "b"))
    y = ref.layer_norm(x, w, b)
    close(y, g["out"])
    y.backward(T(g["dy"]))
    close(x.grad, g["dx"], 1e-4)
    close(w.grad, g["dw"], 1e-4)
    close(b.grad, g["db"], 1e-4)


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_transformer_block(idx):
    g = golden(f"transformer_block_{idx}")
    p = _params(g)
    x = T(g["x"]).clone().requires_grad_(True)
    y = ref.transformer_block(x, p, int(g["H"]), bool(g["causal"]))
    close(y, g["out"], 1e-4)
    y.backward(T(g["dy"]))
    close(x.grad, g["dx"], 1e-4)
    for k, v in p.items():
        if v.requires_grad and "g_" + k in g.files:
            close(v.grad, g["g_" + k], 2e-4)


@pytest.mark.parametrize("idx", [0, 1])
def test_transformer_block_attn_mask(idx):
    """TransformerBlock.forward(x, attn_mask) with a general additive mask (:374, :404-408)."""
    g = golden(f"transformer_block_mask_{idx}")
    p = _params(g)
    x = T(g["x"]).clone().requires_grad_(True)
    y = ref.transformer_block(x, p, int(g["H"]), bool(g["causal"]), attn_mask=T(g["mask"]))
    close(y, g["out"], 1e-4)
    y.backward(T(g["dy"]))
    close(x.grad, g["dx"], 1e-4)
    for k, v in p.items():
        if v.requires_grad and "g_" + k in g.files:
            close(v.grad, g["g_" + k], 2e-4)


def test_mqa():
    g = golden("mqa")
    p = _params(g)
    x = T(g["x"]).clone().requires_grad_(True)
    y = ref.mqa(x, p, 4, ref.causal_mask(x.shape[1]))
    close(y, g["out"], 1e-4)
    y.backward(T(g["dy"]))
    close(x.grad, g["dx"], 1e-4)
    for k, v in p.items():
        close(v.grad, g["g_" + k], 2e-4)


def test_moe_linear():
    g = golden("moe")
    p = _params(g)
    x = T(g["x"]).clone().requires_grad_(True)
    y = ref.moe_linear(x, p, num_experts=4, top_k=2, in_features=16, n_gate_layers=2)
    close(y, g["out"], 1e-5)
    y.backward(T(g["dy"]))
    close(x.grad, g["dx"], 1e-5)


@pytest.mark.parametrize("name", ["cve_2", "cve_20"])
def test_cve(name):
    g = golden(name)
    W = T(g["weight"]).clone().requires_grad_(True)
    y = ref.cve_fwd(T(g["x"]), T(g["projection_mat"]), T(g["grid"]), T(g["pos_offset"]), W)
    close(y, g["out"], 1e-5)
    y.backward(T(g["dy"]))
    close(W.grad, g["dweight"], 1e-5)


def test_simhash():
    g = golden("simhash")
    assert (ref.simhash(T(g["x"]), T(g["projection_mat"])).numpy() == g["out"]).all()


def test_simhash63():
    g = golden("simhash63")
    assert (ref.simhash(T(g["x"]), T(g["projection_mat"])).numpy() == g["out"]).all()


def test_cosine_linear():
    g = golden("cosine_linear")
    x, w = T(g["x"]).clone().requires_grad_(True), T(g["weight"]).clone().requires_grad_(True)
    y = ref.cosine_linear(x, w)
    close(y, g["out"], 1e-5)
    y.backward(T(g["dy"]))
    close(x.grad, g["dx"], 1e-5)
    close(w.grad, g["dweight"], 1e-5)


@pytest.mark.parametrize("tag", ["lcve", "lcve_top5", "lcve_nb7"])
def test_learnable_cve(tag):
    g = golden(tag)
    x, pw, mean, ew = (T(g[k]).clone().requires_grad_(True) for k in ("x", "proj_weight", "mean", "emb_weight"))
    tk = int(g["top_k"]) or None
    y = ref.learnable_cve(x, pw, mean, ew, float(g["sigma2"]), tk)
    close(y, g["out"], 1e-5)
    y.backward(T(g["dy"]))
    for t, k in ((x, "dx"), (pw, "dproj_weight"), (mean, "dmean"), (ew, "demb_weight")):
        close(t.grad, g[k], 1e-4)


@pytest.mark.parametrize("tag", ["pve", "pve_top3"])
def test_probability_ve(tag):
    g = golden(tag)
    x, mean, ew = (T(g[k]).clone().requires_grad_(True) for k in ("x", "mean", "emb_weight"))
    y = ref.probability_ve(x, mean, ew, float(g["sigma2"]), int(g["top_k"]) or None)
    close(y, g["out"], 1e-5)
    y.backward(T(g["dy"]))
    for t, k in ((x, "dx"), (mean, "dmean"), (ew, "demb_weight")):
        close(t.grad, g[k], 1e-4)
