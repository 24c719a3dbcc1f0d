"""GPU parity: GEMM, LayerNorm, attention and the fused TransformerBlock.

Kernel-level tests compare against the fp32 oracle evaluated on the SAME
bf16-quantised operands (tolerance: relative Frobenius error <= 1e-3, the
north-star bound for bf16 activations).  Block-level tests compare against the
reference's own fp32 outputs (tests/golden/transformer_block_*.npz); there the
operands themselves are bf16-rounded inside the block, so the bound is looser
(2e-2 relative Frobenius) and stated per assertion.
"""
import math

import numpy as np
import pytest
import torch

from parity import check, relerr
import torch.nn.functional as F

from conftest import golden
from oracle import ref

pytestmark = pytest.mark.gpu




def bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("M,N,Kd", [(1000, 768, 256), (129, 256, 256), (4096, 1024, 256), (333, 64, 1024), (8, 8, 8)])
@pytest.mark.parametrize("act", [0, 1, 2, 5])
def test_gemm_nt_epilogues(dev, M, N, Kd, act):
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(M + N + Kd + act)
    A = bf(torch.randn(M, Kd, generator=g))
    W = bf(torch.randn(N, Kd, generator=g) / math.sqrt(Kd))
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    out = K.linear_fwd(A.to(dev), W.to(dev), bias=bias.to(dev), act=act, aux_out=pre if act else None,
                       res1=res.to(dev), out_dtype=torch.float32)
    z = A.float() @ W.float().T + bias
    exp = {0: z, 1: F.gelu(z, approximate="tanh"), 2: ref.quick_gelu(z), 5: F.gelu(z, approximate="tanh")}[act] + res
    check('out, exp', relerr(out, exp), 1e-5)
    if act == K.ACT_GELU_D:
        # the saved aux is GELU'(z), rounded once to bf16
        zz = z.clone().requires_grad_(True)
        F.gelu(zz, approximate="tanh").sum().backward()
        assert (pre.float().cpu() - zz.grad).abs().max() < 1.5 * 2.0 ** -8 * zz.grad.abs().max() + 1e-6
    elif act:
        # the saved pre-activation is z rounded once to bf16 (one bf16 ulp of |z|)
        check("pre-activation vs bf16(z)", relerr(pre.float(), bf(z).float()), 1e-3)
        ulp = float((pre.float().cpu() - z).abs().max() / z.abs().max())
        check("pre-activation max abs err / max|z|", ulp, 2.0 ** -8)
    # bf16 output: within 1 bf16 ulp of the rounded oracle
    outb = K.linear_fwd(A.to(dev), W.to(dev), bias=bias.to(dev), act=act, aux_out=pre if act else None)
    check('outb.float(), bf(exp - res).float()', relerr(outb.float(), bf(exp - res).float()), 1e-3)


@pytest.mark.parametrize("M,N,Kd", [(1000, 768, 256), (4096, 256, 1024), (40, 24, 32)])
def test_gemm_dgrad_wgrad(dev, M, N, Kd):
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(7 * M + N)
    dy = bf(torch.randn(M, N, generator=g))
    W = bf(torch.randn(N, Kd, generator=g))
    X = bf(torch.randn(M, Kd, generator=g))
    pre = bf(torch.randn(M, Kd, generator=g))
    dx = K.linear_dgrad(dy.to(dev), W.to(dev), out_dtype=torch.float32)
    check('dx, dy.float() @ W.float()', relerr(dx, dy.float() @ W.float()), 1e-5)
    dxg = K.linear_dgrad(dy.to(dev), W.to(dev), act_grad=K.ACT_GELU_GRAD, aux=pre.to(dev), out_dtype=torch.float32)
    p = pre.float().requires_grad_(True)
    F.gelu(p, approximate="tanh").backward(dy.float() @ W.float())
    check('dxg, p.grad', relerr(dxg, p.grad), 1e-5)
    dxm = K.linear_dgrad(dy.to(dev), W.to(dev), act_grad=K.ACT_MUL_AUX, aux=pre.to(dev), out_dtype=torch.float32)
    check('dxm, (dy.float() @ W.float()) * pre.float()', relerr(dxm, (dy.float() @ W.float()) * pre.float()), 1e-5)
    dw = K.linear_wgrad(dy.to(dev), X.to(dev))
    check('dw, dy.float().T @ X.float()', relerr(dw, dy.float().T @ X.float()), 1e-5)


@pytest.mark.parametrize("M,N,Kd", [(263001, 512, 1536), (70003, 768, 256), (4100, 2048, 512)])
def test_gemm_wgrad_ragged_rows(dev, M, N, Kd):
    """dW = dY^T X with a row count of no alignment (the packed rows of a shared pad prefix):
    the split-K weight-gradient kernel zero-fills the k rows past the end."""
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(M + N)
    dy = bf(torch.randn(M, N, generator=g))
    X = bf(torch.randn(M, Kd, generator=g))
    dw = K.linear_wgrad(dy.to(dev), X.to(dev))
    check("ragged-row wgrad", relerr(dw, dy.double().T @ X.double()), 1e-5)


def test_gemm_wgrad_splitk_large(dev):
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(3)
    M, N, Kd = 131072, 256, 64
    dy = bf(torch.randn(M, N, generator=g))
    X = bf(torch.randn(M, Kd, generator=g))
    acc = torch.randn(N, Kd, generator=g)
    out = acc.clone().to(dev)
    K.linear_wgrad(dy.to(dev), X.to(dev), out=out, accumulate=True)
    exp = (dy.double().T @ X.double()) + acc.double()
    check('out, exp', relerr(out, exp), 1e-5)


@pytest.mark.parametrize("M,N,Kd,act", [(65573, 768, 256, 0), (65573, 768, 256, 1), (50001, 200, 72, 2),
                                         (40000, 1024, 1024, 0)])
def test_gemm_large_nt(dev, M, N, Kd, act):
    """Step-sized shapes (thousands of tiles: interior fast path + ragged edge tiles,
    a partial K-tile, the residual and both activations)."""
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(M + N + Kd)
    A = bf(torch.randn(M, Kd, generator=g))
    W = bf(torch.randn(N, Kd, generator=g) / math.sqrt(Kd))
    bias = torch.randn(N, generator=g)
    res = bf(torch.randn(M, N, generator=g))
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    out = K.linear_fwd(A.to(dev), W.to(dev), bias=bias.to(dev), act=act, aux_out=pre if act else None,
                       res1=res.to(dev), out_dtype=torch.float32)
    z = A.float() @ W.float().T + bias
    exp = {0: z, 1: F.gelu(z, approximate="tanh"), 2: ref.quick_gelu(z)}[act] + res.float()
    check('out, exp', relerr(out, exp), 1e-5)
    if act:
        assert (pre.float().cpu() - z).abs().max() < 0.05


@pytest.mark.parametrize("M,N,Kd,act,res2", [(777, 600, 512, 2, False), (4099, 1100, 2176, 1, True),
                                              (65536, 1024, 2176, 0, False), (300, 2176, 1024, 5, False)])
def test_gemm_256_tiles(dev, M, N, Kd, act, res2):
    """The 256 x 256 kernel (K-contiguous operands, K >= 512): ragged row and column tiles,
    bias, the activations with their saved aux, one or two residuals, f32 and bf16 outputs."""
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(M + 3 * N + Kd)
    A = bf(torch.randn(M, Kd, generator=g))
    W = bf(torch.randn(N, Kd, generator=g) / math.sqrt(Kd))
    bias = torch.randn(N, generator=g)
    r1 = torch.randn(M, N, generator=g)
    r2 = torch.randn(M, N, generator=g) if res2 else None
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    out = K.linear_fwd(A.to(dev), W.to(dev), bias=bias.to(dev), act=act, aux_out=pre if act else None,
                       res1=r1.to(dev), res2=r2.to(dev) if res2 else None, out_dtype=torch.float32)
    z = A.float() @ W.float().T + bias
    exp = {0: z, 1: F.gelu(z, approximate="tanh"), 2: ref.quick_gelu(z), 5: F.gelu(z, approximate="tanh")}[act] + r1
    if res2:
        exp = exp + r2
    check("256-tile out", relerr(out, exp), 1e-5)
    outb = K.linear_fwd(A.to(dev), W.to(dev))
    check("256-tile bf16 out", relerr(outb.float(), bf(A.float() @ W.float().T).float()), 1e-3)


@pytest.mark.parametrize("M,N,Kd", [(70001, 768, 256), (30000, 256, 1024)])
def test_gemm_large_dgrad(dev, M, N, Kd):
    """dX = dY W (K-strided B) at step size, with the GELU-grad epilogue."""
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(M + Kd)
    dy = bf(torch.randn(M, N, generator=g))
    W = bf(torch.randn(N, Kd, generator=g))
    pre = bf(torch.randn(M, Kd, generator=g))
    dx = K.linear_dgrad(dy.to(dev), W.to(dev), out_dtype=torch.float32)
    ref_dx = dy.float() @ W.float()
    check('dx, ref_dx', relerr(dx, ref_dx), 1e-5)
    dxg = K.linear_dgrad(dy.to(dev), W.to(dev), act_grad=K.ACT_GELU_GRAD, aux=pre.to(dev), out_dtype=torch.float32)
    p = pre.float().requires_grad_(True)
    F.gelu(p, approximate="tanh").backward(ref_dx)
    check('dxg, p.grad', relerr(dxg, p.grad), 1e-5)


def test_gemm_large_batched(dev):
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(11)
    Bt, M, N, Kd = 3, 20000, 256, 128
    A = bf(torch.randn(Bt, M, Kd, generator=g))
    Bm = bf(torch.randn(Bt, N, Kd, generator=g))
    out = K.gemm(A.to(dev), Bm.to(dev), M, N, Kd, batch=Bt, sA=M * Kd, sB=N * Kd, out_dtype=torch.float32, alpha=0.5)
    check('out, 0.5 * A.float() @ Bm.float().transpose(1, 2)', relerr(out, 0.5 * A.float() @ Bm.float().transpose(1, 2)), 1e-5)


def test_gemm_batched(dev):
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(5)
    Bt, M, N, Kd = 5, 300, 200, 128
    A = bf(torch.randn(Bt, M, Kd, generator=g))
    Bm = bf(torch.randn(Bt, N, Kd, generator=g))
    out = K.gemm(A.to(dev), Bm.to(dev), M, N, Kd, batch=Bt, sA=M * Kd, sB=N * Kd, out_dtype=torch.float32, alpha=0.5)
    check('out, 0.5 * A.float() @ Bm.float().transpose(1, 2)', relerr(out, 0.5 * A.float() @ Bm.float().transpose(1, 2)), 1e-5)


def test_layernorm_golden(dev):
    from recommendations_amd.commons.transformers.layers import LayerNorm
    g = golden("layernorm")
    ln = LayerNorm(48).to(dev)
    with torch.no_grad():
        ln.weight.copy_(torch.from_numpy(g["w"]))
        ln.bias.copy_(torch.from_numpy(g["b"]))
    x = torch.from_numpy(g["x"]).to(dev).requires_grad_(True)
    y = ln(x)
    np.testing.assert_allclose(y.detach().cpu().numpy(), g["out"], rtol=1e-5, atol=1e-5)
    y.backward(torch.from_numpy(g["dy"]).to(dev))
    np.testing.assert_allclose(x.grad.cpu().numpy(), g["dx"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(ln.weight.grad.cpu().numpy(), g["dw"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(ln.bias.grad.cpu().numpy(), g["db"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("B,T,H,E,causal", [(3, 129, 4, 64, True), (2, 33, 1, 64, True), (4, 17, 2, 32, False),
                                            (2, 200, 2, 64, True), (1, 256, 1, 16, True), (2, 128, 2, 64, True),
                                            (1, 256, 2, 64, False), (2, 64, 2, 128, True), (3, 1, 2, 64, True),
                                            (2, 47, 3, 32, True), (2, 225, 2, 64, True), (3, 97, 1, 64, False),
                                            # windowed long-sequence path (T' > 256; C5 has T' = 513)
                                            (2, 513, 2, 64, True), (3, 300, 1, 64, False), (17, 257, 1, 32, True),
                                            (1, 400, 2, 128, True), (20, 520, 1, 64, True),
                                            # the persistent double-buffered E = 64 backward (B >= 2 x the
                                            # workgroups per head): tail mode, uneven entries per slot
                                            (300, 129, 4, 64, True), (520, 65, 1, 64, False), (600, 100, 2, 64, True)])
def test_attention_vs_oracle(dev, B, T, H, E, causal):
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(B * T + H)
    C = H * E
    qkv = bf(torch.randn(B * T, 3 * C, generator=g))
    table = 0.5 * torch.randn(2 * T + 5, H, generator=g)
    out, lse = K.attn_fwd_qkv(qkv.to(dev), B, T, H, E, table.to(dev), causal)
    q, k, v = qkv.float().view(B, T, 3, H, E).permute(2, 0, 3, 1, 4)
    q = q.clone().requires_grad_(True); k = k.clone().requires_grad_(True); v = v.clone().requires_grad_(True)
    tab = table.clone().requires_grad_(True)
    # oracle: reference SDPA with nk = T -> table row q - k + T
    mask = ref.causal_mask(T) if causal else None
    o = ref.sdpa(q, k, v, mask, tab)
    exp = o.transpose(1, 2).reshape(B * T, C)
    # bf16 output: compare with the bf16-rounded fp32 oracle
    check('out.float(), bf(exp.detach()).float()', relerr(out.float(), bf(exp.detach()).float()), 1e-3)
    dout = bf(torch.randn(B * T, C, generator=g))
    exp.backward(dout.float())
    dqkv, dtab = K.attn_bwd_qkv(qkv.to(dev), out, dout.to(dev), lse, B, T, H, E, table.to(dev), causal)
    dq, dk, dv = dqkv.float().cpu().view(B, T, 3, H, E).permute(2, 0, 3, 1, 4)
    # relative Frobenius 1e-2; gradients that are exactly zero (T = 1: softmax over
    # one key) are checked against an absolute 1e-4 instead
    for got, want in ((dq, q.grad), (dk, k.grad), (dv, v.grad), (dtab, tab.grad[: 2 * T + 1])):
        if float(want.norm()) == 0.0:
            assert float(got.abs().max()) < 1e-4
        else:
            check('got, want', relerr(got, want), 1e-2)


def test_attention_persistent_bwd_matches_default(dev, tmp_path):
    """The persistent double-buffered E = 64 backward (attn_bwd32p_k, opt-in LTHM_ATTN_BWD_P=1,
    read once by the library: run in a child process, tests/attn_pers_worker.py) against the
    default one-workgroup-per-(b, h) kernel on the same inputs: each (b, h)'s units run the
    same arithmetic, so dq / dk / dv are identical; the bias gradient sums the entries per
    workgroup slot before the cross-slot reduction (f32 order only)."""
    import os
    import subprocess
    import sys
    import numpy as np
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from attn_pers_worker import run_case
    cases = [(300, 129, 4, 64, True), (520, 65, 1, 64, False), (600, 100, 2, 64, True)]
    specs = [",".join(str(int(x)) for x in c) for c in cases]
    path = str(tmp_path / "pers.npz")
    env = dict(os.environ, LTHM_ATTN_BWD_P="1")
    here = os.path.dirname(os.path.abspath(__file__))
    subprocess.run([sys.executable, os.path.join(here, "attn_pers_worker.py"), path] + specs, env=env, check=True,
                   timeout=300)
    got = np.load(path)
    for c, spec in zip(cases, specs):
        dq, dt = run_case(dev, *c)
        assert np.array_equal(got[f"{spec}/dqkv"], dq), (spec, np.abs(got[f"{spec}/dqkv"] - dq).max())
        check(f"dtable persistent vs default {spec}", relerr(torch.from_numpy(got[f"{spec}/dtab"]),
                                                            torch.from_numpy(dt)), 1e-5)


def _cfg(d, H, bias, causal, pos):
    from recommendations_amd.commons.transformers.configs import TransformerConfig
    return TransformerConfig(rotator_config={"ff_mult": 4}, is_causal=causal,
                             attn_config=dict(attn_dropout=0.0, bias=bias, dropout=0.0, n_head=H, n_embd=d,
                                              attn_type="multi_head",
                                              pos_bias=None if pos < 0 else {"context_window": pos}))


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_transformer_block_golden(dev, idx):
    from recommendations_amd.commons.transformers.layers import TransformerBlock
    g = golden(f"transformer_block_{idx}")
    d, H, bias, causal, pos = int(g["d"]), int(g["H"]), bool(g["bias"]), bool(g["causal"]), int(g["context_window"])
    blk = TransformerBlock(_cfg(d, H, bias, causal, pos)).to(dev)
    sd = {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("p_")}
    blk.load_state_dict(sd)
    x = torch.from_numpy(g["x"]).to(dev).requires_grad_(True)
    y = blk(x)
    # bf16 operands inside the block (fp32 residual stream): 2e-2 relative Frobenius vs the fp32 reference
    check('y.detach(), g["out"]', relerr(y.detach(), g["out"]), 2e-2)
    y.backward(torch.from_numpy(g["dy"]).to(dev))
    check('x.grad, g["dx"]', relerr(x.grad, g["dx"]), 2e-2)
    for n, p in blk.named_parameters():
        check(f"p.grad, g['g_' + n] {n}", relerr(p.grad, g["g_" + n]), 3e-2)


def test_mqa_golden(dev):
    """MultiQueryAttention (commons/transformers/layers.py:202-234) vs the
    reference's own outputs and gradients (tests/golden/mqa.npz, causal mask, learned
    relative-position bias).  bf16 GEMM operands: 2e-2 forward, 3e-2 gradients."""
    from types import SimpleNamespace
    from recommendations_amd.commons.transformers.layers import MultiQueryAttention
    g = golden("mqa")
    acfg = SimpleNamespace(n_embd=64, n_head=4, attn_dropout=0.0, dropout=0.0, bias=True,
                           pos_bias=SimpleNamespace(context_window=16))
    m = MultiQueryAttention(acfg)
    m.load_state_dict({k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("p_")})
    m = m.to(dev)
    x = torch.from_numpy(g["x"]).to(dev).requires_grad_(True)
    mask = ref.causal_mask(x.shape[1]).to(dev)
    y = m(x, mask)
    check('y, g["out"]', relerr(y, g["out"]), 2e-2)
    y.backward(torch.from_numpy(g["dy"]).to(dev))
    check('x.grad, g["dx"]', relerr(x.grad, g["dx"]), 3e-2)
    for n, p in m.named_parameters():
        check(f"p.grad, g['g_' + n] {n}", relerr(p.grad, g["g_" + n]), 3e-2)


def test_mha_module_vs_oracle(dev):
    """MultiHeadAttention.forward as a standalone module (:247-265) vs oracle/ref.mha."""
    from types import SimpleNamespace
    from recommendations_amd.commons.transformers.layers import MultiHeadAttention
    torch.manual_seed(3)
    acfg = SimpleNamespace(n_embd=128, n_head=2, attn_dropout=0.0, dropout=0.0, bias=True,
                           pos_bias=SimpleNamespace(context_window=40))
    m = MultiHeadAttention(acfg)
    with torch.no_grad():
        m.attn.pos_bias.bias.add_(0.2 * torch.randn(m.attn.pos_bias.bias.shape))
    sd = {k: v.clone().requires_grad_(True) for k, v in m.state_dict().items()}
    m = m.to(dev)
    x = torch.randn(3, 37, 128)
    xd = x.to(dev).requires_grad_(True)
    y = m(xd, ref.causal_mask(37).to(dev))
    xr = x.clone().requires_grad_(True)
    yr = ref.mha(xr, sd, 2, ref.causal_mask(37), prefix="")
    check('y, yr', relerr(y, yr), 2e-2)
    dy = torch.randn(y.shape)
    y.backward(dy.to(dev))
    yr.backward(dy)
    check('xd.grad, xr.grad', relerr(xd.grad, xr.grad), 3e-2)
    for n, p in m.named_parameters():
        check(f"p.grad, sd[n].grad {n}", relerr(p.grad, sd[n].grad), 3e-2)


def test_sparse_token_transformer_block(dev):
    """is_sparse_attn (:352-372, :383-420): seeded kept-token subset through the dense
    block, the rest through the null connector, vs the oracle composition."""
    from recommendations_amd.commons.transformers.configs import TransformerConfig
    from recommendations_amd.commons.transformers.layers import TransformerBlock
    torch.manual_seed(5)
    d, H, T = 64, 1, 24
    cfg = TransformerConfig(rotator_config={"ff_mult": 4}, is_causal=True, is_sparse_attn=True, max_block_size=32,
                            sparsity_factor=0.5,
                            attn_config=dict(attn_dropout=0.0, bias=True, dropout=0.0, n_head=H, n_embd=d,
                                             attn_type="multi_head", pos_bias={"context_window": 32}))
    blk = TransformerBlock(cfg, seed=7, n_cls=1)
    sd = {k: v.clone() for k, v in blk.state_dict().items()}
    blk = blk.to(dev)
    x = torch.randn(2, T, d)
    y = blk(x.to(dev))
    idx = sd["input_mask_idx"][sd["input_mask_idx"] < T]
    nidx = sd["input_mask_not_idx"][sd["input_mask_not_idx"] < T]
    exp = torch.zeros_like(x)
    exp[:, idx] = ref.transformer_block(x[:, idx], sd, H, True)
    exp[:, nidx] = x[:, nidx] + F.linear(x[:, nidx], sd["null_connector.weight"], sd["null_connector.bias"])
    assert idx.numel() > 1 and nidx.numel() > 0
    check('y, exp', relerr(y, exp), 2e-2)
    y.sum().backward()
    assert torch.isfinite(blk.null_connector.weight.grad).all() and float(blk.null_connector.weight.grad.norm()) > 0


def test_moe_golden(dev):
    """MoELinear (commons/transformers/layers.py:101-136, top-k gating) vs the
    reference's own outputs and input gradient (tests/golden/moe.npz), and its parameter
    gradients vs oracle/ref.moe_linear (itself pinned to moe.npz in test_oracle_layers).
    bf16 expert GEMM operands: 2e-2 forward, 3e-2 gradients."""
    from recommendations_amd.commons.transformers.layers import MoELinear
    g = golden("moe")
    m = MoELinear(16, 24, proj_features=32, num_experts=4, top_k=2, gate_sizes=(8,))
    sd = {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("p_")}
    m.load_state_dict(sd)
    m = m.to(dev)
    x = torch.from_numpy(g["x"]).to(dev).requires_grad_(True)
    y = m(x)
    check('y, g["out"]', relerr(y, g["out"]), 2e-2)
    y.backward(torch.from_numpy(g["dy"]).to(dev))
    check('x.grad, g["dx"]', relerr(x.grad, g["dx"]), 3e-2)
    pr = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    yr = ref.moe_linear(torch.from_numpy(g["x"]), pr, 4, 2, 16, 2)
    yr.backward(torch.from_numpy(g["dy"]))
    for n, p in m.named_parameters():
        check(f"p.grad, pr[n].grad {n}", relerr(p.grad, pr[n].grad), 3e-2)


@pytest.mark.parametrize("top_k", [None, 3])
def test_moe_transformer_block_vs_oracle(dev, top_k):
    """TransformerBlock with a MoE rotator ({"moe": {...}}, :340-343) at a larger shape:
    attention + _MoEMLP (c_fc MoE, GELU, c_proj MoE) vs the oracle composition."""
    from types import SimpleNamespace
    from recommendations_amd.commons.transformers.layers import TransformerBlock
    torch.manual_seed(11)
    d, H, T_, B = 128, 2, 40, 6
    moe = dict(num_experts=4, proj_features=64, ff_mult_factor=2.0, top_k=top_k, gate_sizes=[16])
    cfg = SimpleNamespace(is_causal=True, rotator_config={"moe": moe}, is_sparse_attn=False,
                          attn_config=SimpleNamespace(n_embd=d, n_head=H, attn_dropout=0.0, dropout=0.0, bias=True,
                                                      attn_type="multi_head",
                                                      pos_bias=SimpleNamespace(context_window=64)))
    blk = TransformerBlock(cfg)
    assert blk.is_moe
    sd = {k: v.clone() for k, v in blk.state_dict().items()}
    blk = blk.to(dev)
    x = torch.randn(B, T_, d)
    xd = x.to(dev).requires_grad_(True)
    y = blk(xd)
    pr = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
    xr = x.clone().requires_grad_(True)
    h = xr + ref.mha(ref.layer_norm(xr, pr["ln_1.weight"], pr["ln_1.bias"]), pr, H, ref.causal_mask(T_))
    sub = lambda pre: {k[len(pre):]: v for k, v in pr.items() if k.startswith(pre)}  # noqa: E731
    z = ref.layer_norm(h, pr["ln_2.weight"], pr["ln_2.bias"])
    z = ref.moe_linear(z, sub("mlp.c_fc."), 4, top_k, d, 2)
    z = torch.nn.functional.gelu(z, approximate="tanh")
    yr = h + ref.moe_linear(z, sub("mlp.c_proj."), 4, top_k, int(2.0 * d), 2)
    check('y, yr', relerr(y, yr), 2e-2)
    dy = torch.randn(y.shape)
    y.backward(dy.to(dev))
    yr.backward(dy)
    check('xd.grad, xr.grad', relerr(xd.grad, xr.grad), 3e-2)
    for n, p in blk.named_parameters():
        check(f"p.grad, pr[n].grad {n}", relerr(p.grad, pr[n].grad), 3e-2)


# ---------------------------------------------------------------- bf16-mirrored oracle
def _block_oracle(sd, x, dy, H, causal, drop=None, dbl=False, attn_mask=None):
    """oracle/ref.transformer_block with bf16 rounding at the HIP path's own points
    (ref._QB / _QG): what remains is accumulation order and exp / rsqrt rounding."""
    p = {k: v.detach().cpu().float().clone().requires_grad_(True) for k, v in sd.items() if v.is_floating_point()}
    xr = x.detach().cpu().float().clone().requires_grad_(True)
    y = ref.transformer_block(xr, p, H, causal, attn_mask=attn_mask, drop=drop, bf16=True)
    if dbl:
        y = y + xr
    y.backward(dy.detach().cpu().float())
    return y.detach(), xr.grad, {k: v.grad for k, v in p.items()}


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_transformer_block_golden_bf16_oracle(dev, idx):
    """The golden block shapes vs the oracle with the same bf16 operands: the north
    star's 1e-3 relative bound on the bf16-activation forward."""
    from recommendations_amd.commons.transformers.layers import TransformerBlock
    g = golden(f"transformer_block_{idx}")
    d, H, bias, causal, pos = int(g["d"]), int(g["H"]), bool(g["bias"]), bool(g["causal"]), int(g["context_window"])
    blk = TransformerBlock(_cfg(d, H, bias, causal, pos)).to(dev)
    sd = {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("p_")}
    blk.load_state_dict(sd)
    x = torch.from_numpy(g["x"]).to(dev).requires_grad_(True)
    dy = torch.from_numpy(g["dy"])
    y = blk(x)
    yr, dxr, gr = _block_oracle(sd, x, dy, H, causal)
    check("block fwd vs bf16 oracle", relerr(y.detach() - x.detach(), yr - x.detach().cpu()), 1e-3)
    y.backward(dy.to(dev))
    check("dx vs bf16 oracle", relerr(x.grad, dxr), 1e-2)
    for n, p in blk.named_parameters():
        check(f"d{n} vs bf16 oracle", relerr(p.grad, gr[n]), 1e-2)


def _rand_block(dev, B, T, d, H, seed, dropout=0.0, bias=False):
    from recommendations_amd.commons.transformers.layers import TransformerBlock
    from recommendations_amd.commons.transformers.configs import TransformerConfig
    torch.manual_seed(seed)
    cfg = TransformerConfig(rotator_config={"ff_mult": 4}, is_causal=True,
                            attn_config=dict(attn_dropout=dropout, bias=bias, dropout=dropout, n_head=H, n_embd=d,
                                             attn_type="multi_head", pos_bias={"context_window": T}))
    blk = TransformerBlock(cfg)
    with torch.no_grad():
        for n, p in blk.named_parameters():
            if "pos_bias" in n or "ln_" in n or n.endswith("bias"):
                p.add_(0.1 * torch.randn(p.shape))
    sd = {k: v.clone() for k, v in blk.state_dict().items()}
    x = torch.randn(B, T, d)
    dy = torch.randn(B, T, d) / math.sqrt(B * T * d)
    return blk.to(dev), sd, x, dy


@pytest.mark.parametrize("B,T,d,H", [(6, 129, 256, 4), (4, 64, 64, 1), (2, 513, 512, 8)])
def test_block_c2_c5_shapes_vs_bf16_oracle(dev, B, T, d, H):
    """The LTHM encoder block as C2 (T' = 129, d = 256, H = 4) and C5 (T' = 513, d = 512,
    H = 8) run it: causal, relative-position bias, no biases, double residual
    (query_tower.py:135), vs the bf16-mirrored oracle."""
    blk, sd, x, dy = _rand_block(dev, B, T, d, H, seed=B + T)
    xd = x.to(dev).requires_grad_(True)
    y = blk.forward_double_residual(xd)
    yr, dxr, gr = _block_oracle(sd, x, dy, H, True, dbl=True)
    check("block fwd vs bf16 oracle", relerr(y.detach().cpu() - 2 * x, yr - 2 * x), 1e-3)
    y.backward(dy.to(dev))
    check("dx vs bf16 oracle", relerr(xd.grad, dxr), 1e-2)
    for n, p in blk.named_parameters():
        check(f"d{n} vs bf16 oracle", relerr(p.grad, gr[n]), 1e-2)


@pytest.mark.parametrize("p", [0.1, 0.3])
def test_block_dropout_vs_oracle(dev, p):
    """Training-mode dropout (commons/transformers/layers.py:253-256 token dropout of
    q / k / v, :264 residual dropout, :283 MLP dropout): the HIP path's hash masks,
    read back through lthm_dropout_mask, drive the oracle's dropouts; the outputs and
    gradients then match as at p = 0, and each mask keeps 1 - p of its elements."""
    from recommendations_amd import kernels as K
    B, T, d, H = 4, 65, 128, 2
    blk, sd, x, dy = _rand_block(dev, B, T, d, H, seed=11, dropout=p)
    blk.train()
    xd = x.to(dev).requires_grad_(True)
    torch.manual_seed(77)
    y = blk(xd)
    torch.manual_seed(77)
    seed = K.new_dropout_seed()
    M = B * T
    sc = 1.0 / (1.0 - p)
    mrows = K.dropout_mask(3 * M, p, seed, dev).float().cpu() * sc
    drop = {"q": mrows[:M].view(B, T), "k": mrows[M:2 * M].view(B, T), "v": mrows[2 * M:].view(B, T),
            "resid": K.dropout_mask(M * d, p, seed + 1, dev).float().cpu().view(B, T, d) * sc,
            "mlp": K.dropout_mask(M * d, p, seed + 2, dev).float().cpu().view(B, T, d) * sc}
    for nm, m in drop.items():
        kept = float((m > 0).float().mean())
        sigma = math.sqrt(p * (1 - p) / m.numel())
        assert abs(kept - (1 - p)) < 6 * sigma, (nm, kept)
    yr, dxr, gr = _block_oracle(sd, x, dy, H, True, drop=drop)
    check(f"dropout {p} block fwd vs bf16 oracle", relerr(y.detach().cpu() - x, yr - x), 1e-3)
    y.backward(dy.to(dev))
    check(f"dropout {p} dx", relerr(xd.grad, dxr), 1e-2)
    for n, prm in blk.named_parameters():
        check(f"dropout {p} d{n}", relerr(prm.grad, gr[n]), 1e-2)
    blk.eval()  # eval mode: no dropout, identical to a p = 0 block
    with torch.no_grad():
        y0 = blk(x.to(dev))
    yr0, _, _ = _block_oracle(sd, x, dy, H, True)
    check(f"dropout {p} eval fwd", relerr(y0.cpu() - x, yr0 - x), 1e-3)


@pytest.mark.parametrize("dbl", [False, True])
def test_block_gradient_checkpointing(dev, dbl):
    """enable_gradient_checkpointing (commons/transformers/layers.py:374-380): in training
    the block's saved activations are recomputed in the backward. With dropout on (seeds
    drawn from the CPU generator, restored for the recompute) outputs and gradients equal
    the non-checkpointed block's (outputs bit for bit), and the activations kept between forward and
    backward shrink to the block input."""
    B, T, d, H = 8, 129, 256, 4
    blk, sd, x, dy = _rand_block(dev, B, T, d, H, seed=5, dropout=0.1)
    blk.train()
    res = {}
    for ck in (False, True):
        blk.enable_gradient_checkpointing = ck
        blk.zero_grad(set_to_none=True)
        xd = x.to(dev).requires_grad_(True)
        torch.cuda.synchronize()
        m0 = torch.cuda.memory_allocated(dev)
        torch.manual_seed(123)
        y = blk.forward_double_residual(xd) if dbl else blk(xd)
        torch.cuda.synchronize()
        kept = torch.cuda.memory_allocated(dev) - m0 - y.numel() * y.element_size()
        torch.manual_seed(999)  # the recompute must not depend on the generator's state here
        y.backward(dy.to(dev))
        res[ck] = (y.detach().cpu(), xd.grad.cpu(), {n: p.grad.cpu() for n, p in blk.named_parameters()}, kept)
    (y0, dx0, g0, kept0), (y1, dx1, g1, kept1) = res[False], res[True]
    assert torch.equal(y0, y1)
    # same kernels on the same operands; the bias gradient's LDS float atomics may sum
    # in another order, so the gradients are held to 1e-5 rather than bit equality
    check("ckpt dx", relerr(dx1, dx0), 1e-5)
    for n in g0:
        check(f"ckpt d{n}", relerr(g1[n], g0[n]), 1e-5)
    assert kept1 < kept0 / 4, (kept0, kept1)


@pytest.mark.parametrize("idx", [0, 1])
def test_transformer_block_attn_mask_golden(dev, idx):
    """TransformerBlock.forward(x, attn_mask) with a general additive [B, 1, T, T] mask
    (random scores, -inf on padded keys), causal and not (commons/transformers/layers.py:
    374, :404-408; SDPA :57-58), vs the reference's own outputs and gradients
    (tests/golden/transformer_block_mask_*.npz) and vs the bf16-operand oracle."""
    from recommendations_amd.commons.transformers.layers import TransformerBlock
    g = golden(f"transformer_block_mask_{idx}")
    d, H, causal, pos = int(g["d"]), int(g["H"]), bool(g["causal"]), int(g["context_window"])
    blk = TransformerBlock(_cfg(d, H, True, causal, pos)).to(dev)
    sd = {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("p_")}
    blk.load_state_dict(sd)
    mask = torch.from_numpy(g["mask"])
    x = torch.from_numpy(g["x"]).to(dev).requires_grad_(True)
    dy = torch.from_numpy(g["dy"])
    y = blk(x, mask.to(dev))
    check("masked block fwd vs reference", relerr(y.detach(), g["out"]), 2e-2)
    yr, dxr, gr = _block_oracle(sd, x, dy, H, causal, attn_mask=mask)
    check("masked block fwd vs bf16 oracle", relerr(y.detach() - x.detach(), yr - x.detach().cpu()), 1e-3)
    y.backward(dy.to(dev))
    check("masked block dx vs reference", relerr(x.grad, g["dx"]), 3e-2)
    check("masked block dx vs bf16 oracle", relerr(x.grad, dxr), 1e-2)
    for n, p in blk.named_parameters():
        check(f"masked block d{n} vs reference", relerr(p.grad, g["g_" + n]), 3e-2)
        check(f"masked block d{n} vs bf16 oracle", relerr(p.grad, gr[n]), 1e-2)


def test_attn_mask_errors(dev):
    from recommendations_amd import kernels as K
    with pytest.raises(RuntimeError):  # does not broadcast onto [B, H, T, T]
        K.attn_mask_operand(torch.zeros(3, 5, 7, device=dev), 2, 1, 7)
    with pytest.raises(RuntimeError):  # general masks: T <= 256
        K.attn_mask_operand(torch.zeros(300, 300, device=dev), 1, 1, 300)


@pytest.mark.parametrize("M,N,res,twice", [(2048, 1024, 2, False), (1000, 768, 1, True), (257, 512, 0, False),
                                           (5, 64, 1, False), (33000, 1024, 1, True)])
def test_dgrad_layernorm_bwd_vs_fp64(dev, M, N, res, twice):
    """lthm_dgrad_layernorm_bwd (the c_fc / c_attn dgrad fused with the LayerNorm backward,
    commons/transformers/layers.py:142-149, :271-284) against fp64 on the same bf16 operands:
    dh = dy W, dx = LN'(dh) + res1 + res2 (+ res1 with the fold flag), dw = sum dh xhat,
    db = sum dh.  dh stays f32 on chip: 1e-5 relative Frobenius on dx (f32 accumulation
    order), 1e-5 on dw / db; the bf16 copy 4e-3 (bf16 rounding).  Also against the unfused
    pair (bf16 dh), within the bf16 rounding of dh."""
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(M + N + res)
    dy = bf(torch.randn(M, N, generator=g))
    W = bf(torch.randn(N, 256, generator=g) / math.sqrt(N))
    x = torch.randn(M, 256, generator=g) * 2 + 0.5
    w = torch.randn(256, generator=g) * 0.5 + 1
    mu = x.double().mean(1)
    rs = 1.0 / torch.sqrt(x.double().var(1, unbiased=False) + 1e-5)
    r1 = torch.randn(M, 256, generator=g) if res >= 1 else None
    r2 = torch.randn(M, 256, generator=g) if res >= 2 else None
    d = lambda t: None if t is None else t.to(dev)
    assert K.dgrad_layernorm_bwd_ok(d(dy), d(W), d(x))
    dx, dxb, dw, db = K.dgrad_layernorm_bwd(d(dy), d(W), d(x), d(w), d(mu.float()), d(rs.float()), res1=d(r1),
                                            res2=d(r2), res1_twice=twice)
    torch.cuda.synchronize()
    dh = dy.double() @ W.double()
    xh = (x.double() - mu[:, None]) * rs[:, None]
    gg = dh * w.double()
    want = rs[:, None] * (gg - gg.mean(1, keepdim=True) - xh * (gg * xh).mean(1, keepdim=True))
    if r1 is not None:
        want = want + r1.double()
    if r2 is not None:
        want = want + r2.double()
    check("dx bf16 copy", relerr(dxb.float(), want), 4e-3)
    if twice:
        want = want + r1.double()
    check("dx", relerr(dx, want), 1e-5)
    check("dw", relerr(dw, (dh * xh).sum(0)), 1e-5)
    check("db", relerr(db, dh.sum(0)), 1e-5)
    # the unfused pair: bf16 dh written by the GEMM, then lthm_layernorm_bwd_ex
    dh_b = K.linear_dgrad(d(dy), d(W))
    ux, _, uw, ub = K.layernorm_bwd(dh_b, d(x), d(w), d(mu.float()), d(rs.float()), res1=d(r1), res2=d(r2),
                                    res1_twice=twice)
    check("dx vs unfused", relerr(dx, ux), 4e-3)
    check("dw vs unfused", relerr(dw, uw), 4e-3)


@pytest.mark.parametrize("M,Kd,bias,res", [(2048, 256, True, True), (1000, 256, False, True), (7, 64, True, False),
                                           (33001, 512, True, True)])
def test_linear_layernorm_fwd_vs_fp64(dev, M, Kd, bias, res):
    """lthm_linear_layernorm_fwd (the block's c_proj + residual, then ln_2: commons/transformers/
    layers.py:264, :371, :142-149) against fp64 on the same bf16 operands: x1 1e-6 relative
    Frobenius (f32 accumulation), h 4e-3 (bf16 output), mean / rstd 1e-5; and against the
    unfused pair (persistent GEMM with the residual epilogue, then lthm_layernorm_fwd)."""
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(M + Kd)
    x = bf(torch.randn(M, Kd, generator=g))
    W = bf(torch.randn(256, Kd, generator=g) / math.sqrt(Kd))
    b = torch.randn(256, generator=g) if bias else None
    r = torch.randn(M, 256, generator=g) * 3 + 1 if res else None
    lw = torch.randn(256, generator=g) * 0.3 + 1
    lb = torch.randn(256, generator=g) * 0.1
    d = lambda t: None if t is None else t.to(dev)
    assert K.linear_layernorm_fwd_ok(d(x), d(W), d(b), d(r), d(lw), d(lb))
    # an operand the epilogue cannot read directly sends the caller to the unfused path
    assert not K.linear_layernorm_fwd_ok(d(x), d(W), d(b), d(torch.randn(M, 256).to(torch.bfloat16)), d(lw), d(lb))
    assert not K.linear_layernorm_fwd_ok(d(x), d(W), d(b), d(r), None, d(lb))
    x1, h, mu, rs = K.linear_layernorm_fwd(d(x), d(W), d(b), d(r), d(lw), d(lb))
    torch.cuda.synchronize()
    want = x.double() @ W.double().T
    if b is not None:
        want = want + b.double()
    if r is not None:
        want = want + r.double()
    m64 = want.mean(1)
    r64 = 1.0 / torch.sqrt(want.var(1, unbiased=False) + 1e-5)
    h64 = (want - m64[:, None]) * r64[:, None] * lw.double() + lb.double()
    check("x1", relerr(x1, want), 1e-6)
    check("h", relerr(h.float(), h64), 4e-3)
    check("mean", relerr(mu, m64), 1e-5)
    check("rstd", relerr(rs, r64), 1e-5)
    ux = K.linear_fwd(d(x), d(W), d(b), res1=d(r), out_dtype=torch.float32)
    uh, um, ur = K.layernorm_fwd(ux, d(lw), d(lb))
    check("x1 vs unfused", relerr(x1, ux), 1e-6)
    check("h vs unfused", relerr(h.float(), uh.float()), 4e-3)
