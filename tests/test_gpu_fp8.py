"""GPU parity of the fp8 encoder path (BASELINE.json configs[4], C5: CDNA4 fp8 MFMA
for the encoder GEMMs).

* quantize_fp8 is bit-exact to torch's float8_e4m3fn cast of clamp(x / scale)
  with scale = amax / 448 (round-to-nearest-even);
* the fp8 GEMM (v_mfma_scale_f32_16x16x128_f8f6f4, unit block scales) equals the
  fp64 product of the dequantised operands to 3e-5 relative Frobenius (exact
  products, f32 accumulation inside the 128-deep MFMA), through every epilogue form;
* a C5-shaped TransformerBlock (T' = 513, d = 512, H = 8) in fp8 mode vs the fp32
  reference: the forward differs by the recipe's own quantisation error (e4m3 carries
  3 mantissa bits; measured 5.0e-2 relative Frobenius, bound 8e-2), the bf16 backward
  (which runs on the saved bf16 activations) by 4.6e-3 on dx (bound 1e-2) and at most
  4.3e-2 on a parameter gradient (bound 9e-2).  Parity proper is the GEMM test above.
"""
import math

import pytest
import torch

from parity import check, relerr
import torch.nn.functional as F

from oracle import ref

pytestmark = pytest.mark.gpu




def _deq(q, s):
    return q.cpu().view(torch.float8_e4m3fn).double() * float(s.cpu())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_quantize_fp8_bit_exact(dev, dtype):
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(1)
    x = (torch.randn(4096, 256, generator=g) * 3).to(dtype)
    x[0, 0] = 77.0
    q, s = K.quantize_fp8(x.to(dev))
    amax = x.float().abs().max()
    sc = amax / 448.0
    assert float(s.cpu()) == float(sc)
    exp = (x.float() / sc).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    assert torch.equal(q.cpu(), exp)


def _amax_word(t):
    return int(t.float().abs().max().view(torch.int32))


@pytest.mark.parametrize("D,ydt", [(512, torch.bfloat16), (256, torch.float32), (70, torch.bfloat16)])
def test_layernorm_amax_fused(dev, D, ydt):
    """layernorm_fwd(amax=) folds max |y| (of the stored y) into the word, and
    quantize_fp8(amax=) then equals the two-pass quantize_fp8 bit for bit."""
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(D)
    M = 3001 if D != 70 else 4000
    x = (torch.randn(M, D, generator=g) * 2 + 0.5).to(dev)
    w = (1 + 0.3 * torch.randn(D, generator=g)).to(dev)
    b = (0.2 * torch.randn(D, generator=g)).to(dev)
    am = torch.zeros(1, dtype=torch.int32, device=dev)
    y, mu, rs = K.layernorm_fwd(x, w, b, y_dtype=ydt, amax=am)
    y0, _, _ = K.layernorm_fwd(x, w, b, y_dtype=ydt)
    assert torch.equal(y, y0)
    assert int(am.cpu()) == _amax_word(y0.cpu())
    q, s = K.quantize_fp8(y, amax=am)
    q0, s0 = K.quantize_fp8(y0)
    assert torch.equal(q.cpu(), q0.cpu()) and float(s.cpu()) == float(s0.cpu())


@pytest.mark.parametrize("M,N,K,act,odt", [(40000, 2048, 512, 5, torch.bfloat16), (5000, 512, 512, 0, torch.float32),
                                           (333, 256, 128, 1, torch.bfloat16)])
def test_fp8_gemm_amax_out(dev, M, N, K, act, odt):
    """The GEMM epilogue's amax_out equals max |C| of the stored C (fp8 GEMM, persistent
    kernel; and the bf16 one-tile kernel's pass over C for a small M)."""
    from recommendations_amd import kernels as K_
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(torch.bfloat16).to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=dev) if act else None
    am = torch.zeros(1, dtype=torch.int32, device=dev)
    xq, xs = K_.quantize_fp8(x)
    wq, ws = K_.quantize_fp8(w)
    out = K_.linear_fwd_fp8(xq, xs, wq, ws, bias, act=act, aux_out=pre, out_dtype=odt, amax_out=am)
    assert int(am.cpu()) == _amax_word(out.cpu())
    am2 = torch.zeros(1, dtype=torch.int32, device=dev)
    out2 = K_.gemm(x, w, M, N, K, bias=bias, act=act, aux_out=pre, out_dtype=odt, amax_out=am2)
    assert int(am2.cpu()) == _amax_word(out2.cpu())
    am3 = torch.zeros(1, dtype=torch.int32, device=dev)
    K_.amax_(out2, am3)
    assert int(am3.cpu()) == int(am2.cpu())


@pytest.mark.parametrize("M,N,K,act,res", [(40000, 1536, 512, 0, 0), (333, 2048, 512, 1, 0),
                                           (20000, 512, 2048, 0, 2), (5000, 512, 512, 0, 1),
                                           (70001, 768, 256, 2, 0)])
def test_fp8_gemm_vs_dequantised(dev, M, N, K, act, res):
    from recommendations_amd import kernels as K_
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g)
    xq, xs = K_.quantize_fp8(x.to(dev))
    wq, ws = K_.quantize_fp8(w.to(dev))
    r1 = torch.randn(M, N, generator=g) if res >= 1 else None
    r2 = torch.randn(M, N, generator=g) if res >= 2 else None
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=dev) if act else None
    out = K_.linear_fwd_fp8(xq, xs, wq, ws, bias.to(dev), act=act, aux_out=pre,
                            res1=None if r1 is None else r1.to(dev), res2=None if r2 is None else r2.to(dev),
                            out_dtype=torch.float32)
    z = _deq(xq, xs) @ _deq(wq, ws).T + bias.double()
    exp = {0: z, 1: F.gelu(z, approximate="tanh"), 2: z * torch.sigmoid(1.702 * z)}[act]
    if r1 is not None:
        exp = exp + r1.double()
    if r2 is not None:
        exp = exp + r2.double()
    check('out, exp', relerr(out, exp), 3e-5)
    if act:
        check('pre.float(), z', relerr(pre.float(), z), 1e-2)


def test_transformer_block_fp8_c5_shape(dev):
    from recommendations_amd.commons.transformers.configs import TransformerConfig
    from recommendations_amd.commons.transformers.layers import TransformerBlock
    torch.manual_seed(0)
    B, T, d, H = 2, 513, 512, 8
    cfg = TransformerConfig(rotator_config={"ff_mult": 4}, is_causal=True, fp8_gemm=True,
                            attn_config=dict(attn_dropout=0.0, bias=True, dropout=0.0, n_head=H, n_embd=d,
                                             attn_type="multi_head", pos_bias={"context_window": T}))
    blk = TransformerBlock(cfg)
    with torch.no_grad():
        for n, p in blk.named_parameters():
            if "pos_bias" in n or "ln_" in n or n.endswith("bias"):
                p.add_(0.05 * torch.randn(p.shape))
    sd = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    blk = blk.to(dev)
    x = torch.randn(B, T, d)
    xd = x.to(dev).requires_grad_(True)
    y = blk(xd)
    xr = x.clone().requires_grad_(True)
    pr = {k: v.clone().requires_grad_(True) if v.is_floating_point() else v for k, v in sd.items()}
    yr = ref.transformer_block(xr, pr, H, True)
    # residual stream included: compare the block's update y - x (the part the GEMMs produce)
    check('y.detach().cpu() - x, yr.detach() - x', relerr(y.detach().cpu() - x, yr.detach() - x), 8e-2)
    dy = torch.randn(B, T, d)
    y.backward(dy.to(dev))
    yr.backward(dy)
    check('xd.grad, xr.grad', relerr(xd.grad, xr.grad), 1e-2)
    for n, p in blk.named_parameters():
        if pr[n].grad is not None and float(pr[n].grad.norm()) > 0:
            check(f"p.grad, pr[n].grad {n}", relerr(p.grad, pr[n].grad), 9e-2)
