"""GPU parity of the 256 x 256 big-K GEMM (csrc/gemm.hip gemm_bt_k: both operands K-contiguous,
K > 256, M >= 4096, N >= 512 -- the ranker MLPs and the C5 encoder forms) against the fp32
oracle on the SAME bf16 operands: every epilogue form the layer code uses (bias + QuickGELU /
GELU with the pre-activation store, the activation-gradient multiply, the residual add) and
ragged M / N / K edges.  Bound: 1e-5 relative Frobenius for f32 outputs (fp32 accumulation in
another order), 1e-3 for bf16 outputs (one bf16 rounding)."""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import ref
from parity import check, relerr

pytestmark = pytest.mark.gpu


def bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("M,N,Kd", [(8192, 1024, 2176), (4100, 520, 1056), (65536, 512, 1024), (4096, 520, 288)])
@pytest.mark.parametrize("act", [0, 2, 1])
def test_gemm_bigk_forward_epilogues(dev, M, N, Kd, act):
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(M + N + Kd + act)
    A = bf(torch.randn(M, Kd, generator=g))
    W = bf(torch.randn(N, Kd, generator=g) / math.sqrt(Kd))
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    z = A.float() @ W.float().T + bias
    if act == 0:  # bias + residual, f32 out
        out = K.linear_fwd(A.to(dev), W.to(dev), bias=bias.to(dev), res1=res.to(dev), out_dtype=torch.float32)
        check(f"bigk fwd res ({M},{N},{Kd})", relerr(out, z + res), 1e-5)
        return
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    out = K.linear_fwd(A.to(dev), W.to(dev), bias=bias.to(dev), act=act, aux_out=pre)
    exp = ref.quick_gelu(z) if act == 2 else F.gelu(z, approximate="tanh")
    check(f"bigk fwd act{act} ({M},{N},{Kd})", relerr(out.float(), bf(exp).float()), 1e-3)
    check(f"bigk pre-activation ({M},{N},{Kd})", relerr(pre.float(), bf(z).float()), 1e-3)


@pytest.mark.parametrize("M,N,Kd", [(65536, 1024, 512), (8192, 2176, 1024), (5000, 520, 2048)])
def test_gemm_bigk_dgrad(dev, M, N, Kd):
    """dX = (dY W) [* QuickGELU'(pre)] with K = the dY width > 256: the dgrad forms of the ranker."""
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(3 * M + N)
    dy = bf(torch.randn(M, Kd, generator=g))
    W = bf(torch.randn(Kd, N, generator=g) / math.sqrt(Kd))
    pre = bf(torch.randn(M, N, generator=g))
    dx = K.linear_dgrad(dy.to(dev), W.to(dev), out_dtype=torch.float32)
    base = dy.float() @ W.float()
    check(f"bigk dgrad ({M},{N},{Kd})", relerr(dx, base), 1e-5)
    dxq = K.linear_dgrad(dy.to(dev), W.to(dev), act_grad=K.ACT_QGELU_GRAD, aux=pre.to(dev), out_dtype=torch.float32)
    p = pre.float().requires_grad_(True)
    ref.quick_gelu(p).backward(base)
    check(f"bigk dgrad qgelu' ({M},{N},{Kd})", relerr(dxq, p.grad), 1e-5)
