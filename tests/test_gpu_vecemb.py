"""GPU parity of the vector-feature layers (csrc/vecemb.hip, include/lthm.h lthm_rowproj_fwd /
lthm_l2norm_rows* / lthm_cosine_wgrad / lthm_gauss_bins_*): SimhashVectorIndexer, CosineLinear,
LearnableCosineVectorEmbedding and ProbabilityVectorEmbedding (commons/transformers/layers.py:
426-437, 517-595) against the reference's own outputs (tests/golden/, made by importing the
reference) and against the oracle (oracle/ref.py) on larger seeded inputs.

Bounds: SimHash codes bit-exact (a sign bit may differ only where |x . proj| is at f32
rounding level, checked against the oracle's f32 products); CosineLinear and the gaussian
bins are f32 end to end (relative Frobenius 1e-5); the two embeddings feed bf16 bins into the
bf16 MFMA GEMM of their output Linear (north star: bf16 activations), relative 6e-3 (8e-3
for gradients), about 2x the measured error."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref
from parity import check, relerr

pytestmark = pytest.mark.gpu

T = torch.from_numpy


def _load(mod, **tensors):
    with torch.no_grad():
        for name, v in tensors.items():
            obj = mod
            *path, leaf = name.split(".")
            for pth in path:
                obj = getattr(obj, pth)
            getattr(obj, leaf).copy_(T(v))
    return mod


@pytest.mark.parametrize("tag", ["simhash", "simhash63"])
def test_simhash_golden(dev, tag):
    from recommendations_amd.commons.transformers.layers import SimhashVectorIndexer
    g = golden(tag)
    dim, P = g["projection_mat"].shape
    sv = _load(SimhashVectorIndexer(dim, P), projection_mat=g["projection_mat"]).to(dev)
    out = sv(T(g["x"]).to(dev))
    assert out.dtype == torch.int64 and out.shape == g["out"].shape
    assert np.array_equal(out.cpu().numpy(), g["out"])


@pytest.mark.parametrize("rows,dim,P", [(100_000, 64, 16), (4097, 37, 5), (3000, 128, 64), (1, 8, 1)])
def test_simhash_vs_oracle(dev, rows, dim, P):
    from recommendations_amd import kernels as K
    gen = torch.Generator().manual_seed(rows + dim + P)
    x = torch.randn(rows, dim, generator=gen)
    proj = torch.randn(dim, P, generator=gen) / dim ** 0.5
    got = K.simhash(x.to(dev), proj.to(dev)).cpu()
    exp = ref.simhash(x, proj)
    diff = (got ^ exp)
    z = (x.double() @ proj.double()).abs()
    # a differing bit must sit on a product within f32 rounding of zero
    for r in torch.nonzero(diff).flatten().tolist():
        bits = int(diff[r]) & ((1 << P) - 1) if P < 64 else int(diff[r])
        for j in range(P):
            if bits >> j & 1:
                assert float(z[r, j]) < 1e-5, (r, j, float(z[r, j]))
    check("simhash codes differing (f32 near-zero products only)", float((diff != 0).float().mean()), 1e-3)


def test_cosine_linear_golden(dev):
    from recommendations_amd.commons.transformers.layers import CosineLinear
    g = golden("cosine_linear")
    out_dim, dim = g["weight"].shape
    cl = _load(CosineLinear(dim, out_dim), weight=g["weight"]).to(dev)
    x = T(g["x"]).to(dev).requires_grad_(True)
    y = cl(x)
    y.backward(T(g["dy"]).to(dev))
    check("CosineLinear fwd vs reference", relerr(y, g["out"]), 1e-5)
    check("CosineLinear dx vs reference", relerr(x.grad, g["dx"]), 1e-5)
    check("CosineLinear dW vs reference", relerr(cl.weight.grad, g["dweight"]), 1e-5)


@pytest.mark.parametrize("rows,dim,P", [(65_536, 256, 16), (1000, 300, 96), (7, 5, 3)])
def test_cosine_linear_vs_oracle(dev, rows, dim, P):
    from recommendations_amd import kernels as K
    gen = torch.Generator().manual_seed(rows + dim)
    x = torch.randn(rows, dim, generator=gen)
    x[0] = 0.0  # F.normalize's eps branch
    w = torch.randn(P, dim, generator=gen)
    dy = torch.randn(rows, P, generator=gen)
    xd, wd = x.to(dev).requires_grad_(True), w.to(dev).requires_grad_(True)
    y = K.CosineLinearFn.apply(xd, wd)
    y.backward(dy.to(dev))
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    yr = ref.cosine_linear(xr, wr)
    yr.backward(dy)
    check("CosineLinear fwd vs oracle", relerr(y, yr), 1e-5)
    check("CosineLinear dx vs oracle", relerr(xd.grad, xr.grad), 1e-5)
    check("CosineLinear dW vs oracle", relerr(wd.grad, wr.grad), 1e-5)


@pytest.mark.parametrize("n,P,nb,tk", [(200_000, 16, 20, 0), (50_000, 16, 20, 5), (10_001, 3, 7, 3),
                                       (4096, 4, 64, 10), (100, 1, 10, 0), (999, 2, 33, 32)])
def test_gauss_bins_vs_oracle(dev, n, P, nb, tk):
    """The f32 gaussian bins alone: fwd and the gradients to z and to the mean."""
    from recommendations_amd import kernels as K
    gen = torch.Generator().manual_seed(n + nb)
    z = torch.rand(n, P, generator=gen) * 2.4 - 1.2
    mean = torch.rand(P, nb, generator=gen) * 2 - 1
    sigma2 = (1.3 * 2.0 / nb) ** 2
    g = torch.randn(n, P, nb, generator=gen)
    zd, md = z.to(dev).requires_grad_(True), mean.to(dev).requires_grad_(True)
    y = K.GaussBinsFn.apply(zd, md, sigma2, tk, torch.float32).view(n, P, nb)
    y.backward(g.to(dev))
    zr, mr = z.clone().requires_grad_(True), mean.clone().requires_grad_(True)
    yr = ref.gaussian_bins(zr, mr, sigma2, tk or None)
    yr.backward(g)
    check("gaussian bins fwd vs oracle", relerr(y, yr), 1e-5)
    check("gaussian bins dz vs oracle", relerr(zd.grad, zr.grad), 1e-4)
    check("gaussian bins dmean vs oracle", relerr(md.grad, mr.grad), 1e-4)


@pytest.mark.parametrize("tag", ["lcve", "lcve_top5", "lcve_nb7"])
def test_learnable_cve_golden(dev, tag):
    from recommendations_amd.commons.transformers.layers import LearnableCosineVectorEmbedding
    g = golden(tag)
    n_proj, dim = g["proj_weight"].shape
    nb = g["mean"].shape[-1]
    tk = int(g["top_k"]) or None
    m = LearnableCosineVectorEmbedding(dim, g["emb_weight"].shape[0], n_proj=n_proj, num_bins=nb, top_k=tk)
    m.sigma2 = float(g["sigma2"])
    m = _load(m, **{"proj.weight": g["proj_weight"], "mean": g["mean"], "emb.weight": g["emb_weight"]}).to(dev)
    x = T(g["x"]).to(dev).requires_grad_(True)
    y = m(x)
    y.backward(T(g["dy"]).to(dev))
    check(f"{tag} fwd vs reference (bf16 GEMM)", relerr(y, g["out"]), 6e-3)
    check(f"{tag} dx vs reference", relerr(x.grad, g["dx"]), 8e-3)
    check(f"{tag} dproj vs reference", relerr(m.proj.weight.grad, g["dproj_weight"]), 8e-3)
    check(f"{tag} dmean vs reference", relerr(m.mean.grad, g["dmean"]), 8e-3)
    check(f"{tag} demb vs reference", relerr(m.emb.weight.grad, g["demb_weight"]), 6e-3)
    # the f32 gaussian_kernel on its own matches the oracle tightly
    with torch.no_grad():
        z = m.proj(x)
        gk = m.gaussian_kernel(z)
    exp = ref.gaussian_bins(z.cpu(), T(g["mean"]), float(g["sigma2"]), tk)
    check(f"{tag} gaussian_kernel vs oracle", relerr(gk, exp), 1e-5)


@pytest.mark.parametrize("tag", ["pve", "pve_top3"])
def test_probability_ve_golden(dev, tag):
    from recommendations_amd.commons.transformers.layers import ProbabilityVectorEmbedding
    g = golden(tag)
    nb = g["mean"].shape[-1]
    m = ProbabilityVectorEmbedding(g["emb_weight"].shape[0], num_bins=nb, top_k=int(g["top_k"]) or None)
    m.sigma2 = float(g["sigma2"])
    m = _load(m, mean=g["mean"], **{"emb.weight": g["emb_weight"]}).to(dev)
    x = T(g["x"]).to(dev).requires_grad_(True)
    y = m(x)
    y.backward(T(g["dy"]).to(dev))
    check(f"{tag} fwd vs reference (bf16 GEMM)", relerr(y, g["out"]), 6e-3)
    check(f"{tag} dx vs reference", relerr(x.grad, g["dx"]), 8e-3)
    check(f"{tag} dmean vs reference", relerr(m.mean.grad, g["dmean"]), 8e-3)
    check(f"{tag} demb vs reference", relerr(m.emb.weight.grad, g["demb_weight"]), 6e-3)
    with pytest.raises(RuntimeError):
        m(torch.zeros(4, 2, device=dev))


def test_learnable_cve_large_vs_oracle(dev):
    """C2-sized sequence input (bs 64, seq 129, dim 256, 16 projections, 20 bins, top-5)."""
    from recommendations_amd.commons.transformers.layers import LearnableCosineVectorEmbedding
    torch.manual_seed(7)
    m = LearnableCosineVectorEmbedding(256, 128, n_proj=16, num_bins=20, top_k=5)
    x = torch.randn(64, 129, 256)
    dy = torch.randn(64, 129, 128)
    pw, mean, ew = (p.detach().clone().requires_grad_(True) for p in (m.proj.weight, m.mean, m.emb.weight))
    xr = x.clone().requires_grad_(True)
    yr = ref.learnable_cve(xr, pw, mean, ew, m.sigma2, 5)
    yr.backward(dy)
    m = m.to(dev)
    xd = x.to(dev).requires_grad_(True)
    y = m(xd)
    y.backward(dy.to(dev))
    check("LCVE C2-size fwd vs oracle", relerr(y, yr), 6e-3)
    check("LCVE C2-size dx vs oracle", relerr(xd.grad, xr.grad), 8e-3)
    check("LCVE C2-size dmean vs oracle", relerr(m.mean.grad, mean.grad), 8e-3)
    check("LCVE C2-size demb vs oracle", relerr(m.emb.weight.grad, ew.grad), 6e-3)
