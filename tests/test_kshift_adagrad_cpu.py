"""Pin the fused dedup + Adagrad restatement (oracle/ref.py kshift_adagrad_ref, the order
lthm_kshift_adagrad_fused sums in) to the reference's own update: torch.optim.Adagrad over the
dense table, with the table gradient autograd forms through the KShift pool
(embedding_module_gen.py:137,151-153: loss.backward(); optim.step(); commons/layers.py:152-172).
CPU only; the two differ by f32 summation order alone."""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ref


def _pool_torch(ids, W, P, K, F_, mode):
    """[n, F] ids -> [n * F, D] pooled rows of the table-batched W (table f: rows f P ..)."""
    outs = []
    for f in range(F_):
        Wf = W[f * P:(f + 1) * P]
        x = ref.kshift_fwd_torch(torch.from_numpy(ids[:, f]), Wf, K, False) * math.sqrt(K)  # the plain sum
        if mode == 0:
            x = x / math.sqrt(K)
        elif mode == 1:
            x = F.normalize(x, p=2.0, dim=-1)
        outs.append(x)
    return torch.stack(outs, 1).reshape(-1, W.shape[1])


@pytest.mark.parametrize("mode,K,F_,D", [(0, 16, 1, 32), (1, 16, 1, 8), (2, 1, 3, 4), (0, 8, 2, 20)])
def test_kshift_adagrad_ref_matches_torch_adagrad(mode, K, F_, D):
    rng = np.random.default_rng(100 * K + D)
    P, n, lr, eps = 97, 600, 0.5, 1e-10
    W0 = rng.standard_normal((F_ * P, D)).astype(np.float32)
    S0 = np.abs(rng.standard_normal((F_ * P, D))).astype(np.float32)
    W = torch.from_numpy(W0.copy()).requires_grad_(True)
    opt = torch.optim.Adagrad([W], lr=lr, eps=eps, foreach=False)
    opt.state[W]["sum"] = torch.from_numpy(S0.copy())
    opt.state[W]["step"] = torch.tensor(0.0)
    Wo, So = W0, S0
    for step in range(2):
        # full-range ids, about half negative: every shifted row of a negative id is row P - 1,
        # so that row takes the long (chunked) path for K > 1
        ids = rng.integers(-2 ** 63, 2 ** 63 - 1, size=(n, F_), dtype=np.int64)
        dY = rng.standard_normal((n * F_, D)).astype(np.float32)
        y = _pool_torch(ids, W, P, K, F_, mode)
        (y * torch.from_numpy(dY)).sum().backward()
        opt.step()
        opt.zero_grad()
        out = norms = None
        if mode == 1:
            x = ref.kshift_fwd_c(ids[:, 0], Wo, K, 2)
            norms = np.linalg.norm(x.astype(np.float64), axis=-1).astype(np.float32)
            out = (x / np.maximum(norms, 1e-12)[:, None]).astype(np.float32)
        g = ref.kshift_pool_grad(dY, K, mode, out, norms)
        Wo, So = ref.kshift_adagrad_ref(ids, g, P, K, F_, Wo, So, lr, eps)
        if K > 1:
            rows = ref.kshift_rows(ids.reshape(-1), P, K)
            assert (rows == P - 1).sum() > 256  # the long path ran
    np.testing.assert_allclose(Wo, W.detach().numpy(), rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(So, opt.state[W]["sum"].numpy(), rtol=2e-5, atol=2e-5)
