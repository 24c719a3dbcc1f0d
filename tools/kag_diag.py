"""Diagnose a bit-exactness gap of lthm_kshift_adagrad_fused against oracle/ref.py
kshift_adagrad_ref: which rows differ, their pair counts, and whether a plain sequential sum
(no chunking) or the f64 sum matches them instead."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import ref  # noqa: E402


def main():
    from recommendations_amd import kernels as KK
    dev = torch.device("cuda:0")
    K, D, P, n = 16, 32, 1000, 3000
    rng = np.random.default_rng(7 * K + D)
    ids = rng.integers(0, 2 ** 63 - 1, size=(n, 1), dtype=np.int64)
    neg = rng.random((n, 1)) < 0.5
    ids[neg] = -ids[neg] - 1
    W0 = rng.standard_normal((P, D)).astype(np.float32)
    S0 = (np.abs(rng.standard_normal((P, D))).astype(np.float32) * 0.1).astype(np.float32)
    dY = rng.standard_normal((n, D)).astype(np.float32)
    W = torch.from_numpy(W0).to(dev)
    S = torch.from_numpy(S0).to(dev)
    KK.kshift_adagrad_fused(torch.from_numpy(ids).to(dev), torch.from_numpy(dY).to(dev), None, None, P, K, 0, 1, W, S,
                            0.5, 1e-10)
    Wg, Sg = W.cpu().numpy(), S.cpu().numpy()
    g = ref.kshift_pool_grad(dY, K, 0)
    Wo, So = ref.kshift_adagrad_ref(ids, g, P, K, 1, W0, S0, 0.5, 1e-10)
    Wq, Sq = ref.kshift_adagrad_ref(ids, g, P, K, 1, W0, S0, 0.5, 1e-10, ch=10 ** 9)  # no chunking
    rows = ref.kshift_rows(ids.reshape(-1), P, K).reshape(-1)
    cnt = np.bincount(rows, minlength=P)
    bad = np.nonzero((Wg != Wo).any(1) | (Sg != So).any(1))[0]
    print("rows differing:", bad.size, "of", (cnt > 0).sum(), "touched")
    for r in bad[:12]:
        print(f"row {r} pairs {cnt[r]} |dW| {np.abs(Wg[r] - Wo[r]).max():.3e} |dS| {np.abs(Sg[r] - So[r]).max():.3e} "
              f"seq-match {np.array_equal(Wg[r], Wq[r]) and np.array_equal(Sg[r], Sq[r])}")
    # the recovered per-row gradient from the state change: s1 - s0 = g^2
    r = bad[0] if bad.size else P - 1
    gg = np.sqrt(np.maximum(Sg[r].astype(np.float64) - S0[r], 0))
    go = np.sqrt(np.maximum(So[r].astype(np.float64) - S0[r], 0))
    print("row", r, "|g| gpu", gg[:4], "oracle", go[:4])


if __name__ == "__main__":
    main()
