"""Deterministic inputs of the contrastive-loss goldens (tests/golden/contrastive_*.npz).

Shared by the generator (make_goldens.py::gen_contrastive, build container only, where
the reference computes the expected outputs) and by the GPU test
(tests/test_gpu_loss_golden.py), which rebuilds the same inputs from the case
parameters and checks them against the sha256 recorded in the fixture, so the
fixtures hold outputs only.

"exact" inputs make every F.normalize and every logit dot product exact in fp32
AND in the bf16 operands the HIP kernels use: each vector is an integer vector
k (|k_i| < 256, so k_i * 2^e is a bf16 value) with sum(k_i^2) = 65536 exactly,
scaled by a random power of two.  Its norm 256 * 2^e is exact, the normalised
vector k / 256 is exact in bf16, and a dot product of two of them is an integer
/ 65536 with |numerator| <= 65536, exact in fp32.  The reference's loss and our
loss then differ only by fp32 summation order and exp rounding.
"""
from __future__ import annotations

import hashlib
from typing import Dict, List

import numpy as np

NORM2 = 65536  # sum of k_i^2 of every exact vector


def _four_squares_table(dmax: int) -> np.ndarray:
    """t[d] = (a, b, c, e) with a^2 + b^2 + c^2 + e^2 = d for every 0 <= d < dmax."""
    t = np.full((dmax, 4), -1, dtype=np.int64)
    r = int(np.sqrt(dmax)) + 1
    for a in range(r):
        for b in range(a, r):
            s2 = a * a + b * b
            if s2 >= dmax:
                break
            for c in range(b, r):
                s3 = s2 + c * c
                if s3 >= dmax:
                    break
                e = np.arange(c, r)
                d = s3 + e * e
                ok = d < dmax
                for ee, dd in zip(e[ok], d[ok]):
                    if t[dd, 0] < 0:
                        t[dd] = (a, b, c, ee)
    assert (t[:, 0] >= 0).all()
    return t


_TABLE = None


def exact_unit_vectors(rng: np.random.Generator, n: int, D: int) -> np.ndarray:
    """[n, D] int64 vectors with sum of squares exactly NORM2 and |k_i| < 256."""
    global _TABLE
    if _TABLE is None:
        _TABLE = _four_squares_table(8192)
    x = rng.standard_normal((n, D - 4))
    s = 0.97 * np.sqrt(NORM2) / np.linalg.norm(x, axis=1, keepdims=True)
    k = np.rint(x * s).astype(np.int64)
    k = np.clip(k, -255, 255)
    d = NORM2 - (k * k).sum(1)
    assert (d >= 0).all() and (d < 8192).all(), (d.min(), d.max())
    fix = _TABLE[d] * rng.choice([-1, 1], size=(n, 4))
    v = np.concatenate([k, fix], axis=1)
    perm = np.argsort(rng.random((n, D)), axis=1)  # scatter the four fix-up components
    v = np.take_along_axis(v, perm, axis=1)
    assert ((v * v).sum(1) == NORM2).all() and np.abs(v).max() < 256
    return v


def left_pad_mask(rng: np.random.Generator, B: int, T: int) -> np.ndarray:
    """[B, T] bool, True = pad, padding on the left (encoder.py:52-54 flips the right-padded
    history).  Sequence 1 is all pad, sequence 2 keeps one token, sequence 3 two."""
    mask = np.zeros((B, T), dtype=bool)
    for b in range(B):
        npad = int(rng.integers(0, T // 2 + 1))
        if b == 1:
            npad = T
        elif b == 2:
            npad = T - 1
        elif b == 3:
            npad = T - 2
        mask[b, :npad] = True
    return mask


# case name -> parameters.  mode: "train" = train_step (mini-batches of mbs, or the whole
# batch in one helper call when mbs < 0); "val" = val_step (whole batch, training=False).
CASES: Dict[str, dict] = {
    # three mini-batches (32, 32, 6), lookahead with draws, pads, short sequences
    "train_ragged": dict(kind="exact", mode="train", B=70, T=48, De=128, lookahead=[0, 2, 5], mbs=32,
                         tau=0.05, beta=0.0, ks=[1, 5, 10, 100], seed=11),
    # val_step over the whole batch: n = 40 * 160 = 6400 > 4096 logit rows
    "val_whole": dict(kind="exact", mode="val", B=40, T=160, De=128, lookahead=[0, 4], mbs=32,
                      tau=0.05, beta=0.0, ks=[1, 10], seed=12),
    # train_mini_batch_size < 0: one helper call over the whole batch (wrapper.py:82-83)
    "train_whole": dict(kind="exact", mode="train", B=24, T=200, De=128, lookahead=[0, 3], mbs=-1,
                        tau=0.05, beta=0.0, ks=[1, 5], seed=13),
    # logQ correction (beta != 0) on random fp32 inputs
    "train_logq": dict(kind="float", mode="train", B=20, T=30, De=128, lookahead=[0, 2, 4], mbs=8,
                       tau=0.05, beta=0.7, ks=[1, 5], seed=14),
    # random fp32 inputs, the reference yaml's lookahead and mini-batch
    "train_float": dict(kind="float", mode="train", B=40, T=64, De=128, lookahead=[0, 5, 6, 12, 24, 30], mbs=32,
                        tau=0.05, beta=0.0, ks=[1, 5, 10, 100], seed=15),
    # the reference yaml's 32-sequence mini-batch at T = 512 (C5): n = 16,384 logit rows
    "train_t512": dict(kind="exact", mode="train", B=32, T=512, De=128, lookahead=[0, 3], mbs=32,
                       tau=0.05, beta=0.0, ks=[1, 10, 100], seed=16),
    # the NaN-row filter (wrapper.py:210-214): a NaN next_token_emb row in mini-batch 0 (head 0)
    # and in mini-batch 1 (head 1) leaves the mean and used_tokens of its (offset, mini-batch);
    # NaN current_token_emb rows in two sequences of mini-batch 2 make every CE of that
    # mini-batch NaN, so it contributes no loss and no per-offset metric at all
    "train_nan": dict(kind="exact", mode="train", B=70, T=24, De=128, lookahead=[0, 2, 5], mbs=32,
                      tau=0.05, beta=0.0, ks=[1, 5], seed=17,
                      nan_y=[(5, 14, 0), (40, 14, 1)], nan_t=[(64, 20), (65, 20)]),
}


def make_inputs(case: dict) -> Dict[str, np.ndarray]:
    """y [B, T+1, NH, De] f32 (next_token_emb), tgt [B, T, De] f32 (current_token_emb),
    mask [B, T] bool (current_token_mask), logq [B, T] f32 (the logQ values the
    reference's _log_q_calc returns; the loss subtracts beta * logQ)."""
    rng = np.random.default_rng(case["seed"])
    B, T, De, NH = case["B"], case["T"], case["De"], len(case["lookahead"])
    if case["kind"] == "exact":
        y = exact_unit_vectors(rng, B * (T + 1) * NH, De).astype(np.float32)
        y *= np.exp2(rng.integers(-3, 4, size=(y.shape[0], 1))).astype(np.float32)
        t = exact_unit_vectors(rng, B * T, De).astype(np.float32)
        t *= np.exp2(rng.integers(-3, 4, size=(t.shape[0], 1))).astype(np.float32)
    else:
        y = rng.standard_normal((B * (T + 1) * NH, De)).astype(np.float32)
        t = rng.standard_normal((B * T, De)).astype(np.float32)
    mask = left_pad_mask(rng, B, T)
    logq = (rng.random((B, T)) * 9.0).astype(np.float32)  # logQ = -log b, b in (1e-4, 1]
    y, t = y.reshape(B, T + 1, NH, De), t.reshape(B, T, De)
    for b, tt, h in case.get("nan_y", []):  # NaN rows (non-pad positions) for the NaN-row filter
        assert not mask[b, min(tt + max(case["lookahead"]), T - 1)], (b, tt)
        y[b, tt, h, :] = np.nan
    for b, tt in case.get("nan_t", []):
        assert not mask[b, tt], (b, tt)
        t[b, tt, :] = np.nan
    return dict(y=y, tgt=t, mask=mask, logq=logq)


def inputs_digest(inp: Dict[str, np.ndarray]) -> str:
    h = hashlib.sha256()
    for k in sorted(inp):
        h.update(k.encode())
        h.update(np.ascontiguousarray(inp[k]).tobytes())
    return h.hexdigest()


def draw_offsets(lookahead: List[int], n_mb: int, seed: int) -> np.ndarray:
    """The offsets wrapper.py:147-153 draws with the global `random` seeded by `seed`:
    per helper call, head 0 takes lookahead[0], head i randint(previous + 1, lookahead[i])."""
    import random
    rng = random.Random(seed)
    out = np.zeros((n_mb, len(lookahead)), dtype=np.int32)
    for mb in range(n_mb):
        prev = 0
        for i, mx in enumerate(lookahead):
            off = mx if i == 0 else rng.randint(prev + 1, mx)
            prev = off
            out[mb, i] = off
    return out
