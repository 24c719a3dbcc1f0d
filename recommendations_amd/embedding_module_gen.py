"""Item-embedding module generation — drop-in for embedding_module_gen.py:32-156
(the Ray task / S3 I/O around it, :161-209, is out of scope).

* ``train_model``: KShiftEmbedding(1.15 n, D, K=16, normalize_output=True)
  fitted to L2-normalised target embeddings with MSE + Adagrad(lr 0.5)
  (:122-156);
* ``train_mask_model``: KShiftEmbedding(1.15 n, 4, K=16) -> MLP(4 -> 64 -> 1)
  separating catalogue ids from uniform random int64 ids, BCE-with-logits +
  Adagrad (:70-118);
* ``ModelWrapper``: emb(x) * sigmoid(mask(x)) (:32-41), the artifact the LTHM
  encoder consumes (encoder.py:25-29).

The tables train through the touched-row path (``sparse=True``): the KShift
backward records the batch's lookups and ``SparseRowAdagrad(fused=True)`` forms
each touched row's gradient and updates the row in one call (no gradient row
stored; ``LTHM_EMBGEN_FUSED=0``: the backward stages the row gradients and the
row-wise Adagrad updates the touched rows).  For Adagrad (lr_decay = 0, no weight decay) this is exactly the
reference's dense update: a row with zero gradient keeps its value and its
state sum.  The MLP uses ``FusedAdagrad``.  Batches are shuffled with a seeded
numpy Generator (the reference uses the global ``np.random``).
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import numpy as np
import torch
import torch.nn as nn

from . import ingest
from . import kernels as K
from .commons.layers import MLP, KShiftEmbedding
from .optim import FusedAdagrad, SparseRowAdagrad

MAX_LONG_VALUE_PLUS_ONE = 2 ** 63
# the tables step with the fused dedup + Adagrad (lthm_kshift_adagrad_fused): nothing reads or
# clips their gradients between loss.backward() and optim.step() (:137,151-153 / :97-99,113-115).
# LTHM_EMBGEN_FUSED=0: the two-pass path (row gradient staged by the backward, then the
# row-wise Adagrad over the touched rows) for A/B runs
_FUSED = os.environ.get("LTHM_EMBGEN_FUSED", "1") != "0"


class ModelWrapper(nn.Module):
    """embedding_module_gen.py:32-41."""

    def __init__(self, model: nn.Module, mask_model: nn.Module):
        super().__init__()
        self.model = model
        self.mask_model = mask_model

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        emb = self.model(x)
        mask = self.mask_model(x).sigmoid()
        return mask * emb


def massage_embeddings(df):
    """embedding_module_gen.py:53-66: product ids -> xxh64 int64 ids (seed xxh32('product_id'))."""
    seed = ingest.hash_feature_name_to_int("product_id")
    df["product_id"] = ingest.hash_values(df["product_id"].values, seed, False)
    return df


def _batches(n: int, batch_size: int, rng: np.random.Generator):
    idx = np.arange(n)
    rng.shuffle(idx)
    for b in range(0, n, batch_size):
        yield idx[b:b + batch_size]


class _LossLog:
    """Per-batch losses stay on the device and reach ``log`` in groups (one host sync per
    flush instead of one per batch as the reference's ``loss.item()`` print):
    ``log_every`` batches per flush, 0 = once per epoch."""

    def __init__(self, log: Optional[Callable], tag: str, num_epochs: int, log_every: int):
        self.log, self.tag, self.num_epochs, self.every = log, tag, num_epochs, log_every
        self.pending = []

    def add(self, epoch: int, b: int, loss: torch.Tensor) -> None:
        if self.log is None:
            return
        self.pending.append((epoch, b, loss.detach().reshape(1)))
        if self.every > 0 and len(self.pending) >= self.every:
            self.flush()

    def flush(self) -> None:
        if not self.pending:
            return
        vals = torch.cat([p[2] for p in self.pending]).tolist()
        for (epoch, b, _), v in zip(self.pending, vals):
            self.log(self.tag, epoch, self.num_epochs, b, v)
        self.pending = []


def train_model(df, expansion_factor: float, k_shift: int, *, num_epochs: int = 500, batch_size: int = 2 ** 18,
                device: Optional[torch.device] = None, seed: int = 0, lr: float = 5e-1,
                log: Optional[Callable] = print, log_every: int = 0) -> KShiftEmbedding:
    """embedding_module_gen.py:122-156 (reconstruction model); nn.MSELoss on lthm_mse_*."""
    device = device or torch.device("cuda")
    hashed_idx = torch.from_numpy(np.asarray(df["product_id"].values, dtype=np.int64)).to(device)
    x = torch.from_numpy(np.stack(df["embedding"].values).astype(np.float32)).to(device)
    x = K.l2norm_rows(x.contiguous())  # F.normalize(x, p=2.0, dim=-1)
    model = KShiftEmbedding(int(expansion_factor * x.size(0)), x.size(1), num_shifts=k_shift,
                            normalize_output=True, sparse=True).to(device)
    optim = SparseRowAdagrad([model], lr=lr, fused=_FUSED)
    rng = np.random.default_rng(seed)
    losses = _LossLog(log, "Model", num_epochs, log_every)
    for epoch in range(num_epochs):
        for b, idx in enumerate(_batches(x.size(0), batch_size, rng)):
            it = torch.from_numpy(idx).to(device)
            y = model(hashed_idx[it])
            loss = K.mse_loss(y, x[it])
            loss.backward()
            optim.step()
            losses.add(epoch, b, loss)
        losses.flush()
    return model


def train_mask_model(df, expansion_factor: float, k_shift: int, mask_emb_dim: int, *, num_epochs: int = 100,
                     batch_size: int = 2 ** 17, device: Optional[torch.device] = None, seed: int = 0,
                     lr: float = 5e-1, log: Optional[Callable] = print,
                     negatives: Optional[Callable[[int], torch.Tensor]] = None, log_every: int = 0) -> nn.Module:
    """embedding_module_gen.py:70-118 (catalogue-membership mask model).
    ``negatives(k)`` (default: uniform int64 on the device) supplies the k random
    non-catalogue ids of a batch."""
    device = device or torch.device("cuda")
    product_id = torch.from_numpy(np.asarray(df["product_id"].values, dtype=np.int64)).to(device)
    n = product_id.size(0)
    emb = KShiftEmbedding(int(expansion_factor * n), mask_emb_dim, num_shifts=k_shift, normalize_output=False,
                          sparse=True)
    model = nn.Sequential(emb, MLP(mask_emb_dim, 1, [mask_emb_dim * 16])).to(device)
    opt_tab = SparseRowAdagrad([emb], lr=lr, fused=_FUSED)
    opt_mlp = FusedAdagrad(model[1].parameters(), lr=lr)
    rng = np.random.default_rng(seed)
    g = torch.Generator(device=device).manual_seed(seed)
    losses = _LossLog(log, "MASK", num_epochs, log_every)
    for epoch in range(num_epochs):
        for b, idx in enumerate(_batches(n, batch_size, rng)):
            pos = product_id[torch.from_numpy(idx).to(device)]
            if negatives is not None:
                neg = negatives(pos.size(0)).to(device)
            else:
                neg = torch.randint(-MAX_LONG_VALUE_PLUS_ONE, MAX_LONG_VALUE_PLUS_ONE - 1, (pos.size(0),),
                                    dtype=torch.int64, device=device, generator=g)
            ids = torch.cat([pos, neg])
            target = torch.cat([torch.ones(pos.size(0), device=device), torch.zeros(neg.size(0), device=device)])
            pred = model(ids).squeeze(1)
            loss = K.bce_with_logits(pred.float().contiguous(), target)
            loss.backward()
            opt_tab.step()
            opt_mlp.step()
            opt_mlp.zero_grad(set_to_none=True)
            losses.add(epoch, b, loss)
        losses.flush()
    return model
