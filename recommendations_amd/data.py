"""Synthetic (user-sequence, categorical-id) batches for LTHM.

Shapes and id semantics follow the reference data path
(commons/feature_utils.py:40-46 ids = xxh64 - 2^63 over the full int64 range,
:21-25 right padding with 0 to history_length; labels 0..3; epoch-second
timestamps).  Every rank draws from its own generator (seed + rank).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

INT64_MIN, INT64_MAX = -(2 ** 63), 2 ** 63 - 1
TS_2023 = 1672531200  # 2023-01-01T00:00:00Z


def synthetic_lthm_batch(B: int, T: int, n_cat: int = 0, seed: int = 1234, rank: int = 0,
                         device: Optional[torch.device] = None, zipf_vocab: Optional[int] = None,
                         min_len: int = 1) -> Dict[str, torch.Tensor]:
    g = torch.Generator().manual_seed(seed + rank)
    if zipf_vocab:
        # Zipf(1.05) over a catalogue, hashed into the int64 id space
        ranks = torch.arange(1, zipf_vocab + 1, dtype=torch.float64)
        probs = ranks.pow(-1.05)
        probs /= probs.sum()
        idx = torch.multinomial(probs, B * T, replacement=True, generator=g)
        ids = (idx * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & 0x7FFFFFFFFFFFFFFF
        ids = ids.view(B, T)
        ids = torch.where(idx.view(B, T) % 2 == 0, ids, ids - INT64_MAX - 1)
    else:
        ids = torch.randint(INT64_MIN, INT64_MAX, (B, T), generator=g, dtype=torch.int64)
    ids[ids == 0] = 1
    lengths = torch.randint(min_len, T + 1, (B,), generator=g)
    lengths[0] = T  # at least one full history, so the batch trim is 0 like production batches
    pos = torch.arange(T).unsqueeze(0)
    valid = pos < lengths.unsqueeze(1)
    ids = torch.where(valid, ids, torch.zeros_like(ids))
    labels = torch.randint(0, 4, (B, T), generator=g, dtype=torch.int64)
    ts = TS_2023 + torch.randint(0, 365 * 86400, (B, T), generator=g, dtype=torch.int64)
    batch = {"product_ids": ids, "labels": labels, "timestamp": ts}
    if n_cat > 0:
        batch["categorical_ids"] = torch.randint(INT64_MIN, INT64_MAX, (B, n_cat), generator=g, dtype=torch.int64)
    if device is not None:
        batch = {k: v.to(device, non_blocking=True) for k, v in batch.items()}
    return batch


def synthetic_ranker_batch(B: int, n_dense: int = 128, n_cat: int = 64, seed: int = 1234, rank: int = 0,
                           device: Optional[torch.device] = None, ctr: float = 0.1) -> Dict[str, torch.Tensor]:
    """dense [B, n_dense] ~ N(0, 1) f32, categorical [B, n_cat] uniform
    int64 ids, click label ~ Bernoulli(ctr) as float."""
    g = torch.Generator().manual_seed(seed + rank)
    batch = {"dense": torch.randn(B, n_dense, generator=g),
             "categorical": torch.randint(INT64_MIN, INT64_MAX, (B, n_cat), generator=g, dtype=torch.int64),
             "label": (torch.rand(B, generator=g) < ctr).float()}
    if device is not None:
        batch = {k: v.to(device, non_blocking=True) for k, v in batch.items()}
    return batch
