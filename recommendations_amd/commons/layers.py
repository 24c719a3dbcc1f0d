"""Embedding and feature-interaction primitives — drop-in for commons/layers.py.

Class names, constructor signatures and parameter names follow the reference
(``KShiftEmbedding.emb.weight``, ``FlatEmbedding._emb_table.weight``,
``MLP.model.{i}.weight`` ...) so state_dicts interchange.  Forward/backward run
in the gfx950 kernels of ``recommendations_amd/csrc`` through ``kernels``.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.nn as nn

from .. import kernels as K


class KShiftEmbedding(nn.Module):
    """commons/layers.py:125-185.

    ``num_embeddings`` rows (P) of ``emb_dim`` (D); each id reads K rows at
    ``get_row_idx(id, c)`` (the reference's arithmetic-shift "rotation",
    reproduced bit-exactly), sums them in order in fp32, then scales by
    1/sqrt(K) or L2-normalises.  Extra keyword ``out_dtype`` (default: the
    table dtype) lets a bf16 table feed bf16 activations.
    """

    def __init__(self, num_embeddings: int, emb_dim: int, num_shifts: int = 8,
                 normalize_output: bool = False, sparse: bool = False, *, out_dtype=None):
        super().__init__()
        self.emb = nn.Embedding(num_embeddings, emb_dim, sparse=sparse)
        self._num_embeddings = num_embeddings
        self._num_shifts = num_shifts
        self._num_bits = 64
        self._normalize_output = normalize_output
        self._out_dtype = out_dtype
        if num_shifts > 64:
            raise ValueError("num_shifts must be <= 64 (64-bit ids)")

    def forward(self, id_: torch.Tensor) -> torch.Tensor:
        mode = K.KSHIFT_NORMALIZE if self._normalize_output else K.KSHIFT_SCALE
        return K.kshift(id_, self.emb.weight, self._num_embeddings, self._num_shifts, mode,
                        out_dtype=self._out_dtype)

    def get_row_idx(self, x: torch.Tensor, col_idx: int) -> torch.Tensor:
        return K.kshift_rows(x.contiguous(), self._num_embeddings, col_idx + 1)[..., col_idx]


class FlatEmbedding(nn.Module):
    """commons/layers.py:44-61: ``W[x mod P]``, optional L2 normalisation."""

    def __init__(self, num_embeddings: int, emb_dim: int, padding_idx: int = None,
                 zero_init: bool = False, normalize_output: bool = False):
        super().__init__()
        self._num_embeddings = num_embeddings
        self._emb_dim = emb_dim
        self.padding_idx = padding_idx
        self._emb_table = nn.Embedding(num_embeddings, emb_dim, padding_idx=padding_idx)
        self._normalize_output = normalize_output
        if zero_init:
            self._emb_table.weight.data.fill_(0.0)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        mode = K.KSHIFT_NORMALIZE if self._normalize_output else K.KSHIFT_NONE
        w = self._emb_table.weight
        if self.padding_idx is not None and w.requires_grad:
            w = _ZeroRowGrad.apply(w, self.padding_idx)
        return K.kshift(x, w, self._num_embeddings, 1, mode)


class _ZeroRowGrad(torch.autograd.Function):
    """nn.Embedding(padding_idx) semantics: the padding row receives no gradient."""

    @staticmethod
    def forward(ctx, w, row):
        ctx.row = row
        return w.view_as(w)

    @staticmethod
    def backward(ctx, g):
        g = g.clone()
        g[ctx.row].zero_()
        return g, None
