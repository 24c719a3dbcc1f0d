"""Ranker model and wrapper (build-defined composition, see config.py).

forward: dense [B, n_dense] f32 -> DenseMapper.forward_matrix (one quantile-map
kernel + one fused CVE kernel) -> [B, emb_dim];  categorical [B, F] int64 ->
table-batched FlatEmbedding lookups (a KShift gather with K = 1: row = x mod P,
exactly FlatEmbedding's ``W[x % P]``; sparse touched-row gradients) -> [B, F*D];
concat -> MLP with QuickGELU gates (one fused MFMA GEMM chain) -> logits [B, 1].
train_step: BCE-with-logits on ``batch["label"]`` (lthm_bce_logits_* kernels).
Optimizers: FusedAdamW on the dense parameters, SparseRowAdamW on the tables.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.nn as nn

from ... import kernels as K
from ...commons.base_model_wrapper import BaseModelWrapper
import os

from ...commons.layers import MLP, TableBatchedKShiftEmbedding
from ...commons.transformers.layers import DenseMapper
from ...optim import FusedAdamW, SparseRowAdamW


# LTHM_RANKER_INPUT_ROW=0: the MLP input by concatenation (round 5's path; A/B)
_INPUT_ROW = os.environ.get("LTHM_RANKER_INPUT_ROW", "1") != "0"


class RankerModel(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        stats = {f"dense_{i}": list(cfg.dense_quantiles) for i in range(cfg.n_dense)}
        self.dense_mapper = DenseMapper(stats, cfg.emb_dim, list(cfg.dense_n_projs), list(cfg.dense_num_bins))
        self.cat_tables = TableBatchedKShiftEmbedding(
            cfg.n_categorical, cfg.cat_vocab, cfg.cat_emb_dim, num_shifts=1, normalize_output=False, sparse=True,
            gather_dtype=torch.bfloat16 if cfg.cat_gather_bf16 else torch.float32, out_dtype=torch.bfloat16)
        self.interaction = MLP(cfg.interaction_in, cfg.out_dim, list(cfg.gate_sizes))

    def forward(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        dense, cat = batch["dense"], batch["categorical"]
        B = dense.shape[0]
        e_dense = self.dense_mapper.forward_matrix(dense)              # [B, emb_dim] f32
        if _INPUT_ROW and self.cat_tables.into_row_ok():
            # the MLP input [e_dense | table rows] built in one bf16 buffer, the table rows gathered
            # into their columns (MLP.forward_rows): the same values as the concatenation below
            return {"logits": self.interaction.forward_rows(e_dense, cat.contiguous(), self.cat_tables)}
        e_cat = self.cat_tables(cat.contiguous())                      # [B, F, D] bf16
        # the MLP input [e_dense | e_cat] ([B, emb_dim + F*D]) is assembled in bf16 inside the MLP
        # op: the same values the first GEMM reads from an f32 concatenation, without it
        return {"logits": self.interaction.forward_concat(e_dense, e_cat.reshape(B, -1))}


class RankerModelWrapper(BaseModelWrapper):
    """BaseModelWrapper surface (commons/base_model_wrapper.py:9-72) for the ranker."""

    def __init__(self, model_config):
        super().__init__()
        self.model_config = model_config
        self._model = RankerModel(model_config)

    def forward(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        return self._model(batch)

    def _loss(self, batch, output):
        z = output["logits"].reshape(-1)
        y = batch["label"].reshape(-1).float().contiguous()
        return K.bce_with_logits(z, y)

    def train_step(self, batch, output):
        return self._loss(batch, output), {}

    def val_step(self, batch, output):
        return self._loss(batch, output), {}

    def is_sparse(self, param_name: str):
        return super().is_sparse(param_name) or "cat_tables" in param_name

    def optim_group(self, parent_module: nn.Module, full_param_name: str, numel: int) -> Optional[str]:
        return "SPARSE_ROWS" if "cat_tables" in full_param_name else "USE_OPTIM"

    def param_groups(self) -> Dict[str, List[torch.nn.Parameter]]:
        groups: Dict[str, List[torch.nn.Parameter]] = {}
        for name, p in self.named_parameters():
            groups.setdefault(self.optim_group(self, name, p.numel()), []).append(p)
        return groups

    def optimizers_for_param_groups(self, param_groups):
        cfg = self.model_config
        out = []
        dense = [p for p in param_groups.get("USE_OPTIM", []) if p.requires_grad]
        if dense:
            out.append(FusedAdamW(dense, lr=cfg.lr, weight_decay=cfg.weight_decay, betas=cfg.betas))
        if param_groups.get("SPARSE_ROWS"):
            out.append(SparseRowAdamW([self._model.cat_tables], lr=cfg.lr, betas=cfg.betas,
                                      weight_decay=cfg.weight_decay))
        return out
