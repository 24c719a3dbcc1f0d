"""Ranker ("factorized DLRM") config — BASELINE.json configs[3], SURVEY §8d C4.

The reference's ranker is a stub: models/ranker/config.py:16-61 declares
``RankerModelConfig`` (kind RANKER, type "factorized_dlrm", query / item / user
feature lists) and hydra-configs/ranker_config.yaml sets ``emb_dim: 64``, while
models/ranker/builder.py, fdlrm/wrapper.py and fdlrm/towers/ are empty files and
fdlrm/factorized_dlrm.py holds only imports.  The composition built
here is therefore build-defined from the reference's own primitives, as SURVEY
§8d C4 specifies: 128 dense features -> DenseMapper (n_projs [16], num_bins
[20]; commons/transformers/layers.py:490-511) and 64 categorical features ->
FlatEmbedding 1M x 32 (commons/layers.py:44-61), concatenated -> MLP(-> [1024,
512] -> 1) with QuickGELU gates (commons/layers.py:65-81) -> BCE-with-logits on
the click label.
"""
from __future__ import annotations

from statistics import NormalDist
from typing import List, Tuple

from pydantic import BaseModel, Field


def normal_quantiles(n: int = 20) -> List[float]:
    """n evenly spaced N(0, 1) quantiles (dense features ~ N(0, 1))."""
    nd = NormalDist()
    return [nd.inv_cdf((i + 1) / (n + 1)) for i in range(n)]


class RankerModelConfig(BaseModel):
    kind: str = "ranker_ctr_cvr"        # ranker_config.yaml
    type: str = "factorized_dlrm"
    name: str = "ranker_model"
    emb_dim: int = 64                   # dense-feature embedding width (ranker_config.yaml)
    n_dense: int = 128
    dense_quantiles: List[float] = Field(default_factory=lambda: normal_quantiles(20))
    dense_n_projs: List[int] = [16]
    dense_num_bins: List[int] = [20]
    n_categorical: int = 64
    cat_vocab: int = 1_000_000
    cat_emb_dim: int = 32
    # K = 1 tables gather from the fp32 master: the same bf16 outputs as a bf16 shadow (bf16(W[row])
    # either way), and the row-wise step writes no shadow rows: C4 3.65 -> 3.48 ms per step,
    # sparse AdamW 0.79 -> 0.65 ms, gather unchanged (random rows, not bytes, bound it;
    # profiles/r06e/c4_g*.log)
    cat_gather_bf16: bool = False
    gate_sizes: List[int] = [1024, 512]
    out_dim: int = 1
    lr: float = 1e-3
    weight_decay: float = 0.0
    betas: Tuple[float, float] = (0.9, 0.999)
    seed: int = 1234

    @property
    def interaction_in(self) -> int:
        return self.emb_dim + self.n_categorical * self.cat_emb_dim

    def get_builder(self, stats=None):
        from .builder import RankerModelBuilder
        return RankerModelBuilder(self, stats)


def ranker_config(n_dense: int = 128, n_cat: int = 64, cat_vocab: int = 1_000_000, gate_sizes=(1024, 512),
                  **kw) -> RankerModelConfig:
    """Convenience constructor for BASELINE configs[3] (C4) and its reduced test shapes."""
    return RankerModelConfig(n_dense=n_dense, n_categorical=n_cat, cat_vocab=cat_vocab, gate_sizes=list(gate_sizes),
                             **kw)
