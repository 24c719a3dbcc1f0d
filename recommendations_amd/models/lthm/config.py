"""LTHM model config — the fields the reference's LTHM code actually reads.

The reference's own pydantic schema (models/lthm/config.py:17-79) does not
declare most of the fields its towers read, so
its YAML fails validation.  This schema declares every field the towers and
wrapper use, with the reference YAML's values as defaults
(hydra-configs/model/lthm.yaml), so `model/lthm.yaml` maps 1:1.  Fields marked
"build-defined" are additions of this build (documented in DESIGN.md).
"""
from __future__ import annotations

from typing import Any, List, Optional, Tuple

from pydantic import BaseModel, Field

from ...commons.transformers.configs import SelfAttentionConfig, TransformerConfig


class CosineLSHConfig(BaseModel):
    num_bins: int
    num_proj: int


class LatentModelConfig(BaseModel):
    vocab_size_latent: int = 1_000_000
    num_shifts_latent: int = 16
    normalize_embedding: bool = True


class ProductTowerConfig(BaseModel):
    inp_emb_dim: int = 32
    out_emb_dim: int = 512
    item_emb_dim: int = 128
    product_emb_dim: int = 128
    seq_emb_dim: Optional[int] = None
    cosine_lsh_config: List[CosineLSHConfig] = Field(default_factory=lambda: [
        CosineLSHConfig(num_bins=b, num_proj=32) for b in (2, 4, 8, 12, 16, 20)])
    detach_item_tower: bool = True
    norm_threshold: float = 0.05
    norm_bins: int = 20
    model_init_metadata: Optional[Any] = None
    latent_model_config: LatentModelConfig = Field(default_factory=LatentModelConfig)


class LogQConfig(BaseModel):
    num_buckets: int = 2 ** 24
    hash_offsets: List[int] = [0, 34144, 7465477, 64363466, 4234551, 245435435, 143244556]
    alpha: float = 0.05
    p_init: float = 0.001
    beta: float = 0.0


class CategoricalContextConfig(BaseModel):
    """Build-defined: per-sample categorical features (BASELINE configs C2/C3:
    32 / 64 features x 1M vocab) through table-batched KShift tables, concatenated,
    cap_gradients, then commons.layers.MLP (QuickGELU) to d_model, added to the
    CLS position of the sequence."""
    n_features: int = 0
    vocab_size: int = 1_000_000
    emb_dim: int = 32
    num_shifts: int = 8
    gate_sizes: List[int] = [512]
    gather_bf16: bool = True


class EncoderTransformerConfig(TransformerConfig):
    num_layers: int = 16
    dropout: float = 0.0


class LTHMModelConfig(BaseModel):
    kind: str = "lthm"
    type: str = "transformer_encoder"
    name: str = "torch_lthm_model"
    version: str = "v1"
    sparse: bool = False
    log_q_config: LogQConfig = Field(default_factory=LogQConfig)
    context_width: int = 512
    num_layers: int = 16
    product_tower: ProductTowerConfig = Field(default_factory=ProductTowerConfig)
    transformer_config: EncoderTransformerConfig
    loss_type: str = "contrastive"
    softmax_temperature: float = 0.05
    lookahead: List[int] = [0, 5, 6, 12, 24, 30]
    lr: float = 1e-4
    weight_decay: float = 1e-3
    betas: Tuple[float, float] = (0.9, 0.95)
    train_mini_batch_size: int = 32
    min_history_size: int = 0
    use_only_updated_data: bool = False
    metrics_k_all: List[int] = [1, 5, 20, 50]
    categorical: CategoricalContextConfig = Field(default_factory=CategoricalContextConfig)
    item_table_bf16: bool = True
    # build-defined: row-shard the frozen item KShift table over
    # the data-parallel ranks (r on rank r % world) instead of replicating it
    item_table_sharded: bool = False
    seed: int = 1234

    @property
    def emb_dim(self) -> int:
        return self.transformer_config.attn_config.n_embd

    @property
    def export_tokens(self) -> int:
        return len(self.lookahead)

    @property
    def export_span(self) -> int:
        return max(self.lookahead) + 1

    def get_builder(self, stats=None):
        from .builder import LTHMModelBuilder
        return LTHMModelBuilder(stats, self)


def lthm_config(T: int, d: int, n_layers: int, n_head: int, cat_features: int = 0, cat_vocab: int = 1_000_000,
                item_vocab: int = 1_000_000, out_emb_dim: Optional[int] = None, fp8: bool = False,
                gradient_checkpointing: bool = True, **kw) -> LTHMModelConfig:
    """Convenience constructor for the BASELINE configurations (C1-C5; fp8 = C5's
    fp8 encoder GEMMs). gradient_checkpointing follows the reference yaml
    (hydra-configs/model/lthm.yaml:53, on): activations recomputed in the backward."""
    tc = EncoderTransformerConfig(
        rotator_config={"ff_mult": 4}, is_causal=True, num_layers=n_layers, dropout=0.0,
        enable_gradient_checkpointing=gradient_checkpointing, fp8_gemm=fp8,
        attn_config=SelfAttentionConfig(attn_dropout=0.0, bias=False, dropout=0.0, n_head=n_head, n_embd=d,
                                        attn_type="multi_query", pos_bias={"context_window": T + 1}))
    pt = ProductTowerConfig(out_emb_dim=out_emb_dim or d,
                            latent_model_config=LatentModelConfig(vocab_size_latent=item_vocab))
    cat = CategoricalContextConfig(n_features=cat_features, vocab_size=cat_vocab)
    lq = LogQConfig(beta=kw.pop("log_q_beta", 0.0), num_buckets=kw.pop("log_q_buckets", 2 ** 24))
    return LTHMModelConfig(context_width=T, num_layers=n_layers, transformer_config=tc, product_tower=pt,
                           categorical=cat, log_q_config=lq, **kw)
