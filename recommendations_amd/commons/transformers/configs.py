"""Pydantic config schema of the sequence encoder — same fields as the reference's
commons/transformers/configs.py:6-44 (so the reference YAML maps 1:1)."""
from enum import Enum
from typing import Optional, Tuple, Union

from pydantic import BaseModel


class MLPConfig(BaseModel):
    ff_mult: float


class MoEConfig(BaseModel):
    num_experts: int
    proj_features: int
    ff_mult_factor: float
    gate_sizes: Optional[Tuple[int, ...]] = None
    top_k: Optional[int] = None


class SelfAttentionType(Enum):
    MULTI_HEAD: str = "multi_head"
    MULTI_QUERY: str = "multi_query"


class PositionBiasConfig(BaseModel):
    context_window: int


class SelfAttentionConfig(BaseModel):
    attn_dropout: float = 0.1
    bias: bool = True
    dropout: float = 0.1
    n_head: int = 12
    n_embd: int = 768
    pos_bias: Optional[PositionBiasConfig] = None
    attn_type: SelfAttentionType


class TransformerConfig(BaseModel):
    rotator_config: Union[MoEConfig, MLPConfig]
    is_causal: bool = False
    max_block_size: Optional[int] = None
    is_sparse_attn: bool = False
    sparsity_factor: float = 0.5
    enable_gradient_checkpointing: bool = False
    attn_config: SelfAttentionConfig
    # build-defined (BASELINE configs[4], C5): forward encoder GEMMs on the fp8 MFMA
    fp8_gemm: bool = False
