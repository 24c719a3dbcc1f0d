"""Sequence-encoder layers — drop-in for commons/transformers/layers.py.

Module names and parameter names match the reference (``ln_1.weight``,
``attn.c_attn.weight``, ``attn.attn.pos_bias.bias``, ``mlp.c_fc.weight`` ...), so
state_dicts interchange.  The TransformerBlock hot path is one fused autograd op
(``TransformerBlockFn``) whose forward and backward are a fixed sequence of
gfx950 kernels: LayerNorm, MFMA GEMMs with fused bias/GELU/residual epilogues,
and the LDS-resident attention with the in-kernel relative-position bias.

Reference behaviour reproduced "as executed" (SURVEY.md §3.5 #15): the FFN
hidden size is 4*d whatever ``rotator_config.ff_mult`` says, and
``SelfAttention.from_config`` always builds multi-head attention.  Activations
are bf16 (GEMM operands), the residual stream and all accumulations fp32.
"""
from __future__ import annotations

import math
import os
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.utils.checkpoint
import torch.nn as nn

from ... import kernels as K
from ..._lib import require_gpu


def _bf(w):
    """bf16 GEMM operand of a weight: the copy cast at the start of this forward by the
    enclosing K.bf16_operands scope, else a fresh cast."""
    if w is None:
        return None
    return K.bf16_operand(w)


def _f(b):
    return None if b is None else b.detach().contiguous()


def dropout(x: torch.Tensor, p: float, training: bool) -> torch.Tensor:
    """nn.Dropout(p)(x): identity in eval mode or at p = 0, else the HIP hash-mask kernel."""
    if not training or p == 0.0:
        return x
    return K.DropoutFn.apply(x, float(p), K.new_dropout_seed())


# bf16 copy of the input gradient a block's backward produces (its final LayerNorm
# backward writes it for free), handed to the backward of the block below, which
# would otherwise cast the same f32 gradient again.  One slot; it holds the f32
# tensor itself, so a match on (data_ptr, shape, version) is that very tensor.
_GRAD_BF16: Dict[str, Any] = {}


def _stash_grad_bf16(g32: torch.Tensor, gbf: torch.Tensor) -> None:
    _GRAD_BF16["src"], _GRAD_BF16["bf"], _GRAD_BF16["ver"] = g32, gbf, g32._version


def _grad_bf16(g32: torch.Tensor) -> torch.Tensor:
    src = _GRAD_BF16.pop("src", None)
    bf = _GRAD_BF16.pop("bf", None)
    ver = _GRAD_BF16.pop("ver", None)
    if (src is not None and src.data_ptr() == g32.data_ptr() and src.numel() == g32.numel()
            and src.dtype == g32.dtype and ver == src._version and g32.is_contiguous()):
        return bf.view(g32.shape)
    return K.cast(g32, torch.bfloat16)


# training through the fused MLP (forward hidden on chip, backward recomputes it); LTHM_MLP_TRAIN=0
# restores the stored-hidden chain (c_fc GEMM with the GELU' aux, c_proj GEMM, two dgrad GEMMs)
_MLP_TRAIN = os.environ.get("LTHM_MLP_TRAIN", "1") == "1"
# ln_2 inside the fused MLP kernel (LTHM_MLP_LN=1); default: the LayerNorm kernel, then the MLP
# kernel (C2: 81,718 vs 81,523 samples/s, mlp_fwd 0.90 + ln 0.17 vs 1.10 ms, profiles/r04d_*)
_MLP_LN = os.environ.get("LTHM_MLP_LN", "0") == "1"
# ln_2's backward writes dx1 + dy as its f32 output for ln_1's backward (LTHM_LN_FOLD=0: separately)
_LN_FOLD = os.environ.get("LTHM_LN_FOLD", "1") == "1"
# LTHM_MLP_WG=1: the fused MLP's backward without [M, 4d] operands in HBM (round 5:
# lthm_mlp_bwd_dx + lthm_mlp_wgrad, both recomputing the hidden; one wave per SIMD, issue-bound
# on the GELU' VALU: C2 step 40.8-41.0 ms against 39.9 for the default, profiles/r05e/).  Default:
# the recompute kernel writing G / dP for the dX GEMM and the two weight-gradient GEMMs (round 4)
_MLP_WG = os.environ.get("LTHM_MLP_WG", "0") == "1"


class TransformerBlockFn(torch.autograd.Function):
    """x -> x + attn(ln_1 x) -> + mlp(ln_2 .)  [+ x again when double_residual].

    ``drop`` = None (eval, or every dropout p = 0), or (p_attn, p_resid, seed) for
    training with the reference's dropouts (commons/transformers/layers.py:253-256
    token dropout of q / k / v, :264 residual dropout after c_proj, :283 MLP dropout,
    both at ``config.dropout``).  With dropout the two output GEMMs drop their fused
    residual epilogue and lthm_dropout adds the residual instead."""

    @staticmethod
    def forward(ctx, *args):
        with K.gemm_tag("enc"):
            return TransformerBlockFn._forward(ctx, *args)

    @staticmethod
    def backward(ctx, dout):
        with K.gemm_tag("enc"):
            return TransformerBlockFn._backward(ctx, dout)

    @staticmethod
    def _forward(ctx, x, ln1w, ln1b, wqkv, bqkv, wp, bp, table, ln2w, ln2b, w1, b1, w2, b2, H, causal,
                 double_residual, fp8=False, drop=None, mask=None, infer=False, pack=None):
        require_gpu(x)
        if pack is not None:
            # packed rows (shared pad prefix, recommendations_amd/pad_prefix.py): row-wise work on
            # the M packed rows, attention on the full-length sequences rebuilt from them
            M, d = x.shape
            B, T = pack.B, pack.Tp
        else:
            B, T, d = x.shape
            M = B * T
        E = d // H
        x2 = x.contiguous().view(M, d)
        wqkv_b, wp_b, w1_b, w2_b = _bf(wqkv), _bf(wp), _bf(w1), _bf(w2)
        # am: the activations' max |x| words for the fp8 mode, reduced by their producers
        # (layernorm_fwd, the c_fc epilogue; the attention output by one amax pass) so
        # that each quantisation reads its input once
        am = torch.zeros(4, dtype=torch.int32, device=x.device) if fp8 else None
        if fp8:
            # build-defined C5 mode: the four forward GEMMs take per-tensor-scaled e4m3
            # operands on the fp8 MFMA; the backward runs bf16 on the saved activations
            def lin(xb, wb, b, amax_in=None, **kw):
                xq, xs = K.quantize_fp8(xb, amax=amax_in)
                wq, ws = K.quantize_fp8(wb)
                return K.linear_fwd_fp8(xq, xs, wq, ws, b, **kw)
        else:
            def lin(xb, wb, b, amax_in=None, **kw):
                return K.linear_fwd(xb, wb, b, **kw)
        pa, pr, seed = drop if drop is not None else (0.0, 0.0, 0)
        h1, mu1, rs1 = K.layernorm_fwd(x2, ln1w.detach(), _f(ln1b), amax=am[0:1] if fp8 else None)
        qkv = lin(h1, wqkv_b, _f(bqkv), amax_in=am[0:1] if fp8 else None)
        if pa > 0.0:
            K.dropout_rows_(qkv, 3, pa, seed)  # the attention sees (and the backward saves) the scaled q / k / v
        tab = None if table is None else table.detach().contiguous()
        mop = K.attn_mask_operand(mask, B, H, T)
        if pack is not None and K.attn_packed_ok(T, E, mop):
            qkv_f, o_f = qkv, None  # the kernels read the packed rows through the pad-prefix maps
            o, lse = K.attn_fwd_qkv(qkv, B, T, H, E, tab, causal, mop, pack=pack)
        elif pack is not None:
            qkv_f = pack.unpack(qkv)
            o_f, lse = K.attn_fwd_qkv(qkv_f, B, T, H, E, tab, causal, mop)
            o = pack.pack(o_f)
        else:
            qkv_f, o_f = qkv, None
            o, lse = K.attn_fwd_qkv(qkv, B, T, H, E, tab, causal, mop)
        ctx.pack, ctx.o_full = pack, o_f
        if fp8:
            K.amax_(o, am[1:2])
        ln2_done = None  # (h2, mu2, rs2) when ln_2 ran inside the c_proj GEMM
        if pr > 0.0:
            x1 = K.dropout(lin(o, wp_b, _f(bp), out_dtype=torch.float32, amax_in=am[1:2] if fp8 else None), pr,
                           seed + 1, res1=x2)
        elif not fp8 and not _MLP_LN and K.linear_layernorm_fwd_ok(o, wp_b, _f(bp), x2, ln2w.detach(), _f(ln2b)):
            # c_proj + residual, then ln_2, in one kernel (its 256-row tiles hold whole rows)
            x1, h2f, mu2f, rs2f = K.linear_layernorm_fwd(o, wp_b, _f(bp), x2, ln2w.detach(), _f(ln2b))
            ln2_done = (h2f, mu2f, rs2f)
        else:
            x1 = lin(o, wp_b, _f(bp), res1=x2, out_dtype=torch.float32, amax_in=am[1:2] if fp8 else None)
        if not fp8 and pr == 0.0 and K.mlp_supported(d, w1.shape[0]) and (infer or _MLP_TRAIN):
            # ln_2 and the MLP in one kernel: the [M, 4d] hidden stays on chip; in training the
            # backward recomputes it (K.mlp_bwd), so neither the hidden nor GELU' is stored
            w2t_b = w2_b.t().contiguous()
            if _MLP_LN:
                out, h2, mu2, rs2 = K.mlp_fwd_ln(x1, ln2w.detach(), _f(ln2b), w1_b, _f(b1), w2t_b, _f(b2), res1=x1,
                                                 res2=x2 if double_residual else None, save=not infer)
            else:
                h2, mu2, rs2 = ln2_done or K.layernorm_fwd(x1, ln2w.detach(), _f(ln2b))
                out = K.mlp_fwd(h2, w1_b, _f(b1), w2t_b, _f(b2), res1=x1, res2=x2 if double_residual else None)
            if infer:
                return out if pack is not None else out.view(B, T, d)
            ctx.save_for_backward(x2, h1, mu1, rs1, qkv_f, o, lse, x1, h2, mu2, rs2, _f(b1), w2t_b,
                                  wqkv_b, wp_b, w1_b, w2_b, ln1w, ln2w, tab)
            ctx.cfg = (B, T, d, H, E, causal, double_residual, ln1b is not None, bqkv is not None, bp is not None,
                       b1 is not None, b2 is not None, None if table is None else table.shape, pa, pr, seed)
            ctx.mop = mop
            ctx.fused_mlp = True
            return out if pack is not None else out.view(B, T, d)
        h2, mu2, rs2 = ln2_done or K.layernorm_fwd(x1, ln2w.detach(), _f(ln2b), amax=am[2:3] if fp8 else None)
        # pre holds GELU'(c_fc x) (bf16): the backward epilogue is then one multiply
        pre = torch.empty((M, w1.shape[0]), dtype=torch.bfloat16, device=x.device)
        if fp8:
            g = lin(h2, w1_b, _f(b1), act=K.ACT_GELU_D, aux_out=pre, amax_in=am[2:3], amax_out=am[3:4])
        else:
            g = lin(h2, w1_b, _f(b1), act=K.ACT_GELU_D, aux_out=pre)
        gam = am[3:4] if fp8 else None
        if pr > 0.0:
            out = K.dropout(lin(g, w2_b, _f(b2), out_dtype=torch.float32, amax_in=gam), pr, seed + 2, res1=x1,
                            res2=x2 if double_residual else None)
        else:
            out = lin(g, w2_b, _f(b2), res1=x1, res2=x2 if double_residual else None, out_dtype=torch.float32,
                      amax_in=gam)
        ctx.save_for_backward(x2, h1, mu1, rs1, qkv_f, o, lse, x1, h2, mu2, rs2, pre, g,
                              wqkv_b, wp_b, w1_b, w2_b, ln1w, ln2w, tab)
        ctx.cfg = (B, T, d, H, E, causal, double_residual, ln1b is not None, bqkv is not None, bp is not None,
                   b1 is not None, b2 is not None, None if table is None else table.shape, pa, pr, seed)
        ctx.mop = mop
        ctx.fused_mlp = False
        return out if pack is not None else out.view(B, T, d)

    @staticmethod
    def _backward(ctx, dout):
        (x2, h1, mu1, rs1, qkv, o, lse, x1, h2, mu2, rs2, pre, g, wqkv_b, wp_b, w1_b, w2_b, ln1w, ln2w,
         tab) = ctx.saved_tensors
        B, T, d, H, E, causal, dbl, has_ln1b, has_bqkv, has_bp, has_b1, has_b2, tshape, pa, pr, seed = ctx.cfg
        pack = ctx.pack
        M = x2.shape[0]
        dy = dout.contiguous().view(M, d)
        if dy.dtype != torch.float32:
            dy = dy.float()
        # MLP half (dym: the gradient behind the MLP dropout)
        if pr > 0.0:
            dym = K.dropout(dy, pr, seed + 2)
            dyb = K.cast(dym, torch.bfloat16)
        else:
            dym, dyb = dy, _grad_bf16(dy)
        # dh2 = dpre W1 is produced inside ln_2's backward (K.dgrad_layernorm_bwd) where it takes
        # the shapes; dh2 None until then
        dh2 = None
        if ctx.fused_mlp:
            # saved: pre -> b1 (f32 or None), g -> c_proj.weight^T (bf16); the hidden is recomputed
            b1f, w2t_b = pre, g
            if _MLP_WG and K.mlp_wgrad_supported(d, w1_b.shape[0]):
                dh2 = K.mlp_bwd_dx(h2, dyb, w1_b, b1f, w2t_b)
                dw1, dw2, db1 = K.mlp_wgrad(h2, dyb, w1_b, b1f, w2t_b, want_db1=has_b1)
            else:
                dh2, g, dpre = K.mlp_bwd(h2, dyb, w1_b, b1f, w2t_b, want_dx=False)
                dw2 = K.linear_wgrad(dyb, g)
                dw1 = K.linear_wgrad(dpre, h2)
                db1 = K.colsum(dpre) if has_b1 else None
            db2 = K.colsum(dym) if has_b2 else None
        else:
            dw2 = K.linear_wgrad(dyb, g)
            db2 = K.colsum(dym) if has_b2 else None
            dpre = K.linear_dgrad(dyb, w2_b, act_grad=K.ACT_MUL_AUX, aux=pre)
            dw1 = K.linear_wgrad(dpre, h2)
            db1 = K.colsum(dpre) if has_b1 else None
        # double residual, no residual dropout, no c_proj bias: ln_1's backward needs dx1 + dy only
        # (dx = LN1'(dh1) + dx1 + dy), so ln_2's backward writes that sum as its f32 output (the
        # bf16 copy, the attention branch's input, stays dx1): one f32 read less per element
        fold = _LN_FOLD and dbl and pr == 0.0 and not has_bp and d % 4 == 0
        if dh2 is None and K.dgrad_layernorm_bwd_ok(dpre, w1_b, x1):
            dx1, dx1b, dln2w, dln2b = K.dgrad_layernorm_bwd(dpre, w1_b, x1, ln2w.detach(), mu2, rs2, res1=dy,
                                                            need_bias=has_ln1b, res1_twice=fold)
        else:
            if dh2 is None:
                dh2 = K.linear_dgrad(dpre, w1_b)
            dx1, dx1b, dln2w, dln2b = K.layernorm_bwd(dh2, x1, ln2w.detach(), mu2, rs2, res1=dy,
                                                      need_bias=has_ln1b, res1_twice=fold)
        # attention half (dx1r: the gradient behind the residual dropout)
        if pr > 0.0:
            dx1r = K.dropout(dx1, pr, seed + 1)
            dx1b = K.cast(dx1r, torch.bfloat16)
        else:
            dx1r = dx1
        dwp = K.linear_wgrad(dx1b, o)
        dbp = K.colsum(dx1r) if has_bp else None
        do = K.linear_dgrad(dx1b, wp_b)
        if pack is not None and ctx.o_full is None:
            dqkv, dtab = K.attn_bwd_qkv(qkv, o, do, lse, B, T, H, E, tab, causal, ctx.mop, pack=pack)
        elif pack is not None:
            # dO only at the rows the packed output read (the chain from its owner); K / V
            # gradients at pad rows summed over the sequences into the chain rows
            dqkv_f, dtab = K.attn_bwd_qkv(qkv, ctx.o_full, pack.unpack_owner(do), lse, B, T, H, E, tab, causal,
                                          ctx.mop)
            dqkv = pack.reduce(dqkv_f)
        else:
            dqkv, dtab = K.attn_bwd_qkv(qkv, o, do, lse, B, T, H, E, tab, causal, ctx.mop)
        if pa > 0.0:
            K.dropout_rows_(dqkv, 3, pa, seed)
        dwqkv = K.linear_wgrad(dqkv, h1)
        dbqkv = K.colsum(dqkv) if has_bqkv else None
        if K.dgrad_layernorm_bwd_ok(dqkv, wqkv_b, x2):
            dx, dxb, dln1w, dln1b = K.dgrad_layernorm_bwd(dqkv, wqkv_b, x2, ln1w.detach(), mu1, rs1, res1=dx1,
                                                          need_bias=has_ln1b, res2=dy if dbl and not fold else None)
        else:
            dh1 = K.linear_dgrad(dqkv, wqkv_b)
            dx, dxb, dln1w, dln1b = K.layernorm_bwd(dh1, x2, ln1w.detach(), mu1, rs1, res1=dx1,
                                                    need_bias=has_ln1b, res2=dy if dbl and not fold else None)
        _stash_grad_bf16(dx, dxb)
        dtable = None
        if tshape is not None:
            dtable = torch.zeros(tshape, dtype=torch.float32, device=dy.device)
            dtable[: dtab.shape[0]] = dtab
        return (dx if pack is not None else dx.view(B, T, d), dln1w, dln1b if has_ln1b else None, dwqkv, dbqkv, dwp,
                dbp, dtable, dln2w, dln2b if has_ln1b else None, dw1, db1, dw2, db2, None, None, None, None, None, None,
                None, None)


# ------------------------------------------------------------------ modules
class RelativePositionBias(nn.Module):
    """commons/transformers/layers.py:13-35 (table [nq + nk + 1, nh], row q - k + nk)."""

    def __init__(self, nq: int, nk: int, nh: int):
        super().__init__()
        self.nq, self.nk, self.nh = nq, nk, nh
        self.bias = nn.Parameter(torch.zeros((nq + nk + 1, nh)))

    def check(self, nq: int, nk: int):
        if not (nq <= self.nq):
            raise RuntimeError("nq > self.nq")
        if not (nk <= self.nk):
            raise RuntimeError("nk > self.nk")


class ScaledDotProductAttention(nn.Module):
    """commons/transformers/layers.py:41-61; the scores are never materialised."""

    def __init__(self, nq: int, nk: int, nh: int, relative_bias: bool = False):
        super().__init__()
        self.pos_bias = RelativePositionBias(nq, nk, nh) if relative_bias else nn.Identity()

    @property
    def table(self) -> Optional[torch.Tensor]:
        return self.pos_bias.bias if isinstance(self.pos_bias, RelativePositionBias) else None


class LayerNorm(nn.Module):
    """commons/transformers/layers.py:142-149."""

    def __init__(self, ndim: int, bias: bool = True):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(ndim))
        self.bias = nn.Parameter(torch.zeros(ndim)) if bias else None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return LayerNormFn.apply(x, self.weight, self.bias)


class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        require_gpu(x)
        shp = x.shape
        x2 = x.contiguous().view(-1, shp[-1]).float()
        y, mu, rs = K.layernorm_fwd(x2, w.detach(), _f(b), y_dtype=torch.float32)
        ctx.save_for_backward(x2, w, mu, rs)
        ctx.has_b, ctx.shp = b is not None, shp
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mu, rs = ctx.saved_tensors
        dx, _, dw, db = K.layernorm_bwd(dy.contiguous().view(x2.shape).float(), x2, w.detach(), mu, rs,
                                        want_bf16=False, need_bias=ctx.has_b)
        return dx.view(ctx.shp), dw, db


class SelfAttentionConfig:
    """Lightweight attribute config (commons/transformers/layers.py:165-174)."""

    def __init__(self, n_embd: int, n_head: int, attn_dropout: float, dropout: float, bias: bool, pos_bias=None):
        self.n_embd, self.n_head = n_embd, n_head
        self.attn_dropout, self.dropout, self.bias, self.pos_bias = attn_dropout, dropout, bias, pos_bias


class SelfAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        assert config.n_embd % config.n_head == 0
        self.config = config
        if config.pos_bias is None:
            self.attn = ScaledDotProductAttention(0, 0, 0, relative_bias=False)
        else:
            cw = config.pos_bias.context_window
            self.attn = ScaledDotProductAttention(nq=cw, nk=cw, nh=config.n_head, relative_bias=True)

    @classmethod
    def from_config(cls, config):
        # as executed by the reference (:195-199): always multi-head
        return MultiHeadAttention(config)


def _drop_args(mod: nn.Module, p_attn: float, p_resid: float):
    """(p_attn, p_resid, seed) for a fused op in training mode with some p > 0, else None."""
    if not mod.training or (p_attn == 0.0 and p_resid == 0.0):
        return None
    return (float(p_attn), float(p_resid), K.new_dropout_seed())


def _split_mask(mask: Optional[torch.Tensor], T: int):
    """(causal, extra) for an additive attention mask.  The reference's causal mask
    (commons/transformers/layers.py:397-402: -inf above the diagonal and one constant
    elsewhere, a softmax-invariant shift) runs as the kernels' causal flag; any other
    additive mask is added to the scores as given (SDPA :57-58) by the whole-head
    kernels (T <= 256)."""
    if mask is None:
        return False, None
    m = mask.reshape(-1, T, T)
    tri = torch.ones((T, T), dtype=torch.bool, device=mask.device).triu(1)
    kept = m[:, ~tri]
    if bool(torch.isneginf(m[:, tri]).all()) and bool((kept == kept.reshape(-1)[0]).all()):
        return True, None
    return False, mask


class _SelfAttnFn(torch.autograd.Function):
    """Standalone attention module forward/backward on the HIP kernels:
    MHA (commons/transformers/layers.py:247-265: c_attn -> SDPA -> c_proj) when
    ``shared_kv`` is False, MQA (:214-234: q_proj, kv_proj with one K/V head,
    out_proj) when True.  The MQA backward runs the multi-head kernel on K/V
    expanded per head and sums their gradients over the heads."""

    @staticmethod
    def forward(ctx, x, w_in, b_in, w_kv, b_kv, w_out, b_out, table, H, causal, shared_kv, drop=None, mask=None):
        require_gpu(x)
        pa, pr, seed = drop if drop is not None else (0.0, 0.0, 0)
        B, T, C = x.shape
        E = C // H
        M = B * T
        xb = K.cast(x.contiguous().view(M, C), torch.bfloat16)
        w_in_b, w_out_b = _bf(w_in), _bf(w_out)
        tab = None if table is None else table.detach().contiguous()
        mop = ctx.mop = K.attn_mask_operand(mask, B, H, T)
        if shared_kv:
            w_kv_b = _bf(w_kv)
            q = K.linear_fwd(xb, w_in_b, _f(b_in))
            kv = K.linear_fwd(xb, w_kv_b, _f(b_kv))
            if pa > 0.0:  # q (one group over the heads), then k and v of the shared head
                K.dropout_rows_(q, 1, pa, seed)
                K.dropout_rows_(kv, 2, pa, seed + 3)
            o, lse = K.attn_fwd_mqa(q, kv, B, T, H, E, tab, causal, mop)
            saved = (xb, q, kv, o, lse, w_in_b, w_kv_b, w_out_b)
        else:
            qkv = K.linear_fwd(xb, w_in_b, _f(b_in))
            if pa > 0.0:
                K.dropout_rows_(qkv, 3, pa, seed)
            o, lse = K.attn_fwd_qkv(qkv, B, T, H, E, tab, causal, mop)
            saved = (xb, qkv, o, lse, w_in_b, w_out_b)
        y = K.linear_fwd(o, w_out_b, _f(b_out), out_dtype=torch.float32)
        if pr > 0.0:
            y = K.dropout(y, pr, seed + 1)
        ctx.save_for_backward(*saved, tab)
        ctx.cfg = (B, T, C, H, E, causal, shared_kv, b_in is not None, b_kv is not None, b_out is not None,
                   None if table is None else table.shape)
        ctx.drop = (pa, pr, seed)
        return y.view(B, T, C)

    @staticmethod
    def backward(ctx, dy):
        B, T, C, H, E, causal, shared_kv, has_bin, has_bkv, has_bout, tshape = ctx.cfg
        pa, pr, seed = ctx.drop
        M = B * T
        saved = ctx.saved_tensors
        tab = saved[-1]
        dy = dy.contiguous().view(M, C).float()
        if pr > 0.0:
            dy = K.dropout(dy, pr, seed + 1)
        dyb = K.cast(dy, torch.bfloat16)
        if shared_kv:
            xb, q, kv, o, lse, w_in_b, w_kv_b, w_out_b = saved[:-1]
        else:
            xb, qkv, o, lse, w_in_b, w_out_b = saved[:-1]
        dw_out = K.linear_wgrad(dyb, o)
        db_out = K.colsum(dy) if has_bout else None
        do = K.linear_dgrad(dyb, w_out_b)
        dw_kv = db_kv = None
        if shared_kv:
            qkv_e = torch.cat([q, kv[:, :E].repeat(1, H), kv[:, E:].repeat(1, H)], dim=1).contiguous()
            dqkv, dtab = K.attn_bwd_qkv(qkv_e, o, do, lse, B, T, H, E, tab, causal, ctx.mop)
            dq = dqkv[:, :C].contiguous()
            dkv = torch.cat([dqkv[:, C:2 * C].float().view(M, H, E).sum(1),
                             dqkv[:, 2 * C:].float().view(M, H, E).sum(1)], dim=1).contiguous()
            if pa > 0.0:
                K.dropout_rows_(dq, 1, pa, seed)
                K.dropout_rows_(dkv, 2, pa, seed + 3)
            dkvb = K.cast(dkv, torch.bfloat16)
            dw_in = K.linear_wgrad(dq, xb)
            db_in = K.colsum(dq) if has_bin else None
            dw_kv = K.linear_wgrad(dkvb, xb)
            db_kv = K.colsum(dkv) if has_bkv else None
            dx = K.linear_dgrad(dq, w_in_b, out_dtype=torch.float32)
            dx = K.linear_dgrad(dkvb, w_kv_b, out_dtype=torch.float32, res1=dx)
        else:
            dqkv, dtab = K.attn_bwd_qkv(qkv, o, do, lse, B, T, H, E, tab, causal, ctx.mop)
            if pa > 0.0:
                K.dropout_rows_(dqkv, 3, pa, seed)
            dw_in = K.linear_wgrad(dqkv, xb)
            db_in = K.colsum(dqkv) if has_bin else None
            dx = K.linear_dgrad(dqkv, w_in_b, out_dtype=torch.float32)
        dtable = None
        if tshape is not None:
            dtable = torch.zeros(tshape, dtype=torch.float32, device=dy.device)
            dtable[: dtab.shape[0]] = dtab
        return dx.view(B, T, C), dw_in, db_in, dw_kv, db_kv, dw_out, db_out, dtable, None, None, None, None, None


class MultiHeadAttention(SelfAttention):
    """commons/transformers/layers.py:237-265."""

    def __init__(self, config):
        super().__init__(config)
        self.c_attn = nn.Linear(config.n_embd, 3 * config.n_embd, bias=config.bias)
        self.c_proj = nn.Linear(config.n_embd, config.n_embd, bias=config.bias)
        self.attn_dropout = nn.Dropout(config.attn_dropout)
        self.resid_dropout = nn.Dropout(config.dropout)
        self.n_head = config.n_head
        self.n_embd = config.n_embd

    def forward(self, x: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        T = x.shape[1]
        if self.attn.table is not None:
            self.attn.pos_bias.check(T, T)
        causal, extra = _split_mask(mask, T)
        return _SelfAttnFn.apply(x.float(), self.c_attn.weight, self.c_attn.bias, None, None, self.c_proj.weight,
                                 self.c_proj.bias, self.attn.table, self.n_head, causal, False,
                                 _drop_args(self, self.attn_dropout.p, self.resid_dropout.p), extra)


class MultiQueryAttention(SelfAttention):
    """commons/transformers/layers.py:202-234: query heads share one K/V head."""

    def __init__(self, config):
        super().__init__(config)
        self.q_proj = nn.Linear(config.n_embd, config.n_embd, bias=config.bias)
        self.kv_proj = nn.Linear(config.n_embd, 2 * (config.n_embd // config.n_head), bias=config.bias)
        self.out_proj = nn.Linear(config.n_embd, config.n_embd, bias=config.bias)
        self.attn_dropout = nn.Dropout(config.attn_dropout)
        self.resid_dropout = nn.Dropout(config.dropout)
        self.n_head = config.n_head
        self.n_embd = config.n_embd

    def forward(self, x: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        T = x.shape[1]
        if self.attn.table is not None:
            self.attn.pos_bias.check(T, T)
        causal, extra = _split_mask(mask, T)
        return _SelfAttnFn.apply(x.float(), self.q_proj.weight, self.q_proj.bias, self.kv_proj.weight,
                                 self.kv_proj.bias, self.out_proj.weight, self.out_proj.bias, self.attn.table,
                                 self.n_head, causal, True, _drop_args(self, self.attn_dropout.p, self.resid_dropout.p),
                                 extra)


class _MLP(nn.Module):
    """commons/transformers/layers.py:271-284."""

    def __init__(self, n_embd: int, bias: bool, dropout: float, hidden_mult: int):
        super().__init__()
        self.c_fc = nn.Linear(n_embd, int(hidden_mult * n_embd), bias=bias)
        self.gelu = nn.GELU(approximate="tanh")
        self.c_proj = nn.Linear(int(hidden_mult * n_embd), n_embd, bias=bias)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """:279-284 standalone (the block fuses this into TransformerBlockFn)."""
        y = K.mlp_chain(x, [self.c_fc, self.c_proj], [K.ACT_GELU, K.ACT_NONE], out_f32=True)
        return dropout(y, self.dropout.p, self.training)


class TransformerBlock(nn.Module):
    """commons/transformers/layers.py:323-420 (dense path)."""

    def __init__(self, config: Any, seed: Optional[int] = None, n_cls: int = 0):
        super().__init__()
        self.is_causal = config.is_causal
        attn_cfg = config.attn_config
        self.ln_1 = LayerNorm(attn_cfg.n_embd, bias=attn_cfg.bias)
        self.attn = SelfAttention.from_config(attn_cfg)
        self.ln_2 = LayerNorm(attn_cfg.n_embd, bias=attn_cfg.bias)
        rc = config.rotator_config
        if not isinstance(rc, dict) and hasattr(rc, "model_dump"):
            rc = rc.model_dump()
        self.is_moe = isinstance(rc, dict) and rc.get("moe") is not None
        if self.is_moe:
            # :340-343: MoE feed-forward (composed path: attention module + MoE MLP)
            self.mlp = _MoEMLP(attn_cfg.n_embd, attn_cfg.bias, attn_cfg.dropout, rc["moe"])
        else:
            hidden_mult = config.rotator_config if isinstance(config.rotator_config, (int, float)) else 4
            self.mlp = _MLP(attn_cfg.n_embd, attn_cfg.bias, attn_cfg.dropout, hidden_mult)
        self.is_sparse = getattr(config, "is_sparse_attn", False)
        self.enable_gradient_checkpointing = getattr(config, "enable_gradient_checkpointing", False)
        self.fp8_gemm = bool(getattr(config, "fp8_gemm", False))  # build-defined (C5)
        if self.is_sparse:
            # :352-368: a seeded permutation keeps n_cls + sparsity_factor * max_block_size
            # tokens for the block; the rest go through the null connector Linear
            max_block_size = config.max_block_size
            n_non_zeros = int(config.sparsity_factor * max_block_size)
            g = torch.Generator()
            if seed is not None:
                g.manual_seed(seed)
            perm = torch.randperm(max_block_size, generator=g)
            full_mask = torch.cat((torch.arange(0, n_cls, dtype=torch.long), perm[n_cls:]), dim=0)
            idx_sorted, _ = full_mask[:n_non_zeros].sort()
            not_idx_sorted, _ = full_mask[n_non_zeros:].sort()
            self.register_buffer("input_mask_idx", idx_sorted, persistent=True)
            self.register_buffer("input_mask_not_idx", not_idx_sorted, persistent=True)
            self.null_connector = nn.Linear(attn_cfg.n_embd, attn_cfg.n_embd, bias=attn_cfg.bias)
        else:
            self.null_connector = nn.Identity()
            self.register_buffer("input_mask_idx", torch.empty(0, dtype=torch.long), persistent=True)
            self.register_buffer("input_mask_not_idx", torch.empty(0, dtype=torch.long), persistent=True)

    def _args(self):
        a, m = self.attn, self.mlp
        return (self.ln_1.weight, self.ln_1.bias, a.c_attn.weight, a.c_attn.bias, a.c_proj.weight, a.c_proj.bias,
                a.attn.table, self.ln_2.weight, self.ln_2.bias, m.c_fc.weight, m.c_fc.bias, m.c_proj.weight,
                m.c_proj.bias)

    def gemm_weights(self):
        """The weights the fused block reads as bf16 GEMM operands."""
        if self.is_moe:
            return []
        a, m = self.attn, self.mlp
        return [a.c_attn.weight, a.c_proj.weight, m.c_fc.weight, m.c_proj.weight]

    def _fused(self, x, double_residual: bool, attn_mask: Optional[torch.Tensor] = None, pack=None):
        if x.dim() != (2 if pack is not None else 3):
            raise ValueError("TransformerBlock expects [B, T, d] (packed rows: [M, d])")
        if self.is_moe:
            T = x.shape[1]
            mask = attn_mask
            if self.is_causal:
                tri = torch.ones((T, T), dtype=torch.bool, device=x.device).tril(0)
                causal = tri.float().masked_fill(~tri, -float("inf"))[None, None]
                mask = causal if mask is None else mask + causal  # :404-408
            y = x + self.attn(self.ln_1(x), mask)
            y = y + self.mlp(self.ln_2(y))
            return y + x if double_residual else y
        if self.attn.attn.table is not None:
            tl = pack.Tp if pack is not None else x.shape[1]
            self.attn.attn.pos_bias.check(tl, tl)
        drop = _drop_args(self, self.attn.attn_dropout.p, self.attn.resid_dropout.p)
        if drop is not None and self.mlp.dropout.p != drop[1]:
            raise NotImplementedError("the fused block applies one dropout p to the attention output and the MLP")
        args = self._args()
        # no backward can run: the forward may keep intermediates on chip (fused MLP)
        infer = not (torch.is_grad_enabled() and (x.requires_grad or any(
            a is not None and a.requires_grad for a in args)))
        with K.bf16_operands(self.gemm_weights()):
            # a general attn_mask is added to the scores on top of the causal flag (:404-408)
            return TransformerBlockFn.apply(x.float(), *args, self.attn.n_head, self.is_causal,
                                            double_residual, self.fp8_gemm, drop, attn_mask, infer, pack)

    def _checkpointing(self) -> bool:
        return bool(self.enable_gradient_checkpointing and self.training and torch.is_grad_enabled())

    def forward(self, x: torch.Tensor, attn_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """:374-380: with enable_gradient_checkpointing in training the block's activations
        are dropped after the forward and recomputed in the backward (non-reentrant
        checkpoint; the CPU generator the dropout seeds come from is restored for the
        recompute, so the masks match)."""
        fn = self._fused_single if not self.is_sparse else self._sparse_forward
        if self._checkpointing():
            return torch.utils.checkpoint.checkpoint(fn, x, attn_mask, use_reentrant=False,
                                                     preserve_rng_state=True)
        return fn(x, attn_mask)

    def _fused_single(self, x: torch.Tensor, attn_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self._fused(x, False, attn_mask)

    def _null(self, x):
        from ...models.lthm.sequence.query_tower import LinearFn
        shp = x.shape
        y = LinearFn.apply(x.reshape(-1, shp[-1]).float().contiguous(), self.null_connector.weight,
                           self.null_connector.bias)
        return y.float().view(shp)

    def _sparse_forward(self, x_orig: torch.Tensor, attn_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """:383-420: the dense block on the kept tokens (gather), the null connector on the
        others, scattered back into place."""
        T = x_orig.size(1)
        idx = self.input_mask_idx[self.input_mask_idx < T]
        if idx.numel() <= 1:
            return x_orig + self._null(x_orig)
        not_idx = self.input_mask_not_idx[self.input_mask_not_idx < T]
        if attn_mask is not None:  # :389-390
            attn_mask = attn_mask[:, :, idx, :][:, :, :, idx]
        x = self._fused(x_orig[:, idx].contiguous(), False, attn_mask)
        x_final = torch.zeros_like(x_orig)
        x_final[:, idx] = x
        if not_idx.numel():
            rest = x_orig[:, not_idx]
            x_final[:, not_idx] = rest + self._null(rest)
        return x_final

    def forward_double_residual(self, x: torch.Tensor, pack=None) -> torch.Tensor:
        """x + block(x) in one op (models/lthm/sequence/query_tower.py:132-137); checkpointed
        like forward (the reference checkpoints block(x) and adds x outside).  ``pack``: x is
        the packed rows of a shared pad prefix (recommendations_amd/pad_prefix.py)."""
        if self._checkpointing():
            return torch.utils.checkpoint.checkpoint(self._fused, x, True, None, pack, use_reentrant=False,
                                                     preserve_rng_state=True)
        return self._fused(x, True, None, pack)

    def pad_prefix_ok(self) -> bool:
        """The block keeps a pad position's state a function of its position: causal, dense,
        no dropout in effect."""
        return (self.is_causal and not self.is_moe and not self.is_sparse
                and _drop_args(self, self.attn.attn_dropout.p, self.attn.resid_dropout.p) is None
                and (not self.training or self.mlp.dropout.p == 0.0))


# ------------------------------------------------------------------ vector-feature layers
class CVEFn(torch.autograd.Function):
    """Standalone CosineVectorEmbedding(s) (commons/transformers/layers.py:462-471):
    normalise, project, bucketize, EmbeddingBag-sum — the product-tower kernel in
    cve_only mode; backward = LDS-privatised bag scatter into the tables.  The
    input (projected direction) receives no gradient, as in the reference
    (bucketize is piecewise constant)."""

    @staticmethod
    def forward(ctx, x, mods, *tables):
        import ctypes
        from ..._lib import STRUCTS, call, dcode, ptr, stream
        require_gpu(x)
        shp = x.shape
        x2 = x.detach().contiguous().view(-1, shp[-1])
        n, Din = x2.shape
        Dout = tables[0].shape[1]
        dev = x.device
        R = sum(t.shape[0] for t in tables)
        tab = torch.cat([t.detach().float() for t in tables]) if len(tables) > 1 else tables[0].detach().float().contiguous()
        proj = torch.cat([m.projection_mat.reshape(-1) for m in mods])
        grids = torch.cat([m.grid.reshape(-1) for m in mods])
        total = sum(m.n_proj for m in mods)
        emb = torch.empty((n, Dout), dtype=torch.bfloat16, device=dev)
        emb32 = torch.empty((n, Dout), dtype=torch.float32, device=dev)
        rows = torch.empty((n, total), dtype=torch.int16, device=dev)
        d = STRUCTS["lthm_ptower_desc"]()
        d.ids, d.x, d.x_dtype, d.Din, d.n, d.Dout = None, ptr(x2), dcode(x2), Din, n, Dout
        d.n_mod = len(mods)
        d.proj, d.grids, d.tables, d.tab_dtype = ptr(proj), ptr(grids), ptr(tab), dcode(tab)
        d.proj_total, d.grid_total, d.cve_rows, d.norm_bins, d.cve_only = proj.numel(), grids.numel(), R, 0, 1
        ro = po = go = 0
        for j, m in enumerate(mods):
            d.mod_nproj[j], d.mod_nbins[j] = m.n_proj, m.num_bins
            d.mod_row_off[j], d.mod_proj_off[j], d.mod_grid_off[j] = ro, po, go
            ro += (m.num_bins + 1) * m.n_proj
            po += m.projection_mat.numel()
            go += m.grid.numel()
        d.emb_out, d.rows_out, d.emb_dtype = ptr(emb32), ptr(rows), dcode(emb32)
        call("lthm_product_tower_fwd", ctypes.addressof(d), stream())
        ctx.save_for_backward(rows)
        segs, cmods, so = [], [], 0
        for j, m in enumerate(mods):
            segs += K.cve_segments(m.n_proj, m.num_bins + 1, so, d.mod_row_off[j])
            cmods.append((so, m.n_proj, d.mod_row_off[j], m.num_bins + 1))
            so += m.n_proj
        ctx.meta = ([t.shape for t in tables], R, shp, segs, cmods)
        return emb32.view(*shp[:-1], Dout)

    @staticmethod
    def backward(ctx, dy):
        (rows,) = ctx.saved_tensors
        shapes, R, shp, segs, cmods = ctx.meta
        dyc = dy.contiguous().view(rows.shape[0], -1).float()
        D = dyc.shape[1]
        if (D in (16, 32, 64, 128, 256) or D % 256 == 0) and len(cmods) <= 16 and rows.shape[0] >= 4096:
            # large batches: the one-hot MFMA reduction (the product tower's; C4 DenseMapper:
            # 65,536 rows x 16 projections into 336 rows, where the LDS scatter-add ran at 36 GB/s).
            # It carries the f32 dY as bf16 hi + lo (2^-17 relative per term); small batches keep
            # the exact f32 LDS accumulation (the reference goldens pin it at 1e-5)
            dtab = K.cve_table_bwd(rows, dyc, R, cmods)
        else:
            dtab = K.segmented_table_bwd(rows, dyc, R, segs)
        out, r = [], 0
        for s in shapes:
            out.append(dtab[r:r + s[0]])
            r += s[0]
        return (None, None, *out)


class CosineVectorEmbedding(nn.Module):
    """commons/transformers/layers.py:443-471 (buffers projection_mat, grid, pos_offset; emb.weight)."""

    def __init__(self, inp_dim: int, emb_dim: int, n_proj: int = 16, num_bins: int = 20):
        super().__init__()
        proj = torch.randn((inp_dim, n_proj))
        proj = torch.nn.functional.normalize(proj, p=2.0, dim=0)
        self.register_buffer("projection_mat", proj, persistent=True)
        resolution = 2.0 / float(num_bins)
        grid = torch.linspace(-1.0, 1.0, steps=num_bins + 1)[:-1] + 0.5 * resolution
        self.register_buffer("grid", grid, persistent=True)
        self.register_buffer("pos_offset", ((num_bins + 1) * torch.arange(0, n_proj, dtype=torch.long)).reshape(n_proj),
                             persistent=True)
        self.emb = nn.EmbeddingBag((num_bins + 1) * n_proj, emb_dim, mode="sum")
        self.emb_dim, self.n_proj, self.num_bins = emb_dim, n_proj, num_bins

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return CVEFn.apply(x, [self], self.emb.weight)


class SimhashVectorIndexer(nn.Module):
    """commons/transformers/layers.py:426-437: int64 codes of the sign bits of
    x @ projection_mat (buffer [inp_dim, n_proj], n_proj <= 64), one HIP kernel."""

    def __init__(self, inp_dim: int, n_proj: int = 16):
        super().__init__()
        self.register_buffer("projection_mat", torch.randn((inp_dim, n_proj)) / math.sqrt(float(inp_dim)),
                             persistent=True)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        codes = K.simhash(x.reshape(-1, x.shape[-1]), self.projection_mat)
        return codes.view(x.shape[:-1])


class CosineLinear(nn.Module):
    """commons/transformers/layers.py:517-525: F.linear(normalize(x), normalize(W)) in f32
    (K.CosineLinearFn)."""

    def __init__(self, inp_dim: int, out_dim: int):
        super().__init__()
        self.weight = nn.Parameter(torch.randn((out_dim, inp_dim)) / math.sqrt(float(inp_dim)))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return K.CosineLinearFn.apply(x, self.weight)


def _gauss_linear(z: torch.Tensor, mean: torch.Tensor, sigma2: float, top_k: Optional[int], emb: nn.Linear,
                  rows_shape) -> torch.Tensor:
    """gaussian_kernel -> view -> emb: the bins come out of the HIP kernel as the bf16
    operand of the MFMA GEMM (K.mlp_chain with one Linear, f32 output)."""
    bins = K.GaussBinsFn.apply(z, mean, sigma2, 0 if top_k is None else top_k, torch.bfloat16)
    return K.mlp_chain(bins.view(*rows_shape, -1), [emb], [K.ACT_NONE], out_f32=True)


def _check_top_k(top_k: Optional[int], num_bins: int) -> Optional[int]:
    if top_k is None:
        return None
    if top_k < 1:
        raise ValueError(f"top_k must be >= 1, got {top_k}")
    return min(top_k, num_bins)


class LearnableCosineVectorEmbedding(nn.Module):
    """commons/transformers/layers.py:531-569: CosineLinear projection, gaussian bins around a
    learnable mean (1, 1, n_proj, num_bins), optional top-k, Linear(n_proj * num_bins, emb_dim)."""

    def __init__(self, inp_dim: int, emb_dim: int, n_proj: int = 16, num_bins: int = 20,
                 sigma_inflation_factor: float = 1.0, top_k: Optional[int] = None):
        super().__init__()
        self.emb_dim, self.n_proj, self.num_bins = emb_dim, n_proj, num_bins
        self.top_k = _check_top_k(top_k, num_bins)
        self.sigma2 = (sigma_inflation_factor * 2.0 / num_bins) ** 2
        self.proj = CosineLinear(inp_dim, n_proj)
        self.mean = nn.Parameter(2 * torch.rand((1, 1, n_proj, num_bins)) - 1)
        self.emb = nn.Linear(n_proj * num_bins, emb_dim, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        bs, seq_len, _ = x.shape
        return _gauss_linear(self.proj(x), self.mean, self.sigma2, self.top_k, self.emb, (bs, seq_len))

    def gaussian_kernel(self, z: torch.Tensor) -> torch.Tensor:
        """:558-569 on its own (f32 out): [bs, seq_len, n_proj] -> [bs, seq_len, n_proj, num_bins]."""
        out = K.GaussBinsFn.apply(z, self.mean, self.sigma2, self.top_k or 0, torch.float32)
        return out.view(*z.shape, self.num_bins)


class ProbabilityVectorEmbedding(nn.Module):
    """commons/transformers/layers.py:575-595: gaussian bins of a probability x [bs, 1]
    around a learnable mean (1, 1, num_bins), optional top-k, Linear(num_bins, emb_dim)."""

    def __init__(self, emb_dim: int, num_bins: int = 10, sigma_inflation_factor: float = 1.0,
                 top_k: Optional[int] = None):
        super().__init__()
        self.emb_dim, self.num_bins = emb_dim, num_bins
        self.top_k = _check_top_k(top_k, num_bins)
        self.sigma2 = (sigma_inflation_factor * 1.0 / num_bins) ** 2
        self.mean = nn.Parameter(torch.rand((1, 1, num_bins)))
        self.emb = nn.Linear(num_bins, emb_dim, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        bs, d = x.shape
        if d != 1:
            raise RuntimeError("ProbabilityVectorEmbedding expects input dim 1")
        return _gauss_linear(x, self.mean, self.sigma2, self.top_k, self.emb, (bs,))

    def gaussian_kernel(self, x: torch.Tensor) -> torch.Tensor:
        """:588-595 on its own (f32 out): [bs, 1] -> [bs, 1, num_bins]."""
        out = K.GaussBinsFn.apply(x, self.mean, self.sigma2, self.top_k or 0, torch.float32)
        return out.view(*x.shape, self.num_bins)


class QuantileMapper(nn.Module):
    """commons/transformers/layers.py:477-487: bucketize(x, q) / (len(q) + 1) - 0.5."""

    def __init__(self, quantiles: List[float]):
        super().__init__()
        self.register_buffer("quantiles", torch.tensor(quantiles), persistent=True)
        self.n_bins = len(quantiles) + 1

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return K.quantile_map(x.contiguous().float(), self.quantiles.view(1, -1).contiguous(), shared=True)


class DenseMapper(nn.Module):
    """commons/transformers/layers.py:490-511: per-feature quantile mapping, concat,
    sum of CosineVectorEmbedding bags (one fused kernel for all modules)."""

    def __init__(self, stats: Dict[str, Any], emb_dim: int, n_projs: List[int], num_bins: List[int]):
        super().__init__()
        self.mappers = nn.ModuleDict({f: QuantileMapper(stats[f]) for f in stats})
        assert len(n_projs) == len(num_bins)
        self.emb = nn.ModuleList([CosineVectorEmbedding(len(self.mappers), emb_dim, n_proj=p, num_bins=b)
                                  for p, b in zip(n_projs, num_bins)])

    def quantile_table(self) -> torch.Tensor:
        return torch.stack([m.quantiles for m in self.mappers.values()])

    def forward(self, batch: Dict[str, torch.Tensor]) -> torch.Tensor:
        x = torch.cat([batch[f].reshape(-1, 1) for f in self.mappers], dim=1).float().contiguous()
        return self.forward_matrix(x)

    def forward_matrix(self, x: torch.Tensor) -> torch.Tensor:
        """Same as forward for the features already stacked as columns of x [B, F]
        (in the mappers' order): one quantile-map kernel, one fused CVE kernel."""
        z = K.quantile_map(x.float().contiguous(), self.quantile_table().contiguous(), shared=False)
        return CVEFn.apply(z.unsqueeze(1), list(self.emb), *[m.emb.weight for m in self.emb]).squeeze(1)


class MLP(nn.Module):
    """commons/transformers/layers.py:67-81 (Linear + GELU-tanh gates)."""

    def __init__(self, in_features: int, out_features: int, gate_sizes: Optional[Tuple[int, ...]] = None, bias: bool = True):
        super().__init__()
        gate_sizes = gate_sizes if gate_sizes is not None else []
        blocks: List[nn.Module] = []
        prev = in_features
        for gsz in gate_sizes:
            blocks.append(nn.Linear(prev, gsz, bias=bias))
            blocks.append(nn.GELU(approximate="tanh"))
            prev = gsz
        blocks.append(nn.Linear(prev, out_features, bias=bias))
        self.model = nn.Sequential(*blocks)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        lins = [m for m in self.model if isinstance(m, nn.Linear)]
        return K.mlp_chain(x, lins, [K.ACT_GELU] * (len(lins) - 1) + [K.ACT_NONE], out_f32=True)


# ------------------------------------------------------------------ mixture of experts
class _MoEGateFn(torch.autograd.Function):
    """softmax(top-k-masked logits / sqrt(in_features)), commons/transformers/layers.py:122-128."""

    @staticmethod
    def forward(ctx, logits, scale, top_k):
        from ..._lib import call, ptr, stream
        require_gpu(logits)
        lg = logits.contiguous()
        M, E = lg.shape
        probs = torch.empty_like(lg)
        call("lthm_moe_gate_fwd", ptr(lg), M, E, scale, top_k, ptr(probs), stream())
        ctx.save_for_backward(probs)
        ctx.scale = scale
        return probs

    @staticmethod
    def backward(ctx, dp):
        from ..._lib import call, ptr, stream
        (probs,) = ctx.saved_tensors
        dp = dp.contiguous().float()
        dl = torch.empty_like(probs)
        call("lthm_moe_gate_bwd", ptr(probs), ptr(dp), probs.shape[0], probs.shape[1], ctx.scale, ptr(dl), stream())
        return dl, None, None


class _MoEExpertsFn(torch.autograd.Function):
    """sum_e g_e (l2_e(gelu(l1_e(x)))) (:130-136) as two GEMMs over the stacked experts:
    H = gelu(x W1^T + b1) with W1 = [l1_0; ...; l1_{E-1}] (one GEMM, GELU epilogue),
    GH = g (x) H per expert block (kernel), out = GH W2^T + g B2 with W2 = [l2_0 | ... ]
    along K and B2 the stacked l2 biases (the bias mix is one more GEMM, fed in as the
    residual of the second)."""

    @staticmethod
    def forward(ctx, x2, g, E, P, *params):
        from ..._lib import call, ptr, stream
        require_gpu(x2, g)
        M = x2.shape[0]
        w1s, b1s, w2s, b2s = params[:E], params[E:2 * E], params[2 * E:3 * E], params[3 * E:]
        W1b = K.cast(torch.cat([w.detach() for w in w1s], 0).contiguous(), torch.bfloat16)   # [E*P, in]
        b1 = torch.cat([b.detach() for b in b1s], 0).contiguous()                            # [E*P]
        W2b = K.cast(torch.cat([w.detach() for w in w2s], 1).contiguous(), torch.bfloat16)   # [out, E*P]
        B2 = torch.stack([b.detach() for b in b2s], 0).contiguous()                          # [E, out]
        xb = K.cast(x2, torch.bfloat16)
        pre = torch.empty((M, E * P), dtype=torch.bfloat16, device=x2.device)
        H = K.linear_fwd(xb, W1b, b1, act=K.ACT_GELU, aux_out=pre)
        GH = torch.empty_like(H)
        gc = g.contiguous()
        call("lthm_moe_scale", ptr(H), ptr(gc), M, E, P, ptr(GH), stream())
        gb = K.cast(gc, torch.bfloat16)
        B2tb = K.cast(B2.t().contiguous(), torch.bfloat16)                                   # [out, E]
        mix = K.linear_fwd(gb, B2tb, out_dtype=torch.float32)                                # g B2
        out = K.linear_fwd(GH, W2b, res1=mix, out_dtype=torch.float32)
        ctx.save_for_backward(xb, H, pre, GH, gc, gb, W1b, W2b, B2)
        ctx.dims = (E, P)
        return out

    @staticmethod
    def backward(ctx, dout):
        from ..._lib import call, ptr, stream
        xb, H, pre, GH, g, gb, W1b, W2b, B2 = ctx.saved_tensors
        E, P = ctx.dims
        M = xb.shape[0]
        dO = dout.contiguous().float()
        dOb = K.cast(dO, torch.bfloat16)
        dW2 = K.linear_wgrad(dOb, GH)                       # [out, E*P]
        dB2 = K.linear_wgrad(dOb, gb).t().contiguous()      # [E, out]
        dGH = K.linear_dgrad(dOb, W2b, out_dtype=torch.float32)
        dpre = torch.empty_like(pre)
        dg = torch.empty((M, E), dtype=torch.float32, device=xb.device)
        call("lthm_moe_hidden_bwd", ptr(dGH), ptr(H), ptr(pre), ptr(g), M, E, P, ptr(dpre), ptr(dg), stream())
        dg = dg + K.linear_fwd(dOb, K.cast(B2, torch.bfloat16), out_dtype=torch.float32)
        dW1 = K.linear_wgrad(dpre, xb)                      # [E*P, in]
        db1 = K.colsum(dpre)
        dx = K.linear_dgrad(dpre, W1b, out_dtype=torch.float32)
        return (dx, dg, None, None, *dW1.split(P, 0), *db1.split(P, 0), *dW2.split(P, 1),
                *[dB2[e] for e in range(E)])


class _MoEUnit(nn.Module):
    """commons/transformers/layers.py:87-95."""

    def __init__(self, in_features: int, out_features: int, proj_features: int):
        super().__init__()
        self.l1 = nn.Linear(in_features, proj_features)
        self.activation = nn.GELU(approximate="tanh")
        self.l2 = nn.Linear(proj_features, out_features)


class MoELinear(nn.Module):
    """commons/transformers/layers.py:101-136 (softmax-gated dense mixture of experts,
    optional top-k threshold), on the HIP GEMMs + gate kernels."""

    def __init__(self, in_features: int, out_features: int, proj_features: int, num_experts: int, bias: bool = True,
                 top_k: Optional[int] = None, gate_sizes: Optional[Tuple[int, ...]] = None):
        super().__init__()
        self._in_features = in_features
        self._out_features = out_features
        self.expert_gates = MLP(in_features, num_experts, gate_sizes=gate_sizes, bias=bias)
        self.experts = nn.ModuleList([_MoEUnit(in_features, out_features, proj_features) for _ in range(num_experts)])
        self.top_k = top_k

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shp = x.shape
        x2 = x.reshape(-1, self._in_features).float().contiguous()
        logits = self.expert_gates(x2)
        E = len(self.experts)
        g = _MoEGateFn.apply(logits, 1.0 / math.sqrt(float(self._in_features)),
                             0 if self.top_k is None else min(self.top_k, E))
        P = self.experts[0].l1.out_features
        params = ([m.l1.weight for m in self.experts] + [m.l1.bias for m in self.experts] +
                  [m.l2.weight for m in self.experts] + [m.l2.bias for m in self.experts])
        out = _MoEExpertsFn.apply(x2, g, E, P, *params)
        return out.view(*shp[:-1], self._out_features)


class _MoEMLP(nn.Module):
    """commons/transformers/layers.py:287-317."""

    def __init__(self, n_embd: int, bias: bool, dropout: float, moe_config: Dict[str, Any]):
        super().__init__()
        kw = dict(proj_features=moe_config["proj_features"], num_experts=moe_config["num_experts"], bias=bias,
                  top_k=moe_config.get("top_k", None), gate_sizes=tuple(moe_config.get("gate_sizes", [])))
        self.c_fc = MoELinear(n_embd, int(moe_config["ff_mult_factor"] * n_embd), **kw)
        self.gelu = nn.GELU(approximate="tanh")
        self.c_proj = MoELinear(int(moe_config["ff_mult_factor"] * n_embd), n_embd, **kw)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = self.c_fc(x)
        h = K.ActivationFn.apply(h.contiguous(), K.ACT_GELU)
        return dropout(self.c_proj(h), self.dropout.p, self.training)  # :316
