"""ORACLE — test infrastructure only (see oracle/__init__.py).

fp32 torch-CPU restatement of the LTHM training step, written from the
reference's source (it cannot be imported: SURVEY.md §3.5 #1):

  Encoder.forward                      models/lthm/sequence/encoder.py:44-61
  ProductTower.forward                 models/lthm/sequence/product_tower.py:43-62
  QueryTower.forward/transformer_enc.  models/lthm/sequence/query_tower.py:60-137
  _mini_batch_mapper / _train_or_val_step_helper   wrapper.py:78-245 (beta = 0)

with the same bug resolutions as the product (DESIGN.md §"Bug resolutions").
Components with reference goldens (KShift, CVE, TransformerBlock, MLP,
cap_gradients) are pinned by tests/test_oracle_golden.py; the composition is
pinned by tests/test_lthm_step_golden_cpu.py against one training step of the
reference's own Encoder / ProductTower / QueryTower forward code and loss
(tests/golden/lthm_step_*.npz; build-defined stand-ins only where the reference
cannot be constructed): the loss is bit-equal, the gradients within 2e-7.

Parameters are read from the product model's state_dict (same names), so the
two paths run identical weights.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import ref


def _p(sd: Dict[str, torch.Tensor], name: str) -> torch.Tensor:
    return sd["_model." + name]


def lthm_forward_loss(sd: Dict[str, torch.Tensor], cfg, batch: Dict[str, torch.Tensor], offsets: np.ndarray,
                      return_outputs: bool = False, logq: Optional[torch.Tensor] = None):
    """Returns the training loss (and intermediate outputs) of one LTHM step on CPU, fp32."""
    pt = cfg.product_tower
    lm = pt.latent_model_config
    d = cfg.emb_dim
    H = cfg.transformer_config.attn_config.n_head
    ids, labels, ts = batch["product_ids"], batch["labels"], batch["timestamp"]
    B, T_full = ids.shape
    # encoder.py:46 (item table is stored bf16 in the product; upcast is exact)
    W_item = _p(sd, "product_emb_module.emb.weight").float()
    embs = ref.kshift_fwd_torch(ids, W_item, lm.num_shifts_latent, lm.normalize_embedding)
    # product_tower.py:43-62
    x = embs.detach()
    x_norm = x.norm(p=2.0, dim=-1)
    mask = torch.logical_or(x_norm < pt.norm_threshold, ids == 0)
    x = F.normalize(x, p=2.0, dim=-1)
    emb = F.linear(x, _p(sd, "product_tower.emb_mapper.weight"), _p(sd, "product_tower.emb_mapper.bias"))
    for j in range(len(pt.cosine_lsh_config)):
        pre = f"product_tower.direction_emb.{j}."
        emb = emb + ref.cve_fwd(x, _p(sd, pre + "projection_mat"), _p(sd, pre + "grid"), _p(sd, pre + "pos_offset"),
                                _p(sd, pre + "emb.weight"))
    if pt.norm_bins > 1:
        emb = emb + ref.histogram_embedding(x_norm, 0.0, 1.0, pt.norm_bins, _p(sd, "product_tower.norm_emb.emb.weight"))
    emb = emb.masked_fill(mask.unsqueeze(-1), 0.0)
    prod = F.linear(emb, _p(sd, "product_tower.product_mapper.weight"))
    # encoder.py:52-54 flip to left padding
    inp, target, mask, labels, ts, ids = [torch.flip(t, dims=[1]) for t in (emb, prod, mask, labels, ts, ids)]
    # query_tower.py:73-86 trim
    span = cfg.export_span
    mask_all_bs = mask.unsqueeze(-1).all(dim=0)
    if mask_all_bs.sum() > T_full - span:
        trim = T_full - span
    else:
        trim = int(torch.nonzero(((~mask_all_bs).cumsum(dim=0) > 0).squeeze(1)).squeeze(1)[0])
    inp, mask, labels, ts, target, ids = [t[:, trim:] for t in (inp, mask, labels, ts, target, ids)]
    T = inp.shape[1]  # seq_len = x.size(1) (query_tower.py:98); a negative trim keeps the last |trim| columns
    trim = T_full - T
    # query_tower.py:89-111
    q = "query_tower."
    xq = F.linear(inp, _p(sd, q + "inp_proj.weight"), _p(sd, q + "inp_proj.bias"))
    xq = xq + ref.flat_fwd(labels, _p(sd, q + "action_embedding._emb_table.weight"), False)
    xq = xq + ref.pattern_from_timelocal(ts, 3600, 24, _p(sd, q + "time_embedding.hod.emb.weight"))
    xq = xq + ref.pattern_from_timelocal(ts, 3600, 24 * 7, _p(sd, q + "time_embedding.how.emb.weight"))
    xq = xq + ref.pattern_from_timelocal(ts, 86400, 7, _p(sd, q + "time_embedding.dow.emb.weight"))
    xq = torch.where(mask.unsqueeze(-1), _p(sd, q + "pad").expand(B, T, -1), xq)
    pos = T - torch.arange(0, T + 1).unsqueeze(0)
    cls = torch.zeros(B, 1, d)
    if cfg.categorical.n_features > 0:
        cls = cls + user_context(sd, cfg, batch["categorical_ids"]).unsqueeze(1)
    xq = torch.cat((cls, xq), dim=1)
    xq = xq + F.embedding(pos, _p(sd, q + "wpe.weight"))
    # query_tower.py:132-137 (double residual) over TransformerBlock (transformers/layers.py:382-415)
    for i in range(cfg.transformer_config.num_layers):
        pre = f"{q}transformer.residual_attn.{i}."
        p = {k[len("_model." + pre):]: v for k, v in sd.items() if k.startswith("_model." + pre)}
        xq = xq + ref.transformer_block(xq, p, H, cfg.transformer_config.is_causal)
    # query_tower.py:118-123
    outcomes = torch.cat((labels, torch.zeros(B, 1, dtype=torch.long)), dim=-1)
    xq = xq + ref.flat_fwd(outcomes, _p(sd, q + "outcome_conditioning._emb_table.weight"), False)
    y = torch.stack([F.linear(xq, _p(sd, f"{q}emb_heads.{i}.weight")) for i in range(cfg.export_tokens)], dim=2)
    loss, stats = contrastive_loss(y, target, mask, offsets, cfg.train_mini_batch_size, cfg.softmax_temperature,
                                   list(cfg.metrics_k_all), logq=logq)
    if return_outputs:
        return loss, dict(y=y, target=target, mask=mask, trim=trim, stats=stats)
    return loss


def user_context(sd, cfg, cat_ids):
    c = cfg.categorical
    W = _p(sd, "user_context.tables.weight")
    P = c.vocab_size
    # feature f reads rows [f P, (f + 1) P) of the batched table; one gather over all
    # features and shifts (one dense table gradient, not one per feature and shift)
    off = (torch.arange(c.n_features, dtype=torch.int64) * P).view(1, -1, 1)
    rows = torch.stack([ref.kshift_row_idx_torch(cat_ids, k, P) for k in range(c.num_shifts)], -1) + off
    g = F.embedding(rows, W)  # [B, F, K, D]
    x = g[:, :, 0]
    for k in range(1, c.num_shifts):  # in-order sum (commons/layers.py:163-166)
        x = x + g[:, :, k]
    x = x / math.sqrt(c.num_shifts)
    e = ref.cap_gradients(x.reshape(cat_ids.shape[0], -1))
    n = len(c.gate_sizes) + 1
    ws = [_p(sd, f"user_context.mlp.model.{2 * i}.weight") for i in range(n)]
    bs = [_p(sd, f"user_context.mlp.model.{2 * i}.bias") for i in range(n)]
    return ref.mlp_quickgelu(e, ws, bs)


def contrastive_loss(next_emb, cur_emb, mask, offsets: np.ndarray, mbs: int, tau: float, ks: List[int],
                     normalize: bool = True, logq: Optional[torch.Tensor] = None):
    """wrapper.py:78-245, offsets given per mini-batch.  ``logq``: None (beta = 0, the
    term vanishes) or the per-token additive correction -beta * logQ [B, T] that
    wrapper.py:131-135, 204-208 subtracts from every logit but the positive's, inside
    the cross entropy only (the rank metrics use the plain logits).
    ``normalize=False`` takes already-normalised embeddings (kernel-level tests feed
    the same bf16-rounded unit vectors the GPU path uses)."""
    B = next_emb.shape[0]
    n_mb = (B + mbs - 1) // mbs
    total = 0.0
    stats = []
    for mb in range(n_mb):
        sl = slice(mb * mbs, min((mb + 1) * mbs, B))
        output_emb = F.normalize(next_emb[sl], p=2.0, dim=-1) if normalize else next_emb[sl]
        input_emb = F.normalize(cur_emb[sl], p=2.0, dim=-1) if normalize else cur_emb[sl]
        m = mask[sl]
        bsz = output_emb.size(0)
        De = output_emb.size(-1)
        seq_len = input_emb.size(-2)
        loss = torch.zeros(())
        st = []
        for i in range(output_emb.size(2)):
            offset = int(offsets[mb, i])
            mask_ = m[:, offset:].contiguous()
            this_seq_len = seq_len - offset
            input_emb_ = input_emb[:, offset:].reshape(-1, De)
            output_emb_ = output_emb[:, :this_seq_len, i].reshape(-1, De)
            bs_ = output_emb_.size(0)
            labels = torch.arange(0, bs_)
            pos = torch.arange(0, bsz).unsqueeze(1).repeat(1, this_seq_len).view(-1, 1)
            pos_matrix = torch.eq(pos, pos.T)
            eye = torch.eye(bs_, dtype=torch.bool)
            mask_ = mask_.view(-1)
            logits = (output_emb_ @ input_emb_.T) / tau
            logits = torch.where(pos_matrix & ~eye, -float("inf"), logits)
            logits = torch.where(mask_.unsqueeze(0), -float("inf"), logits)
            logits = torch.where(mask_.unsqueeze(1), -float("inf"), logits)
            num_negatives = (~torch.isinf(logits)).sum(dim=-1) - 1
            not_use = torch.logical_or(mask_, num_negatives <= 0)
            if bool(not_use.all()):
                st.append(None)
                continue
            logits = logits[~not_use]
            labels = labels[~not_use]
            num_negatives = num_negatives[~not_use]
            ce_logits = logits
            if logq is not None:
                corr = logq[sl][:, offset:].reshape(1, -1).repeat(bs_, 1)
                corr[torch.arange(bs_), torch.arange(bs_)] = 0.0  # :136-141 zero on the positive
                ce_logits = logits + corr[~not_use]
            lu = F.cross_entropy(ce_logits, labels, reduction="none")
            lu = lu[~lu.isnan()]
            if lu.numel() == 0:
                st.append(None)
                continue
            la = lu.mean()
            loss = loss + la
            rank = (logits > logits.gather(1, labels[:, None])).sum(1)
            hits = []
            for k_ in ks:
                k = min(k_, int(num_negatives.min()))
                hits.append(float((logits.topk(k=k)[1] == labels.unsqueeze(-1)).sum(dim=1).float().mean()))
            st.append(dict(loss=float(la), used=int(lu.numel()), neg=float(num_negatives.float().mean()),
                           mean_rank=float(rank.float().mean()), median_rank=float(rank.float().quantile(0.5)),
                           hits=hits))
        total = total + loss / n_mb
        stats.append(st)
    return total, stats
