"""LTHMModelWrapper — drop-in for models/lthm/sequence/wrapper.py:16-275.

Same BaseModelWrapper surface: ``forward(batch) -> dict``, ``train_step``,
``val_step``, ``optim_group``, ``optimizers_for_param_groups``.  The loss of
``_mini_batch_mapper`` + ``_train_or_val_step_helper`` (wrapper.py:78-245) is
one fused op over all mini-batches (``ContrastiveLossFn``, csrc/loss.hip):
identical math per 32-sequence mini-batch and lookahead head, with the
lookahead offsets drawn per mini-batch exactly as wrapper.py:147-153 does
(from a seeded ``random.Random`` instead of the global ``random``).

Bug resolutions: #11 ``self._model_config`` -> ``self.model_config``;
#12 ``current_token_id`` -> ``current_token_ids``; #13 ``sparse`` /
``log_q_config`` / ``loss_type`` declared in the config.  The logQ streaming
estimates are trained on every helper call whatever beta is, as in the reference
(wrapper.py:131-136); the correction enters the loss kernels only when
``log_q_config.beta != 0`` (the shipped YAML has beta = 0, where it is exactly zero).
``train_step`` / ``val_step`` return ``(loss, metrics)`` with the reference's metric
dict (``StepMetrics``: materialised from the device statistics on first read).
"""
from __future__ import annotations

import ctypes
import os
import random
from collections.abc import MutableMapping
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn

from .... import kernels as K
from ...._lib import STRUCTS, TIMER_RECORDS, call, dcode, load, ptr, stream, sub_events, timer_on
from ....commons.base_model_wrapper import BaseModelWrapper
from ....commons.layers import CascadedStreamingLogQCorrectionModule
from ....optim import FusedAdamW, SparseRowAdamW
from .encoder import Encoder

NSTAT_BASE = 8  # csrc/loss.hip CL_NSTAT: stats before hits@k
LOSS_DE = 128  # operand width the loss kernels are compiled for (csrc/loss.hip DE)
_KS_DEV: Dict[tuple, torch.Tensor] = {}  # (metric ks, device) -> int32 device copy


class ContrastiveLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, target, mask, offsets_dev, cfg, logq=None):
        """y [B, T+1, NH, De] (next_token_emb), target [B, T, De] (current_token_emb),
        mask [B, T] uint8 (row stride = mask.stride(0)), offsets_dev int32 [n_mb, NH];
        logq: None or f32 [B, T], the additive logit correction -beta * logQ of each input token."""
        B, Tp, NH, De = y.shape
        T = Tp - 1
        mbs, tau, ks = cfg["mb"], cfg["tau"], cfg["ks"]
        n_mb = (B + mbs - 1) // mbs
        n_max = ((mbs * T + 63) // 64) * 64
        dev = y.device
        yc = y.contiguous()
        tc = target.contiguous()
        rows = (ctx.needs_input_grad[0] and not _OLD_BWD and not _NO_FUSED_ROWS and logq is None
                and 2.0 / tau <= 80.0 and mbs <= 4096 and yc.dtype in (torch.bfloat16, torch.float32))
        if rows and not _NO_VC:
            # the compact path's gather normalises the `out` rows it reads (their norms into ynorm)
            yn, ynorm = None, torch.empty(B * Tp * NH, dtype=torch.float32, device=y.device)
        else:
            yn, ynorm = K.rownorm(yc.view(-1, De))
        # pad positions of `in` are zero rows: every logit against them is excluded
        # anyway, and the loss kernels then need no per-element pad test
        tn, tnorm = K.rownorm(tc.view(-1, De), row_mask=mask)
        f32 = dict(dtype=torch.float32, device=dev)
        lse = torch.empty((NH, n_mb, n_max), **f32)
        pos = torch.empty((NH, n_mb, n_max), **f32)
        diag = torch.empty((NH, n_mb, n_max), **f32)
        w = torch.empty((NH, n_mb, n_max), **f32)
        cnt = torch.empty((NH, n_mb, n_max), dtype=torch.int32, device=dev)
        rank = torch.empty((NH, n_mb, n_max), dtype=torch.int32, device=dev)
        nstat = NSTAT_BASE + len(ks)
        stats = torch.empty((NH, n_mb, nstat), **f32)
        ks_dev = _KS_DEV.get((tuple(ks), dev))  # uploaded once per (ks, device), not per step
        if ks_dev is None:
            ks_dev = _KS_DEV[(tuple(ks), dev)] = torch.tensor(ks, dtype=torch.int32).to(dev)
        lqc = torch.empty((NH, n_mb, n_max), **f32) if logq is not None else None
        # every head in one set of launches (head h's buffers at h * n_mb * n_max)
        d = ContrastiveLossFn._desc(yn, tn, mask, B, T, NH, 0, De, mbs, n_mb, n_max, tau, offsets_dev,
                                    lse[0], pos[0], cnt[0], rank[0], diag[0], w[0], logq,
                                    None if lqc is None else lqc[0])
        d.heads_run, d.head_stride = NH, n_mb * n_max
        wsb = load().lthm_contrastive_ws_bytes(n_mb, n_max, NH)
        ws = torch.empty((wsb + 7) // 8, dtype=torch.float64, device=dev)
        d.stats_ws, d.stats_ws_bytes = ptr(ws), ws.numel() * 8
        # training at the fixed shift: the forward also runs the row side of the backward and
        # writes dy (unit upstream gradient) -- one S pass instead of the forward's plus ROWS'
        dy = None
        vc = None
        if rows:
            dy = torch.empty_like(yc)
            d.y_raw, d.y_norm, d.dy, d.y_dtype = ptr(yc), ptr(ynorm), ptr(dy), dcode(yc)
            if not _NO_VC:
                # valid-row compaction: the S passes run over the non-pad indices only (the
                # workspace is shared with this forward's backward)
                vc = torch.empty(load().lthm_contrastive_vc_ws_bytes(B, T, NH, mbs, n_mb, n_max),
                                 dtype=torch.uint8, device=dev)
                d.vc_ws, d.vc_ws_bytes = ptr(vc), vc.numel()
        # algorithmic work: 2 n^2 De per head (S); with the row side also dS . in (2 n^2 De); with
        # the compaction n is the valid count m of each (mini-batch, head), read after the step
        work = (2.0 if rows else 1.0) * float(sum(cfg["flops"]))
        ev = sub_events("cl_fr32_k" if rows else "cl_fwd_main", work, "flop")
        if ev is not None:  # the fused pass alone, timed inside the call (bench.py's roofline kernel)
            d.main_ev0, d.main_ev1 = ev[0].cuda_event, ev[1].cuda_event
        call("lthm_contrastive_fwd", ctypes.addressof(d), ptr(stats), nstat, ptr(ks_dev), len(ks),
             1.0 / n_mb, stream(), _key="cl_fwd_k", _work=work, _unit="flop")
        if vc is not None and timer_on():
            # the timer's work of both compact passes: 2 x 2 m^2 De per (mini-batch, head); kept
            # for the backward's record also when this forward's passes are not timed
            mv = vc[:NH * n_mb * 4].view(torch.int32).clone()
            vwork = lambda: 4.0 * De * float((mv.double() ** 2).sum())  # noqa: E731
            want = {"cl_fr32_k", "cl_fwd_k"}  # this call's two records, the latest of their keys
            for rec in reversed(TIMER_RECORDS()):
                if rec[0] in want:
                    rec[3] = vwork
                    want.discard(rec[0])
                    if not want:
                        break
            cfg["vc_work"] = vwork
        # loss = sum_mb sum_heads mean-CE / n_mb  (wrapper.py:109-111)
        loss = torch.empty(1, **f32)
        call("lthm_colsum", ptr(stats), 0, NH * n_mb, 1, nstat, ptr(loss), 0, stream())
        loss = loss / n_mb
        ctx.save_for_backward(yc, tc, yn, tn, ynorm, tnorm, lse, w, diag, mask, offsets_dev, logq, lqc, dy)
        ctx.vc = vc
        ctx.vc_work = cfg.get("vc_work")
        ctx.meta = (B, T, NH, De, mbs, n_mb, n_max, tau)
        ctx.stats = stats
        cfg.get("stats_out", []).append(stats)
        ctx.flops = cfg["flops"]
        return loss

    @staticmethod
    def _desc(yn, tn, mask, B, T, NH, h, De, mbs, n_mb, n_max, tau, offsets_dev, lse, pos, cnt, rank, diag, w,
              logq=None, lqc=None):
        d = STRUCTS["lthm_contrastive_desc"]()
        if logq is not None:
            d.logq, d.logq_stride, d.logq_col = ptr(logq), logq.stride(0), ptr(lqc)
        d.out_n, d.in_n, d.mask, d.mask_stride = ptr(yn), ptr(tn), ptr(mask), mask.stride(0)
        d.B, d.T, d.n_heads, d.head, d.De = B, T, NH, h, De
        d.mb_size, d.n_mb, d.n_max, d.tau = mbs, n_mb, n_max, tau
        d.offsets = ptr(offsets_dev)
        d.lse, d.pos, d.cnt, d.rank, d.diag, d.w = ptr(lse), ptr(pos), ptr(cnt), ptr(rank), ptr(diag), ptr(w)
        return d

    @staticmethod
    def backward(ctx, dloss):
        yc, tc, yn, tn, ynorm, tnorm, lse, w, diag, mask, offsets_dev, logq, lqc, dy_f = ctx.saved_tensors
        B, T, NH, De, mbs, n_mb, n_max, tau = ctx.meta
        g = dloss.contiguous().float()
        if _OLD_BWD:
            return ContrastiveLossFn._backward_per_head(ctx, g)
        # every head in one call: the ROWS kernel writes dy per head through F.normalize (or the
        # forward already did: rows_done, dy scaled by g here), the COLS kernel sums dIn over the
        # six heads on chip and writes dt once through F.normalize
        if dy_f is not None and getattr(ctx, "dy_consumed", False):
            # a second backward through this graph (retain_graph): the first one scaled the
            # forward's dy in place and returned it, so run the ROWS side again into a fresh dy
            dy_f = None
        if yn is None and dy_f is None:  # the full passes read every normalised `out` row
            yn, ynorm = K.rownorm(yc.view(-1, De))
        if dy_f is not None:
            ctx.dy_consumed = True
        dy = dy_f if dy_f is not None else torch.empty_like(yc)
        dt = torch.empty_like(tc)
        d = ContrastiveLossFn._desc(yn, tn, mask, B, T, NH, 0, De, mbs, n_mb, n_max, tau, offsets_dev,
                                    lse[0], None, None, None, diag[0], w[0],  # diag: shift scratch
                                    logq, None if lqc is None else lqc[0])
        d.heads_run, d.head_stride = NH, n_mb * n_max
        d.gscale = ptr(g)
        d.y_raw, d.y_norm, d.dy, d.y_dtype = ptr(yc), ptr(ynorm), ptr(dy), dcode(yc)
        d.t_raw, d.t_norm, d.dt, d.t_dtype = ptr(tc), ptr(tnorm), ptr(dt), dcode(tc)
        d.rows_done = 1 if dy_f is not None else 0
        vw = None
        if dy_f is not None and ctx.vc is not None:  # the forward's compact index lists and images
            d.vc_ws, d.vc_ws_bytes = ptr(ctx.vc), ctx.vc.numel()
            vw = ctx.vc_work
        if dy_f is not None:  # the columns pass alone: S recompute + dS^T . out, 4 n^2 De per head
            ev = sub_events("cl_bwd32_k", vw or 2.0 * float(sum(ctx.flops)), "flop")
            if ev is not None:
                d.main_ev0, d.main_ev1 = ev[0].cuda_event, ev[1].cuda_event
        # algorithmic work per head: one S recompute + dS^T . out (2 x 2 n^2 De) with the row side
        # done in the forward; else also dS . in (3 x; the ROWS and COLS kernels each recompute S)
        call("lthm_contrastive_bwd", ctypes.addressof(d), stream(), _key="cl_bwd_k",
             _work=vw or (2.0 if dy_f is not None else 3.0) * float(sum(ctx.flops)), _unit="flop")
        return dy, dt, None, None, None, None

    @staticmethod
    def _backward_per_head(ctx, g):
        """The round-2 backward (16x16x32 kernels, one call per head, f32 d_in read-modify-written
        per head); kept behind LTHM_CL_BWD_OLD=1 for A/B measurements."""
        yc, tc, yn, tn, ynorm, tnorm, lse, w, diag, mask, offsets_dev, logq, lqc, _ = ctx.saved_tensors
        B, T, NH, De, mbs, n_mb, n_max, tau = ctx.meta
        dev = yc.device
        fuse = yc.dtype == torch.bfloat16
        dy = torch.empty_like(yc) if fuse else None
        d_out = None if fuse else torch.empty((B, T + 1, NH, De), dtype=torch.float32, device=dev)
        d_in = K.zeros((B, T, De), torch.float32, dev)
        for h in range(NH):
            d = ContrastiveLossFn._desc(yn, tn, mask, B, T, NH, h, De, mbs, n_mb, n_max, tau, offsets_dev,
                                        lse[h], None, None, None, diag[h], w[h], logq, None if lqc is None else lqc[h])
            d.gscale, d.d_out, d.d_in = ptr(g), ptr(d_out), ptr(d_in)
            if fuse:
                d.y_raw, d.y_norm, d.dy, d.y_dtype = ptr(yc), ptr(ynorm), ptr(dy), dcode(yc)
            call("lthm_contrastive_bwd", ctypes.addressof(d), stream(), _key="cl_bwd_k",
                 _work=3.0 * ctx.flops[h], _unit="flop")
        if not fuse:
            dy, _ = K.rownorm_bwd(yc.view(-1, De), ynorm, d_out.view(-1, De))
        dt, _ = K.rownorm_bwd(tc.view(-1, De), tnorm, d_in.view(-1, De))
        return dy.view(yc.shape), dt.view(tc.shape), None, None, None, None


_OLD_BWD = os.environ.get("LTHM_CL_BWD_OLD") == "1"
_NO_FUSED_ROWS = os.environ.get("LTHM_CL_NO_FUSED_ROWS") == "1"  # A/B: separate forward and ROWS passes
_NO_VC = os.environ.get("LTHM_CL_VC") == "0"  # A/B: the full n x n passes (no valid-row compaction)


def contrastive_step(y, tgt, mask, offs: np.ndarray, mbs: int, tau: float, ks: List[int], logq=None):
    """All helper calls of one train / val step (wrapper.py:78-245) on the fused kernels.

    y [B, T+1, NH, De] next_token_emb, tgt [B, T, De] current_token_emb, mask [B, T] pad
    mask, offs [n_mb, NH] the lookahead offsets drawn per helper call, mbs sequences per
    helper call (B: the whole batch).  Returns the loss (mean over helper calls of the
    per-call sum over heads) and the device statistics [NH, n_mb, 8 + len(ks)]."""
    B, T = y.shape[0], y.shape[1] - 1
    n_mb = (B + mbs - 1) // mbs
    assert offs.shape[0] == n_mb, (offs.shape, n_mb)
    offsets_dev = torch.from_numpy(np.ascontiguousarray(offs, dtype=np.int32)).pin_memory().to(
        y.device, non_blocking=True)
    flops = []  # algorithmic logits flops per head: sum over mini-batches of 2 n^2 De
    for h in range(offs.shape[1]):
        tot = 0.0
        for mb in range(n_mb):
            n = min(mbs, B - mb * mbs) * max(T - int(offs[mb, h]), 0)
            tot += 2.0 * n * n * y.shape[-1]
        flops.append(tot)
    holder = []
    cfg = dict(mb=mbs, tau=tau, ks=list(ks), flops=flops, stats_out=holder)
    if mask.dtype == torch.bool:
        mask = mask.view(torch.uint8)
    loss = ContrastiveLossFn.apply(y, tgt, mask, offsets_dev, cfg, logq)
    return loss, holder[0]


class LTHMModelWrapper(BaseModelWrapper):
    def __init__(self, model_config, stats=None):
        super().__init__(dummy_params=model_config.sparse, sparse=model_config.sparse)
        self.model_config = model_config
        de = model_config.product_tower.product_emb_dim
        if de != LOSS_DE:
            # the fused loss kernels are compiled for one operand width (csrc/loss.hip DE); refuse at
            # construction instead of at the first train_step (query_tower.py:54-55, product_tower.py:37-39)
            raise ValueError(f"product_emb_dim={de} is not supported by the fused contrastive loss kernels "
                             f"(built for product_emb_dim={LOSS_DE}, model/lthm.yaml:22)")
        self._sparse = model_config.sparse
        self._softmax_temperature = model_config.softmax_temperature
        self._export_span = model_config.export_span
        self._export_tokens = model_config.export_tokens
        self._loss_type = model_config.loss_type
        self._metrics_k_all = list(model_config.metrics_k_all)
        self._lookahead = list(model_config.lookahead)
        self._model = Encoder(model_config)
        # wrapper.py:34-42 (built whatever beta is, so the state_dict carries its a / b buffers)
        lq = model_config.log_q_config
        self._log_q_beta = float(lq.beta)
        self._log_q_calc = CascadedStreamingLogQCorrectionModule(
            num_buckets=lq.num_buckets, hash_offsets=lq.hash_offsets, alpha=lq.alpha, p_init=lq.p_init)
        self.batch_idx = 0
        self._rng = random.Random(model_config.seed)
        self.last_stats = None

    # wrapper.py:48-64
    def format_inputs(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        for k in ("product_ids", "labels", "timestamp"):
            assert batch[k].dtype == torch.int64, f"{k} was expected to be of type long but was {batch[k].dtype}"
        return batch

    def forward(self, batch: Dict[str, torch.Tensor]):
        return self._model(self.format_inputs(batch))

    def prefetch(self, batch: Dict[str, torch.Tensor], ready=None) -> None:
        """Run the frozen item-table lookup of a later ``forward(batch)`` now, on a side
        stream (``Encoder.prefetch``; build-defined, the reference has no pipelining).
        ``ready``: an event recorded when ``batch``'s ids became valid."""
        self._model.prefetch(self.format_inputs(batch), ready)

    def draw_offsets(self, n_mb: int) -> np.ndarray:
        """wrapper.py:147-153, once per mini-batch: head 0 uses lookahead[0], head i
        draws randint(previous + 1, lookahead[i])."""
        out = np.zeros((n_mb, len(self._lookahead)), dtype=np.int32)
        for mb in range(n_mb):
            prev = 0
            for i, mx in enumerate(self._lookahead):
                if i == 0:
                    off = mx
                else:
                    off = self._rng.randint(prev + 1, mx)
                prev = off
                out[mb, i] = off
        return out

    def train_step(self, batch, output):
        return self._loss_and_metrics(output, training=True)

    def val_step(self, batch, output):
        return self._loss_and_metrics(output, training=False)

    def _loss_and_metrics(self, output, training: bool):
        """_mini_batch_mapper (wrapper.py:78-112): training splits the batch into
        train_mini_batch_size sequences per helper call; val_step and a negative
        train_mini_batch_size run the helper (wrapper.py:114-245) once over the whole
        batch.  Every helper call of the step runs in one fused launch set."""
        y = output["next_token_emb"]
        tgt = output["current_token_emb"]
        mask = output["current_token_mask"]
        B, Tp = y.shape[0], y.shape[1]
        T = Tp - 1
        step_type = "train" if training else "val"
        mbs = self.model_config.train_mini_batch_size
        whole = (not training) or mbs < 0
        mbs = B if whole else min(mbs, B)
        n_mb = (B + mbs - 1) // mbs
        offs = self.draw_offsets(n_mb)  # a head whose offset reaches past T has no rows (wrapper.py:157-159)
        # wrapper.py:126-130 per helper call in order, train and val alike: logQ train_step on its
        # non-pad ids, then the correction -beta * logQ of its ids (zeroed on the positive
        # in-kernel).  The streaming estimates advance whatever beta is, as the reference's do;
        # the correction enters the loss only when beta != 0 (with beta = 0 it is exactly zero)
        want = self._log_q_beta != 0.0
        logq = self._log_q_calc.stream_correction(output["current_token_ids"], mask, mbs, self.batch_idx,
                                                  self._log_q_beta, want_out=want)
        loss, stats = contrastive_step(y, tgt, mask, offs, mbs, self._softmax_temperature, self._metrics_k_all, logq)
        self.batch_idx += n_mb  # the reference counts helper calls, one per mini-batch
        self.last_stats = (stats, offs, step_type, B, T, mbs, whole)
        return loss, StepMetrics(stats, offs, step_type, self._metrics_k_all, B, T, mbs, whole)

    def metrics(self) -> Dict[str, float]:
        """Metric dict of the last train_step / val_step as a plain dict (the same values
        train_step / val_step return)."""
        if self.last_stats is None:
            return {}
        stats, offs, step_type, B, T, mbs, whole = self.last_stats
        return lthm_metrics(stats.cpu().numpy(), offs, step_type, self._metrics_k_all, B, T, mbs, whole)

    def is_sparse(self, param_name: str):
        return super().is_sparse(param_name) or "user_context.tables" in param_name

    def optim_group(self, parent_module: nn.Module, full_param_name: str, numel: int) -> Optional[str]:
        return "SPARSE_ROWS" if "user_context.tables" in full_param_name else "USE_OPTIM"

    def optimizers_for_param_groups(self, param_groups: Dict[str, List[torch.nn.Parameter]]):
        result = []
        dense = [p for p in param_groups.get("USE_OPTIM", []) if p.requires_grad]
        if dense:
            result.append(FusedAdamW(dense, lr=self.model_config.lr, weight_decay=self.model_config.weight_decay,
                                     betas=self.model_config.betas))
        if param_groups.get("SPARSE_ROWS") and self._model.user_context is not None:
            result.append(SparseRowAdamW([self._model.user_context.tables], lr=self.model_config.lr,
                                         betas=self.model_config.betas, weight_decay=self.model_config.weight_decay))
        return result

    def param_groups(self) -> Dict[str, List[torch.nn.Parameter]]:
        groups: Dict[str, List[torch.nn.Parameter]] = {}
        for name, p in self.named_parameters():
            groups.setdefault(self.optim_group(self, name, p.numel()), []).append(p)
        return groups


class StepMetrics(MutableMapping):
    """The metric dict ``train_step`` / ``val_step`` return (wrapper.py:71-112, 139-142,
    221-245: same keys, same values), built lazily from the loss kernels' device statistics.

    Construction issues one non-blocking device->host copy of the [NH, n_mb, 8 + len(ks)]
    statistics into pinned memory on the current stream and records an event; nothing
    waits for the GPU until a key, the length or the repr is first read, so a training
    loop that never reads the dict pays no synchronisation.  After that it behaves as a
    plain mutable dict (the reference trainer adds into the first step's dict in place,
    accelerate_training_strategy.py:405-409)."""

    __slots__ = ("_pending", "_d")

    def __init__(self, stats: torch.Tensor, offs: np.ndarray, step_type: str, ks: List[int], B: int, T: int,
                 mbs: int, whole: bool):
        host = torch.empty(stats.shape, dtype=stats.dtype, pin_memory=True)
        host.copy_(stats, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pending = (host, ev, offs, step_type, list(ks), B, T, mbs, whole)
        self._d: Optional[Dict[str, float]] = None

    def _dict(self) -> Dict[str, float]:
        if self._d is None:
            host, ev, offs, step_type, ks, B, T, mbs, whole = self._pending
            ev.synchronize()
            self._d = lthm_metrics(host.numpy(), offs, step_type, ks, B, T, mbs, whole)
            self._pending = None
        return self._d

    def __getitem__(self, k):
        return self._dict()[k]

    def __setitem__(self, k, v):
        self._dict()[k] = v

    def __delitem__(self, k):
        del self._dict()[k]

    def __iter__(self):
        return iter(self._dict())

    def __len__(self):
        return len(self._dict())

    def __repr__(self):
        return repr(self._dict())

    def copy(self) -> Dict[str, float]:
        return dict(self._dict())


def lthm_metrics(stats: np.ndarray, offs: np.ndarray, step_type: str, ks: List[int], B: int, T: int, mbs: int,
                 whole: bool) -> Dict[str, float]:
    """The reference's metric dict from the per-(head, mini-batch) kernel statistics.

    Per helper call (wrapper.py:139-142, 221-242): batch size, sequence length, and per head
    with a usable row the offset-keyed effective batch size, mean negatives, used tokens,
    mean CE, mean / median hit position and hits@k, then the summed loss.  A head none of whose
    used rows has a finite CE records nothing (wrapper.py:210-214: ``used_tokens == 0``);
    effective batch size and used tokens differ only when some CE is NaN.  With mini-batches
    (wrapper.py:95-111) each key is averaged over the helper calls that produced it and
    ``{step}_overall_batch_size`` is added; a whole-batch call returns its dict as is."""
    NH, n_mb, _ = stats.shape
    per = []
    for mb in range(n_mb):
        m = {f"{step_type}_batch_size": min(mbs, B - mb * mbs), f"{step_type}_seq_len": T}
        loss_mb = 0.0
        for h in range(NH):
            st = stats[h, mb]
            off = int(offs[mb, h])
            used, used_tokens = int(st[1]), int(st[7])
            if used == 0 or used_tokens == 0:
                continue
            loss_mb += float(st[0])
            m[f"{step_type}_effective_batch_size_offset_{off}"] = used
            m[f"{step_type}_average_negatives_per_token_offset_{off}"] = float(st[2])
            m[f"{step_type}_used_tokens_offset_{off}"] = used_tokens
            m[f"{step_type}_loss_all_tokens_offset_{off}"] = float(st[0])
            m[f"{step_type}_average_hit_position_offset_{off}"] = float(st[4])
            m[f"{step_type}_median_hit_position_offset_{off}"] = float(st[5])
            for q, k in enumerate(ks):
                m[f"{step_type}_hit_rate_at_{k}_offset_{off}"] = float(st[NSTAT_BASE + q])
        m[f"{step_type}_loss"] = loss_mb
        per.append(m)
    if whole:
        return per[0]
    acc: Dict[str, float] = {}
    cnt: Dict[str, int] = {}
    for m in per:
        for k, v in m.items():
            acc[k] = acc.get(k, 0.0) + v
            cnt[k] = cnt.get(k, 0) + 1
    out = {k: acc[k] / cnt[k] for k in acc}
    out[f"{step_type}_overall_batch_size"] = B
    return out
