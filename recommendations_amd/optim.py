"""Optimizers whose steps are single fused HIP kernels (include/lthm.h).

``FusedAdamW`` / ``FusedAdagrad`` reproduce torch.optim.AdamW / Adagrad update
rules (wrapper.py:263-275, embedding_module_gen.py:97,137) on fp32 parameters.
``SparseRowAdamW`` / ``SparseRowAdagrad`` update only the rows of a
``TableBatchedKShiftEmbedding`` that the step touched (lazy Adam: untouched
rows do not decay) — the documented deviation that makes 100M-row tables
trainable; bias corrections use the optimizer's global step.
"""
from __future__ import annotations

from typing import Iterable

import os

import torch

from . import kernels as K


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self._plans = {}

    def load_state_dict(self, state_dict):
        self._plans = {}  # the plans point at the moment buffers being replaced
        super().load_state_dict(state_dict)

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        """One multi-tensor launch per (param group, step count) bucket of up to 48
        tensors (lthm_adamw_multi) instead of one launch per parameter."""
        loss = closure() if closure is not None else None
        fast = self.__dict__.setdefault("_plans", {})  # (set in __init__; kept for unpickled optimizers)
        for gi, g in enumerate(self.param_groups):
            # steady state: the same parameters, gradients at the same addresses and one
            # shared step count -> reuse the previous step's pointer arrays (the per-tensor
            # checks and ctypes packing cost ~0.6 ms of host time per C2 step)
            live = [p for p in g["params"] if p.grad is not None]
            key = self._plan_key(live)
            hit = fast.get(gi)
            if hit is not None and hit[0] == key:
                step = hit[2] + 1
                for p in live:
                    self.state[p]["step"] = step
                fast[gi] = (self._plan_key(live), hit[1], step)
                K.adamw_multi_run(hit[1], g["lr"], g["betas"], g["eps"], g["weight_decay"], step,
                                  grad_scale=grad_scale)
                continue
            fast.pop(gi, None)
            buckets = {}
            for p in g["params"]:
                if p.grad is None:
                    continue
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32:
                    raise TypeError("FusedAdamW keeps fp32 masters")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = K.zeros(p.shape, torch.float32, p.device)
                    st["exp_avg_sq"] = K.zeros(p.shape, torch.float32, p.device)
                st["step"] += 1
                grad = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                b = buckets.setdefault(st["step"], ([], [], [], []))
                for lst, t in zip(b, (p.data, grad, st["exp_avg"], st["exp_avg_sq"])):
                    lst.append(t)
            for step, (ps, gs, ms, vs) in buckets.items():
                K.adamw_multi_(ps, gs, ms, vs, g["lr"], g["betas"], g["eps"], g["weight_decay"], step,
                               grad_scale=grad_scale)
            if len(buckets) == 1 and all(p.grad.is_contiguous() for p in live):
                (step, (ps, gs, ms, vs)), = buckets.items()
                fast[gi] = (self._plan_key(live), K.adamw_multi_plan(ps, gs, ms, vs), step)
        return loss

    def _plan_key(self, live):
        """What a kept pointer plan depends on: each parameter, its gradient, its moment
        buffers (a state entry replaced other than by load_state_dict invalidates the plan
        instead of leaving the kernel updating orphaned buffers) and its step count."""
        out = []
        for p in live:
            st = self.state.get(p)
            if st:
                step = st["step"]
                out.append((id(p), p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                            st["exp_avg_sq"].data_ptr(), float(step) if torch.is_tensor(step) else step))
            else:
                out.append((id(p), p.data_ptr(), p.grad.data_ptr(), 0, 0, -1))
        return tuple(out)


class FusedAdagrad(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-2, lr_decay=0.0, weight_decay=0.0, eps=1e-10, initial_accumulator_value=0.0):
        super().__init__(params, dict(lr=lr, lr_decay=lr_decay, weight_decay=weight_decay, eps=eps,
                                      initial_accumulator_value=initial_accumulator_value))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["sum"] = torch.full_like(p, g["initial_accumulator_value"])
                st["step"] += 1
                K.adagrad_(p.data, p.grad.contiguous(), st["sum"], g["lr"], g["lr_decay"], g["eps"],
                           g["weight_decay"], st["step"])
        return loss


# The bitmap tables' row-wise step leaves the gradient rows (the next backward stores them at their
# first touch): C4 sparse AdamW 1.078 -> 0.939 ms, step 3.995 -> 3.848 ms (profiles/r06c/).
# LTHM_SPARSE_KEEP_GRAD=0 re-zeroes them as the int32-flag tables' step does (A/B)
_KEEP_GRAD = os.environ.get("LTHM_SPARSE_KEEP_GRAD", "1") != "0"


def _clear_touched(m, bits):
    """After a row-wise step: the touched-row list is consumed; a touched-row bitmap (K = 1
    tables, F * P / 8 bytes) is cleared whole, int32 flags were re-zeroed per row by the kernel."""
    if bits:
        m.sparse_flags.zero_()
    m.sparse_count.zero_()
    m.sparse_pending = 0


class SparseRowAdamW:
    """Row-wise AdamW over TableBatchedKShiftEmbedding modules (sparse=True)."""

    def __init__(self, modules: Iterable, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.modules = list(modules)
        self.lr, self.betas, self.eps, self.weight_decay = lr, tuple(betas), eps, weight_decay
        self.step_count = 0
        self.state = {}

    @torch.no_grad()
    def step(self):
        self.step_count += 1
        for m in self.modules:
            if m.sparse_count is None or m.sparse_pending == 0:
                continue
            st = self.state.get(id(m))
            if st is None:
                st = self.state[id(m)] = (K.zeros(m.weight.shape, torch.float32, m.weight.device),
                                          K.zeros(m.weight.shape, torch.float32, m.weight.device))
            shadow = m.shadow_current()
            bits = getattr(m, "sparse_flag_bits", False)
            # a bitmap table's next backward stores each row at its first touch: no re-zeroing
            K.sparse_adamw_(m.sparse_rows, m.sparse_count, min(m.sparse_pending, m.weight.shape[0]), m.weight.data,
                            m.sparse_grad, st[0], st[1], None if bits else m.sparse_flags, self.lr, self.betas,
                            self.eps, self.weight_decay, self.step_count, shadow=shadow, keep_grad=bits and _KEEP_GRAD)
            _clear_touched(m, bits)

    def zero_grad(self, set_to_none: bool = True):
        pass  # the row-wise step consumes and re-zeroes exactly the rows it updates


class SparseRowAdagrad(SparseRowAdamW):
    """Row-wise Adagrad over KShift tables (sparse=True).

    ``fused=True``: the tables' backward only records its lookups and ``step`` runs the fused
    dedup + Adagrad (lthm_kshift_adagrad_fused): each touched row's gradient is summed and
    consumed by its update in one call, no gradient row stored and no [F * P, D] gradient buffer
    allocated.  Valid where nothing reads or rescales the table gradients between backward and
    step -- the item-embedding generator (embedding_module_gen.py:137,151-153: ``loss.backward();
    optim.step()`` with torch.optim.Adagrad, no clipping)."""

    def __init__(self, modules: Iterable, lr=1e-2, lr_decay=0.0, eps=1e-10, fused: bool = False):
        super().__init__(modules, lr=lr)
        self.lr_decay, self.eps = lr_decay, eps
        self.fused = fused
        if fused:
            for m in self.modules:
                m.fused_row_step = True
                m.fused_pending = []

    @torch.no_grad()
    def _step_fused(self, m):
        recs, m.fused_pending = m.fused_pending, []
        if not recs:
            return
        st = self.state.get(id(m))
        if st is None:
            st = self.state[id(m)] = K.zeros(m.weight.shape, torch.float32, m.weight.device)
        if len(recs) == 1:
            ids, gy, out, norms = recs[0]
        else:  # several backwards before one step: their lookups in order
            ids = torch.cat([r[0].reshape(-1, m._F) for r in recs])
            gy = torch.cat([r[1].reshape(-1, r[1].shape[-1]) for r in recs])
            out = None if recs[0][2] is None else torch.cat([r[2].reshape(-1, r[2].shape[-1]) for r in recs])
            norms = None if recs[0][3] is None else torch.cat([r[3].reshape(-1) for r in recs])
        # torch.optim.Adagrad: clr = lr / (1 + (step - 1) * lr_decay), in double, applied as f32
        clr = self.lr / (1.0 + (self.step_count - 1) * self.lr_decay)
        K.kshift_adagrad_fused(ids, gy, out, norms, m._num_embeddings, m._num_shifts, m._mode, m._F, m.weight.data,
                               st, clr, self.eps)
        m.invalidate_shadow()  # rows rewritten outside torch's version counter

    def zero_grad(self, set_to_none: bool = True):
        """fused: the recorded lookups are the tables' pending gradient -- dropped, as
        torch's zero_grad drops .grad (the two-pass form keeps its row-wise semantics)."""
        if self.fused:
            for m in self.modules:
                m.fused_pending = []

    @torch.no_grad()
    def step(self):
        self.step_count += 1
        for m in self.modules:
            if self.fused:
                self._step_fused(m)
                continue
            if m.sparse_count is None or m.sparse_pending == 0:
                continue
            st = self.state.get(id(m))
            if st is None:
                st = self.state[id(m)] = K.zeros(m.weight.shape, torch.float32, m.weight.device)
            shadow = m.shadow_current()
            bits = getattr(m, "sparse_flag_bits", False)
            K.sparse_adagrad_(m.sparse_rows, m.sparse_count, min(m.sparse_pending, m.weight.shape[0]), m.weight.data,
                              m.sparse_grad, st, None if bits else m.sparse_flags, self.lr, self.lr_decay, self.eps,
                              self.step_count, shadow=shadow, keep_grad=bits and _KEEP_GRAD)
            _clear_touched(m, bits)
