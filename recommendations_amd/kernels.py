"""torch.autograd.Function wrappers over the C ABI (include/lthm.h).

These are the only places the product path computes anything: each op checks
that its tensors are on the GPU (no CPU fallback), allocates outputs through
torch, and launches the gfx950 kernel on torch's current stream.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ._lib import BF16, F32, call, dcode, ptr, require_gpu, stream

KSHIFT_SCALE, KSHIFT_NORMALIZE, KSHIFT_NONE = 0, 1, 2


# ----------------------------------------------------------------- KShift
def kshift_rows(ids: torch.Tensor, P: int, K: int) -> torch.Tensor:
    """All K row indices of every id: [.., K] int64 (commons/layers.py:174-185)."""
    require_gpu(ids)
    rows = torch.empty(ids.shape + (K,), dtype=torch.int64, device=ids.device)
    call("lthm_kshift_rows", ptr(ids), ids.numel(), P, K, ptr(rows), stream())
    return rows


class KShiftFn(torch.autograd.Function):
    """Gather + in-order pool of K table rows (commons/layers.py:152-172).

    ``F`` > 1 selects the table-batched layout: ids [..., F], weight [F*P, D],
    feature f reading rows [f*P, (f+1)*P).
    """

    @staticmethod
    def forward(ctx, ids, weight, P: int, K: int, mode: int, F: int, out_dtype):
        require_gpu(ids, weight)
        D = weight.shape[1]
        n = ids.numel() // F
        out = torch.empty(ids.shape + (D,), dtype=out_dtype, device=ids.device)
        need_norms = mode == KSHIFT_NORMALIZE and weight.requires_grad
        norms = torch.empty(ids.shape, dtype=torch.float32, device=ids.device) if need_norms else None
        call("lthm_kshift_fwd_multi", ptr(ids), n, F, ptr(weight), dcode(weight), P, D, K, mode,
             ptr(out), dcode(out), ptr(norms), stream())
        ctx.save_for_backward(ids, out if mode == KSHIFT_NORMALIZE else None, norms)
        ctx.cfg = (P, K, mode, F, D, weight.shape, weight.dtype)
        return out

    @staticmethod
    def backward(ctx, gy):
        ids, out, norms = ctx.saved_tensors
        P, K, mode, F, D, wshape, wdtype = ctx.cfg
        gy = gy.contiguous()
        dW = torch.zeros(wshape, dtype=torch.float32, device=gy.device)
        n = ids.numel() // F
        call("lthm_kshift_bwd_dense", ptr(ids), n, F, ptr(gy), dcode(gy),
             ptr(out) if out is not None else None, dcode(out) if out is not None else F32,
             ptr(norms), P, D, K, mode, ptr(dW), stream())
        if wdtype != torch.float32:
            dW = dW.to(wdtype)
        return None, dW, None, None, None, None, None


def kshift(ids, weight, P: int, K: int, mode: int, F: int = 1, out_dtype=None):
    if out_dtype is None:
        out_dtype = weight.dtype
    return KShiftFn.apply(ids.contiguous(), weight, P, K, mode, F, out_dtype)
