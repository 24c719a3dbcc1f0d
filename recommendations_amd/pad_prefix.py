"""Shared pad prefix of the LTHM encoder (query_tower.py:99-137 over the left-padded histories
encoder.py:52 produces).

With causal attention, no dropout and the same position-0 token in every sequence, a pad
position p of sequence b attends to positions 0 .. p only, all of them pads, so its state at
every layer is a function of p alone.  The encoder then runs one "packed" token set:
the pad chain (positions 0 .. P, P the longest pad prefix, once) followed by each sequence's
positions past its pads.  Row-wise work (LayerNorm, the GEMMs, the MLP) runs on the packed rows;
attention reads full-length sequences rebuilt by a row gather (a sequence's pad positions from
the chain), and its key / value gradients at pad positions are summed over the sequences into
the chain rows (lthm_pad_prefix_sum).  Exact: the same functions of the same parameters, the
gradients summed in another order.  csrc/misc.hip, include/lthm.h (lthm_pad_prefix_*).
"""
from __future__ import annotations

import torch

from . import kernels as K
from ._lib import call, dcode, load, ptr, stream


class PadPrefix:
    """Index maps of one batch: ``build`` returns None when a mask row is not a prefix or the
    packed set would not be smaller than 0.9 of the full one."""

    def __init__(self, B, T, P, owner, npad, pof, pof_x, fop):
        self.B, self.T, self.Tp, self.P, self.owner = B, T, T + 1, P, owner
        self.npad, self.pof, self.pof_x, self.fop = npad, pof, pof_x, fop
        self.M = fop.numel()

    @staticmethod
    def build(mask: torch.Tensor, min_gain: float = 0.1):
        """mask [B, T] uint8 view (row stride mask.stride(0)): 1 = pad.  One 16-byte device ->
        host read (the packed shapes)."""
        B, T = mask.shape
        dev = mask.device
        npad = torch.empty(B, dtype=torch.int32, device=dev)
        stats = torch.empty(4, dtype=torch.int32, device=dev)
        call("lthm_pad_prefix_stats", ptr(mask), mask.stride(0), B, T, ptr(npad), ptr(stats), stream())
        ok, valid, P, owner = stats.tolist()
        M = P + 1 + valid
        if ok != 1 or M > (1.0 - min_gain) * B * (T + 1):
            return None
        nv = (T - npad).to(torch.int64)
        voff = torch.cumsum(nv, 0) - nv
        pof = torch.empty(B * (T + 1), dtype=torch.int32, device=dev)
        pof_x = torch.empty_like(pof)
        fop = torch.empty(M, dtype=torch.int32, device=dev)
        call("lthm_pad_prefix_maps", ptr(npad), ptr(voff), B, T + 1, P, owner, ptr(pof), ptr(pof_x), ptr(fop), stream())
        return PadPrefix(B, T, P, owner, npad, pof, pof_x, fop)

    # full rows [B * Tp, W] <-> packed rows [M, W]
    def pack(self, full2d):
        return K.rows_gather(full2d, self.fop)

    def unpack(self, packed2d):
        return K.rows_gather(packed2d, self.pof)

    def unpack_owner(self, packed2d):
        """The adjoint of ``pack``: pad rows of every sequence but the chain's owner are zero."""
        return K.rows_gather(packed2d, self.pof_x)

    def reduce(self, full2d):
        """The adjoint of ``unpack``: valid rows copied, chain row p = the sum of row p over the
        sequences with npad >= p."""
        W = full2d.shape[1]
        dst = K.rows_gather(full2d, self.fop)
        self.chain_sum(full2d, W, self.Tp, dst)
        return dst

    def chain_sum(self, src, W, rows_per_seq, dst):
        """dst rows 0 .. P (leading dim dst.stride(0)) = the chain sums of src viewed as
        [B, rows_per_seq, src.stride(0)] (the first W columns of each row)."""
        wsb = load().lthm_pad_prefix_ws_bytes(self.B, self.P, W)
        ws = torch.empty((wsb + 3) // 4, dtype=torch.float32, device=src.device)
        call("lthm_pad_prefix_sum", ptr(src), src.stride(0), dcode(src), W, ptr(self.npad), self.B, rows_per_seq,
             self.P, ptr(dst), dst.stride(0), ptr(ws), ws.numel() * 4, stream(), _key="pad_prefix_sum")


class PackFn(torch.autograd.Function):
    """[B, Tp, d] -> packed [M, d] (the chain rows read from the owner sequence)."""

    @staticmethod
    def forward(ctx, x, pp):
        ctx.pp = pp
        return pp.pack(x.contiguous().view(-1, x.shape[-1]))

    @staticmethod
    def backward(ctx, g):
        pp = ctx.pp
        return pp.unpack_owner(g.contiguous()).view(pp.B, pp.Tp, -1), None


class UnpackFn(torch.autograd.Function):
    """packed [M, d] -> [B, Tp, d] (every sequence's pad rows read the chain)."""

    @staticmethod
    def forward(ctx, xp, pp):
        ctx.pp = pp
        return pp.unpack(xp.contiguous()).view(pp.B, pp.Tp, -1)

    @staticmethod
    def backward(ctx, g):
        pp = ctx.pp
        return pp.reduce(g.contiguous().view(pp.B * pp.Tp, -1)), None
