"""ProductTower — drop-in for models/lthm/sequence/product_tower.py:10-62.

Module tree and parameter names follow the reference (``emb_mapper``,
``direction_emb.{j}.emb.weight`` + buffers, ``norm_emb.emb.weight``,
``product_mapper.weight``).  The forward is one fused gfx950 kernel per token
(``lthm_product_tower_fwd``) plus the product_mapper MFMA GEMM; the backward
is an LDS-privatised scatter into the 6 CVE tables + histogram table and two
weight-gradient GEMMs.  Bug resolutions: #1 HistogramEmbedding
is build-defined (commons/layers.py here), #2 ``num_proj`` maps to ``n_proj``,
#3 the config fields are declared (models/lthm/config.py).
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn as nn

from .... import kernels as K
from ...._lib import STRUCTS, call, dcode, ptr, require_gpu, stream
from ....commons.layers import HistogramEmbedding
from ....commons.transformers.layers import CosineVectorEmbedding


# token compaction: a pad token (id 0) has its embedding masked to zero (product_tower.py:49,
# 58), so no output or gradient of the tower depends on it; the tower runs on the non-pad tokens
# and its outputs are expanded with zero rows (LTHM_TOWER_COMPACT=0: every token)
_COMPACT = os.environ.get("LTHM_TOWER_COMPACT", "1") != "0"


class ProductTowerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, x, w_map, b_map, w_pm, hist_w, tower, *tables):
        require_gpu(ids, x)
        n_full = ids.numel()
        ctx.full = None
        # compaction gathers x, emb, prod and their gradients by 16-B row pieces (rows_gather): every
        # one of those row widths must be a multiple of 16 bytes; and it reads one count to the host,
        # which a CUDA-graph capture cannot do
        rows16 = (x.shape[-1] * x.element_size() % 16 == 0 and w_map.shape[0] % 8 == 0 and w_pm.shape[0] % 8 == 0)
        if _COMPACT and n_full > 0 and rows16 and not torch.cuda.is_current_stream_capturing():
            ids_f = ids.reshape(-1)
            valid = ids_f != 0
            pos = torch.cumsum(valid, 0, dtype=torch.int32)
            c = int(pos[-1])  # one 4-byte device->host read: the compact shapes
            if c < n_full:
                inv = torch.where(valid, pos - 1, torch.full_like(pos, -1))  # full row -> compact row or -1
                idx = torch.nonzero(valid).view(-1).to(torch.int32)          # compact row -> full row
                shape = ids.shape
                ids = ids_f.index_select(0, idx.long())
                x = K.rows_gather(x.reshape(n_full, -1).contiguous(), idx)
                ctx.full = (shape, n_full, idx, inv)
        n = ids.numel()
        Din, Dout = x.shape[-1], w_map.shape[0]
        dev = x.device
        cve = tower.direction_emb
        R_cve = sum(t.shape[0] for t in tables)
        nb = tower.norm_bins if tower.norm_bins > 1 else 0
        # bf16 gather images of the small tables (one buffer) and the product_mapper operand:
        # one multi-tensor cast launch (f32 masters; a per-table cast was 8 launches)
        tab = torch.empty((R_cve + max(nb, 1), Dout), dtype=torch.bfloat16, device=dev)
        w_pm_b = torch.empty(w_pm.shape, dtype=torch.bfloat16, device=dev)
        srcs, dsts, r = [], [], 0
        for t in tables:
            srcs.append(t.detach().contiguous())
            dsts.append(tab[r:r + t.shape[0]])
            r += t.shape[0]
        if nb:
            srcs.append(hist_w.detach().contiguous())
            dsts.append(tab[R_cve:R_cve + nb])
        srcs.append(w_pm.detach().contiguous())
        dsts.append(w_pm_b)
        if all(t.dtype == torch.float32 for t in srcs):
            K.cast_multi_bf16_into(srcs, dsts)
        else:
            for t, o in zip(srcs, dsts):
                call("lthm_cast", ptr(t), dcode(t), ptr(o), dcode(o), t.numel(), stream())
        # the CVE buffers' concatenation, kept while the buffers are unchanged
        key = tuple((m.projection_mat.data_ptr(), m.projection_mat._version, m.grid.data_ptr(), m.grid._version)
                    for m in cve)
        hit = getattr(tower, "_cve_cat", None)
        if hit is not None and hit[0] == key:
            proj, grids = hit[1], hit[2]
        else:
            proj = torch.cat([m.projection_mat.reshape(-1) for m in cve]) if len(cve) else torch.zeros(1, device=dev)
            grids = torch.cat([m.grid.reshape(-1) for m in cve]) if len(cve) else torch.zeros(1, device=dev)
            tower._cve_cat = (key, proj, grids)
        total = sum(m.n_proj for m in cve) + (1 if nb else 0)
        emb = torch.empty((n, Dout), dtype=torch.bfloat16, device=dev)
        rows = torch.empty((n, total), dtype=torch.int16, device=dev)
        xn = torch.empty((n, Din), dtype=torch.bfloat16, device=dev)
        mask = torch.empty(n, dtype=torch.uint8, device=dev)
        d = STRUCTS["lthm_ptower_desc"]()
        d.ids, d.x, d.x_dtype, d.Din, d.n, d.Dout = ptr(ids), ptr(x), dcode(x), Din, n, Dout
        d.n_mod = len(cve)
        d.w_map, d.b_map = ptr(w_map.detach()), ptr(b_map.detach()) if b_map is not None else None
        d.proj, d.grids = ptr(proj), ptr(grids)
        d.tables, d.hist, d.tab_dtype = ptr(tab), ptr(tab[R_cve]) if nb else None, dcode(tab)
        d.proj_total, d.grid_total, d.cve_rows, d.norm_bins = proj.numel(), grids.numel(), R_cve, nb
        d.norm_threshold, d.cve_only, d.emb_dtype = float(tower.norm_threshold), 0, dcode(emb)
        ro = po = go = 0
        for j, m in enumerate(cve):
            d.mod_nproj[j], d.mod_nbins[j] = m.n_proj, m.num_bins
            d.mod_row_off[j], d.mod_proj_off[j], d.mod_grid_off[j] = ro, po, go
            ro += (m.num_bins + 1) * m.n_proj
            po += m.projection_mat.numel()
            go += m.grid.numel()
        d.emb_out, d.rows_out, d.xn_out, d.mask_out = ptr(emb), ptr(rows), ptr(xn), ptr(mask)
        call("lthm_product_tower_fwd", ctypes.addressof(d), stream())
        prod = K.linear_fwd(emb, w_pm_b)
        # masked_fill (product_tower.py:58): no gradient reaches a masked token's pre-mask embedding;
        # the backward zeroes those rows of `de` by a gather through this map (-1: zero row)
        keep = torch.where(mask.bool(), torch.full((n,), -1, dtype=torch.int32, device=dev),
                           torch.arange(n, dtype=torch.int32, device=dev))
        ctx.save_for_backward(rows, xn, emb, w_pm_b, keep)
        ctx.meta = (R_cve, nb, [t.shape for t in tables], b_map is not None)
        mods, so = [], 0  # backward layout: per CVE module (slot0, n_proj, row0, nb+1) + the histogram slot
        for j, m in enumerate(cve):
            mods.append((so, m.n_proj, d.mod_row_off[j], m.num_bins + 1))
            so += m.n_proj
        if nb:
            mods.append((so, 1, R_cve, nb))
        ctx.modules = mods
        ctx.mark_non_differentiable(mask)
        if ctx.full is not None:
            shape, n_full, idx, inv = ctx.full
            emb_f = K.rows_gather(emb, inv)
            prod_f = K.rows_gather(prod, inv)
            mask_f = torch.ones(n_full, dtype=torch.uint8, device=dev)
            mask_f.index_copy_(0, idx.long(), mask)
            return emb_f.view(*shape, Dout), prod_f.view(*shape, -1), mask_f.view(shape)
        return emb.view(*ids.shape, Dout), prod.view(*ids.shape, -1), mask.view(ids.shape)

    @staticmethod
    def backward(ctx, d_emb, d_prod, _dmask):
        rows, xn, emb, w_pm_b, keep = ctx.saved_tensors
        R_cve, nb, shapes, has_b = ctx.meta
        Dout = emb.shape[1]
        dpb = d_prod.contiguous().view(-1, d_prod.shape[-1])
        dpb = dpb if dpb.dtype == torch.bfloat16 else K.cast(dpb, torch.bfloat16)
        res = None if d_emb is None else d_emb.contiguous().view(-1, Dout)
        if ctx.full is not None:  # the compact tokens' rows of the upstream gradients
            idx = ctx.full[2]
            dpb = K.rows_gather(dpb, idx)
            if res is not None:
                res = K.rows_gather(res, idx)
        dw_pm = K.linear_wgrad(dpb, emb)
        de = K.linear_dgrad(dpb, w_pm_b, res1=res)  # bf16 total gradient of `emb`
        if Dout % 8 == 0:  # masked tokens: zero (in place: each row reads itself or nothing)
            de = K.rows_gather(de, keep, out=de)
        else:  # rows of a width rows_gather cannot move
            de = de.masked_fill_((keep < 0)[:, None], 0)
        dw_map = K.linear_wgrad(de, xn)
        db_map = K.colsum(de) if has_b else None
        R = R_cve + max(nb, 1)
        if (Dout in (16, 32, 64, 128, 256) or Dout % 256 == 0) and len(ctx.modules) <= 16:
            dtab = K.cve_table_bwd(rows, de, R, ctx.modules)
        else:
            segs = []
            for s0, ns, r0, rps in ctx.modules:
                segs += K.cve_segments(ns, rps, s0, r0)
            dtab = K.segmented_table_bwd(rows, de, R, segs)
        grads, r = [], 0
        for s in shapes:
            grads.append(dtab[r:r + s[0]])
            r += s[0]
        dhist = dtab[R_cve:R_cve + nb] if nb else None
        return (None, None, dw_map, db_map, dw_pm, dhist, None, *grads)


class ProductTower(nn.Module):
    def __init__(self, model_config):
        super().__init__()
        tc = model_config.product_tower
        self.inp_emb_dim, self.out_emb_dim = tc.inp_emb_dim, tc.out_emb_dim
        self.norm_threshold, self.norm_bins = tc.norm_threshold, tc.norm_bins
        self.emb_mapper = nn.Linear(tc.inp_emb_dim, tc.out_emb_dim)
        self.direction_emb = nn.ModuleList([
            CosineVectorEmbedding(tc.inp_emb_dim, tc.out_emb_dim, n_proj=c.num_proj, num_bins=c.num_bins)
            for c in tc.cosine_lsh_config])
        if self.norm_bins > 1:
            self.norm_emb = HistogramEmbedding(0, 1, tc.norm_bins, emb_dim=tc.out_emb_dim)
        self.product_mapper = nn.Linear(tc.out_emb_dim, tc.product_emb_dim, bias=False)

    def forward(self, ids: torch.Tensor, x: torch.Tensor):
        """ids [B, T] int64, x [B, T, inp_emb_dim] (item embedding; detached as in
        product_tower.py:47) -> (emb [B, T, out] bf16, prod_emb [B, T, P_e] bf16, mask [B, T] uint8)."""
        x = x.detach().contiguous()
        hist = self.norm_emb.emb.weight if self.norm_bins > 1 else None
        return ProductTowerFn.apply(ids.contiguous(), x, self.emb_mapper.weight, self.emb_mapper.bias,
                                    self.product_mapper.weight, hist, self,
                                    *[m.emb.weight for m in self.direction_emb])
