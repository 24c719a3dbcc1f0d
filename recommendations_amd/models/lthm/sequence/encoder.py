"""Encoder — drop-in for models/lthm/sequence/encoder.py:18-61.

``product_emb_module`` is the item KShiftEmbedding (encoder.py:32-37; bf16
table, normalised output, forward-only because product_tower.py:47 detaches
it).  The history is flipped to left padding first (encoder.py:52-54) —
equivalent to the reference's flip after the per-token product tower.
``user_context`` (build-defined, BASELINE C2-C4 categorical features):
table-batched KShift lookups -> cap_gradients -> MLP(QuickGELU) -> CLS token.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn

from .... import kernels as K
from ....distributed import world_size
from ....commons.functional import cap_gradients
from ....commons.layers import (KShiftEmbedding, MLP, RowShardedKShiftEmbedding, TableBatchedKShiftEmbedding,
                                TableShardedKShiftEmbedding)
from .item_artifact import load_item_artifact
from .product_tower import ProductTower
from .query_tower import QueryTower


class UserContext(nn.Module):
    def __init__(self, cfg, d_model: int):
        super().__init__()
        self.tables = TableBatchedKShiftEmbedding(cfg.n_features, cfg.vocab_size, cfg.emb_dim, cfg.num_shifts,
                                                  normalize_output=False, sparse=True,
                                                  gather_dtype=torch.bfloat16 if cfg.gather_bf16 else torch.float32,
                                                  out_dtype=torch.bfloat16)
        with torch.no_grad():
            self.tables.weight.normal_(0.0, 1.0)
        self.mlp = MLP(cfg.n_features * cfg.emb_dim, d_model, cfg.gate_sizes)

    def shard_tables(self, rank: int, world: int) -> None:
        """Data-parallel training over ``world`` ranks: keep only this rank's tables
        (table-wise sharding, commons.layers.TableShardedKShiftEmbedding).  Call before
        the optimizers are built; the replicas must hold identical tables on entry."""
        if world > 1 and not isinstance(self.tables, TableShardedKShiftEmbedding):
            self.tables = TableShardedKShiftEmbedding(self.tables, rank, world)

    def forward(self, cat_ids: torch.Tensor) -> torch.Tensor:
        B = cat_ids.shape[0]
        e = self.tables(cat_ids)                       # [B, F, Dc] bf16
        e = cap_gradients(e.view(B, -1))               # commons/functional.py:28
        return self.mlp(e)                             # [B, d] f32


class Encoder(nn.Module):
    def __init__(self, model_config):
        super().__init__()
        pt = model_config.product_tower
        lm = pt.latent_model_config
        # fp32 output: the CVE bucketize downstream is discontinuous, a bf16-rounded
        # input would flip ~1% of the bucket decisions relative to the reference
        if pt.model_init_metadata is not None:
            # encoder.py:25-29: a pre-trained item-embedding artifact replaces the KShift
            # table (local safetensors file; the S3 fetch is out of scope)
            md = pt.model_init_metadata
            path = md["embedding_module_path"] if isinstance(md, dict) else md.embedding_module_path
            self.product_emb_module = load_item_artifact(
                path, table_dtype=torch.bfloat16 if model_config.item_table_bf16 else None)
        elif model_config.item_table_sharded:
            self.product_emb_module = RowShardedKShiftEmbedding(
                lm.vocab_size_latent, pt.inp_emb_dim, num_shifts=lm.num_shifts_latent,
                normalize_output=lm.normalize_embedding,
                dtype=torch.bfloat16 if model_config.item_table_bf16 else torch.float32, out_dtype=torch.float32)
        else:
            self.product_emb_module = KShiftEmbedding(lm.vocab_size_latent, pt.inp_emb_dim,
                                                      num_shifts=lm.num_shifts_latent,
                                                      normalize_output=lm.normalize_embedding, out_dtype=torch.float32)
            if model_config.item_table_bf16:
                self.product_emb_module.emb.weight.data = self.product_emb_module.emb.weight.data.to(torch.bfloat16)
            self.product_emb_module.emb.weight.requires_grad_(False)  # detached by product_tower.py:47
        self.product_tower = ProductTower(model_config)
        self.query_tower = QueryTower(model_config)
        self.user_context = UserContext(model_config.categorical, model_config.emb_dim) \
            if model_config.categorical.n_features > 0 else None

    @torch.no_grad()
    def prefetch(self, batch: Dict[str, torch.Tensor], ready: Optional["torch.cuda.Event"] = None) -> None:
        """Pipelined item lookup for a later ``forward(batch)`` (the same
        ``batch["product_ids"]`` tensor, unmodified): the item table is frozen
        (product_tower.py:47), so the whole lookup -- for the row-sharded table (C3) the
        routing, the count exchange the host reads and both all_to_alls (on a communicator
        of their own, distributed.row_exchange_group) -- runs on a side stream of the device.
        ``ready`` marks when the ids are valid (default: everything issued so far on the
        current stream).  At world > 1 the call blocks the host until the count exchange
        has landed, so issue it once the current step's backward has been enqueued (with
        ``ready`` recorded when the next batch landed): the host's wait then overlaps the
        queued backward.  Every rank must issue it at the same program point (collective
        order)."""
        raw = batch["product_ids"]
        K.require_gpu(raw)
        side = _side_stream(raw.device)
        if ready is None:
            ready = torch.cuda.Event()
            ready.record()
        side.wait_event(ready)
        with torch.cuda.stream(side):
            ids = K.flip_tokens(raw.contiguous())
            embs = self.product_emb_module(ids)
            done = torch.cuda.Event()
            done.record(side)
        self._prefetched = (raw, raw._version, ids, embs, done)

    def _item_lookup(self, raw: torch.Tensor):
        p = getattr(self, "_prefetched", None)
        if p is not None:
            self._prefetched = None
            if p[0] is raw and p[1] == raw._version:
                _, _, ids, embs, done = p
                cur = torch.cuda.current_stream(raw.device)
                cur.wait_event(done)
                ids.record_stream(cur)
                embs.record_stream(cur)
                return ids, embs
            if isinstance(self.product_emb_module, RowShardedKShiftEmbedding) and world_size() > 1:
                # the inline lookup's collectives would run on this rank alone if another rank's
                # prefetch hit: refuse instead of hanging the group
                raise RuntimeError("a prefetched item lookup does not match this forward's ids; with a "
                                   "row-sharded item table every rank must consume its prefetch")
        ids = K.flip_tokens(raw.contiguous())
        with torch.no_grad():
            embs = self.product_emb_module(ids)
        return ids, embs

    def forward(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        ids, embs = self._item_lookup(batch["product_ids"])
        labels = K.flip_tokens(batch["labels"].contiguous())
        ts = K.flip_tokens(batch["timestamp"].contiguous())
        inp, target, mask = self.product_tower(ids, embs)
        ctx = self.user_context(batch["categorical_ids"]) if self.user_context is not None else None
        return self.query_tower(inp, target, mask, labels, ts, ids, ctx)


_SIDE_STREAMS: Dict[torch.device, "torch.cuda.Stream"] = {}


def _side_stream(dev: torch.device) -> "torch.cuda.Stream":
    s = _SIDE_STREAMS.get(dev)
    if s is None:
        s = torch.cuda.Stream(device=dev)
        _SIDE_STREAMS[dev] = s
    return s

