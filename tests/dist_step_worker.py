"""Worker for tests/test_gpu_dist.py::test_full_step_world2_matches_world1: the full LTHM
training step (table-sharded categorical tables, row-sharded item table, bucketed dense
all-reduce overlapped with the backward, row-wise sparse and dense AdamW, activation
checkpointing) through the HIP kernels, at world 1 on a 64-sequence batch or at world 2
with each rank holding one 32-sequence half of it.  Both ranks of a world-2 run share
cuda:0 of the one-GPU box over a gloo process group (CUDA tensors: gloo stages them
through the host); the collective calls are the ones the bench makes over RCCL.

Usage (env from torch.distributed.run, or WORLD_SIZE unset for world 1):
    python tests/dist_step_worker.py OUT_PREFIX STEPS
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

B_RANK, T, N_CAT = 32, 32, 2
OFFSETS = [0, 3, 6, 9, 17, 25]


def main():
    out_prefix, steps = sys.argv[1], int(sys.argv[2])
    from recommendations_amd.data import synthetic_lthm_batch
    from recommendations_amd.distributed import GradBucketAllReduce, init_from_env
    from recommendations_amd.models.lthm.builder import LTHMModelBuilder
    from recommendations_amd.models.lthm.config import lthm_config

    rank, _, world = init_from_env(backend="gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(1234)  # identical replicas
    cfg = lthm_config(T=T, d=64, n_layers=1, n_head=1, cat_features=N_CAT, cat_vocab=1000, item_vocab=1000,
                      item_table_sharded=True, train_mini_batch_size=32)
    model = LTHMModelBuilder(None, cfg).build().to(dev)
    enc = model._model
    full_item = torch.randn(1000, 32, generator=torch.Generator().manual_seed(7))
    enc.product_emb_module.load_full_weight(full_item.to(dev))
    if world > 1:
        enc.user_context.shard_tables(rank, world)
    opts = model.optimizers_for_param_groups(model.param_groups())
    dense = [(n, p) for n, p in model.named_parameters() if p.requires_grad and not model.is_sparse(n)]
    allreduce = GradBucketAllReduce([p for _, p in dense], bucket_bytes=1 << 16)
    # the same lookahead offsets for every mini-batch, so world 1 (two mini-batches) and
    # each world-2 rank (one) draw the same ones
    model.draw_offsets = lambda n_mb: np.array([OFFSETS] * n_mb, dtype=np.int32)

    full = synthetic_lthm_batch(B_RANK * 2, T, n_cat=N_CAT, seed=5)
    # the query tower trims the history to the batch's longest sequence (the reference's
    # trim): one full-length sequence in each half keeps both ranks at the world-1 length
    longest = synthetic_lthm_batch(2, T, n_cat=N_CAT, seed=6, min_len=T)
    for k in full:
        full[k][0::B_RANK] = longest[k]
    lo, hi = (0, 2 * B_RANK) if world == 1 else (rank * B_RANK, (rank + 1) * B_RANK)
    batch = {k: v[lo:hi].contiguous().to(dev) for k, v in full.items()}
    init = {n: p.detach().float().cpu().clone() for n, p in dense}
    losses = []
    for _ in range(steps):
        out = model(batch)
        loss, _ = model.train_step(batch, out)
        loss.backward()
        allreduce()
        for o in opts:
            o.step()
            o.zero_grad(set_to_none=True)
        lt = loss.detach().float().reshape(1).clone()
        if world > 1:
            torch.distributed.all_reduce(lt)
            lt /= world
        losses.append(float(lt))
    torch.cuda.synchronize()
    if rank == 0:
        print(f"world {world} losses {losses}", flush=True)
    res = {"losses": torch.tensor(losses, dtype=torch.float64)}
    for n, p in dense:
        res["dense." + n] = p.detach().float().cpu() - init[n]  # the update over the steps
    tabs = enc.user_context.tables
    w = tabs.weight.detach().float().cpu()
    if world > 1:  # this rank's tables [f0, f1) of the full stack
        f0 = tabs._bounds[rank]
        res["tables_f0"] = torch.tensor(f0)
    res["tables"] = w
    torch.save(res, f"{out_prefix}_w{world}_r{rank}.pt")
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
