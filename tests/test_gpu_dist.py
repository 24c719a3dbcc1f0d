"""The N > 1 data-parallel path's device side on one GPU: a one-rank RCCL process
group drives the table-wise sharded categorical tables (all_to_all_single of int64
ids, bf16 pooled rows and bf16 gradients) and the backward-overlapped dense
all-reduce through the real kernels.  At world 1 the routing is the identity, so
the sharded module must reproduce the unsharded TableBatchedKShiftEmbedding: forward
rows bit for bit, the row-wise gradient up to the order of its f32 atomics.  The world-2 routing itself is
covered on the CPU by tests/test_dist_gloo.py."""
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture
def rccl1(dev):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    store = dist.TCPStore("127.0.0.1", port, 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        yield
    finally:
        dist.destroy_process_group()


def test_table_sharded_world1_matches_unsharded(dev, rccl1):
    from recommendations_amd.commons.layers import TableBatchedKShiftEmbedding, TableShardedKShiftEmbedding
    torch.manual_seed(0)
    F, P, D, Kk, B = 8, 5000, 32, 8, 512
    full = TableBatchedKShiftEmbedding(F, P, D, Kk, sparse=True, gather_dtype=torch.bfloat16,
                                       out_dtype=torch.bfloat16).to(dev)
    shard = TableShardedKShiftEmbedding(full, 0, 1).to(dev)
    ids = torch.randint(-2 ** 63, 2 ** 63 - 1, (B, F), dtype=torch.int64, device=dev)
    gy = torch.randn(B, F, D, device=dev).to(torch.bfloat16)
    y0, y1 = full(ids), shard(ids)
    assert torch.equal(y0, y1)
    y0.backward(gy)
    y1.backward(gy)
    # same kernel on the same operands; the row sums' f32 atomics may land in another order
    torch.testing.assert_close(shard.sparse_grad, full.sparse_grad, rtol=1e-5, atol=1e-5)
    assert int(full.sparse_count) == int(shard.sparse_count)
    n = int(full.sparse_count)
    assert torch.equal(full.sparse_rows[:n].sort().values, shard.sparse_rows[:n].sort().values)


def test_overlapped_allreduce_world1(dev, rccl1):
    """At world 1 the bucket all-reduce is the identity (no hooks, no launch)."""
    from recommendations_amd.distributed import GradBucketAllReduce
    lin = torch.nn.Linear(64, 64).to(dev)
    ar = GradBucketAllReduce(lin.parameters(), bucket_bytes=1024)
    lin(torch.randn(8, 64, device=dev)).sum().backward()
    g = lin.weight.grad.clone()
    ar()
    assert torch.equal(g, lin.weight.grad)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_full_step_world2_matches_world1(dev, tmp_path):
    """The whole data-parallel training step at world 2 (both ranks on this box's one GPU,
    gloo over CUDA tensors; tests/dist_step_worker.py): table-sharded categorical tables
    (all_to_all of ids, pooled rows and gradients), the row-sharded item table (device
    routing, count exchange, two all_to_alls), the bucketed dense all-reduce launched from
    the backward's gradient hooks, sparse row-wise and dense AdamW, activation
    checkpointing.  Each rank holds half of a 64-sequence batch (one loss mini-batch), so
    the rank-averaged loss and every update equal a world-1 step on the whole batch (two
    mini-batches, loss averaged over them): losses of three steps to 1e-4, dense weight
    updates to 1e-2 (relative Frobenius), the categorical tables after them to 1e-3."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    worker = os.path.join(root, "tests", "dist_step_worker.py")
    prefix = str(tmp_path / "step")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    steps = "3"
    subprocess.run([sys.executable, worker, prefix, steps], env=env, check=True, timeout=300)
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                    "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), worker, prefix, steps],
                   env=env, check=True, timeout=300)
    w1 = torch.load(prefix + "_w1_r0.pt", weights_only=True)
    w2 = [torch.load(prefix + f"_w2_r{r}.pt", weights_only=True) for r in range(2)]
    torch.testing.assert_close(w2[0]["losses"], w1["losses"], rtol=1e-4, atol=0)
    assert torch.equal(w2[0]["losses"], w2[1]["losses"])
    for k, v in w1.items():
        if not k.startswith("dense."):
            continue
        assert torch.equal(w2[0][k], w2[1][k]), f"replicas diverged: {k}"
        # k holds the update over the steps; AdamW's first steps move an element by about
        # lr * sign(g), so a gradient within rounding of 0 may step either way: the update
        # is compared in relative Frobenius norm
        err = float((w2[0][k] - v).norm() / v.norm().clamp_min(1e-12))
        assert err <= 1e-2, (k, err)
    P = w1["tables"].shape[0] // 2
    for r in range(2):
        f0 = int(w2[r]["tables_f0"])
        ref_rows = w1["tables"][f0 * P:f0 * P + w2[r]["tables"].shape[0]]
        err = float((w2[r]["tables"] - ref_rows).abs().max())
        assert err <= 1e-3, (r, err)
