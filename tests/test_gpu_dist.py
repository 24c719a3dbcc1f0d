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
