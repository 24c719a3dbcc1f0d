"""Multi-process (world_size 2, gloo on CPU) tests of the N > 1 path's host logic:
the bucketed dense all-reduce, the replicated-table sparse-gradient gather, and
the folded stop/NaN flag (recommendations_amd/distributed.py).  The GPU kernels
themselves are covered by the -m gpu tests; here the row update is applied with
the C oracle (oracle/kshift_ref.c), so the test checks that every replica ends
with the same table and that it equals the single-process update of the
rank-averaged loss."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from recommendations_amd.distributed import init_from_env
        r, _, w = init_from_env(backend="gloo")
        assert (r, w) == (rank, world)
        q.put((rank, fn(rank, world)))
    except Exception as e:  # surfaced by the parent
        q.put((rank, e))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _spawn_once(fn, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    return res


def spawn(fn, world=2):
    # the free port is only probed, not held: another process can take it before the
    # rendezvous binds it, so an address-in-use rendezvous failure is retried once
    for attempt in range(2):
        res = _spawn_once(fn, world)
        errs = [v for v in res.values() if isinstance(v, Exception)]
        if attempt == 0 and errs and any("address already in use" in str(e).lower() or "eaddrinuse" in str(e).lower()
                                         for e in errs):
            continue
        for e in errs:
            raise e
        return [res[r] for r in range(world)]


def _bucket_allreduce(rank, world):
    from recommendations_amd.distributed import GradBucketAllReduce
    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.zeros(s)) for s in [(3, 5), (7,), (64, 33), (1,)]]
    for i, p in enumerate(params):
        p.grad = torch.full(p.shape, float(rank + 1) * (i + 1))
    GradBucketAllReduce(params, bucket_bytes=256)()  # tiny buckets: several flushes
    return [p.grad.clone() for p in params]


def test_grad_bucket_allreduce_averages():
    out = spawn(_bucket_allreduce)
    for i, (a, b) in enumerate(zip(*out)):
        assert torch.equal(a, b)
        assert torch.allclose(a, torch.full(a.shape, 1.5 * (i + 1)))


def _gather_sparse(rank, world):
    from recommendations_amd.distributed import gather_sparse_grads
    from oracle.ref import kshift_bwd_c
    g = np.random.default_rng(100 + rank)
    ids = torch.from_numpy(g.integers(-2**63, 2**63 - 1, size=(64, 3), dtype=np.int64))
    gy = torch.from_numpy(g.standard_normal((64, 3, 8)).astype(np.float32))
    ids_all, gy_all, _, _ = gather_sparse_grads(ids, gy)
    # every replica applies every rank's pairs (table-batched layout: F = 3 blocks of P rows)
    P, K, F = 50, 4, 3
    dW = np.zeros((F * P, 8), np.float32)
    rows_ids = ids_all.numpy()
    for f in range(F):
        dW[f * P:(f + 1) * P] += kshift_bwd_c(rows_ids[:, f].copy(), gy_all[:, f].numpy().copy(), P, K, 0)
    return ids, gy, dW


def test_replicated_sparse_update_matches_single_process():
    from oracle.ref import kshift_bwd_c
    (i0, g0, w0), (i1, g1, w1) = spawn(_gather_sparse)
    assert np.array_equal(w0, w1)  # replicas stay identical
    P, K, F = 50, 4, 3
    ids = torch.cat([i0, i1]).numpy()
    gy = (torch.cat([g0, g1]) / 2).numpy()  # gradient of the rank-averaged loss
    ref = np.zeros_like(w0)
    for f in range(F):
        ref[f * P:(f + 1) * P] += kshift_bwd_c(ids[:, f].copy(), gy[:, f].copy(), P, K, 0)
    np.testing.assert_allclose(w0, ref, rtol=1e-6, atol=1e-6)


def _flags(rank, world):
    from recommendations_amd.distributed import step_flags
    a = step_flags(rank == 1, torch.tensor(1.0))
    b = step_flags(False, torch.tensor(float("nan")) if rank == 0 else torch.tensor(2.0))
    c = step_flags(False, torch.tensor(3.0))
    return a, b, c


def test_step_flags_fold_stop_and_nan():
    for a, b, c in spawn(_flags):
        assert a.tolist() == [1.0, 0.0]
        assert b.tolist() == [0.0, 1.0]
        assert c.tolist() == [0.0, 0.0]


def _gather_rows(rank, world):
    from recommendations_amd.distributed import all_gather_rows
    return all_gather_rows(torch.arange(6).view(3, 2) + 100 * rank)


def test_all_gather_rows_rank_order():
    for out in spawn(_gather_rows):
        assert torch.equal(out, torch.cat([torch.arange(6).view(3, 2), torch.arange(6).view(3, 2) + 100]))


def _sharded_lookup(rank, world):
    """Row-sharded table (r on rank r % world): every rank exchanges its own
    deduplicated KShift rows and gets exactly the full table's rows back."""
    from recommendations_amd.distributed import exchange_rows
    from oracle.ref import kshift_rows, kshift_fwd_c
    P, D, Kk = 1000, 8, 16
    W = torch.from_numpy(np.random.default_rng(5).standard_normal((P, D)).astype(np.float32))
    shard = W[rank::world].contiguous()
    g = np.random.default_rng(40 + rank)
    ids = g.integers(-2**63, 2**63 - 1, size=300 + 50 * rank, dtype=np.int64)
    rows = torch.from_numpy(kshift_rows(ids, P, Kk))
    uniq, inv = torch.unique(rows.view(-1), return_inverse=True)
    vals = exchange_rows(uniq, shard)
    exact = torch.equal(vals, W.index_select(0, uniq))
    # in-order pool of the exchanged rows == the unsharded gather (oracle)
    pooled = vals[inv.view(-1, Kk)].sum(dim=1)
    ref = torch.from_numpy(kshift_fwd_c(ids, W.numpy(), Kk, 2))
    return exact, float((pooled - ref).abs().max())


def test_row_sharded_exchange():
    for exact, err in spawn(_sharded_lookup):
        assert exact
        assert err < 1e-5
