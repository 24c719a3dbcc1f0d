"""Multi-process (world_size 2, gloo on CPU) tests of the N > 1 path's host logic:
the bucketed dense all-reduce, the replicated-table sparse-gradient gather, and
the folded stop/NaN flag (recommendations_amd/distributed.py).  The GPU kernels
themselves are covered by the -m gpu tests; here the row update is applied with
the C oracle (oracle/kshift_ref.c), so the test checks that every replica ends
with the same table and that it equals the single-process update of the
rank-averaged loss."""
import math
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


class _Tensor:
    """A result tensor sent back as a plain array: torch's fd-sharing of tensors through
    a Queue needs the sending child alive until the parent has received, which it is not."""

    def __init__(self, t):
        self.a = t.detach().cpu().numpy().copy()


def _pack(v):
    if isinstance(v, torch.Tensor):
        return _Tensor(v)
    if isinstance(v, (list, tuple)):
        return type(v)(_pack(x) for x in v)
    if isinstance(v, dict):
        return {k: _pack(x) for k, x in v.items()}
    return v


def _unpack(v):
    if isinstance(v, _Tensor):
        return torch.from_numpy(v.a)
    if isinstance(v, (list, tuple)):
        return type(v)(_unpack(x) for x in v)
    if isinstance(v, dict):
        return {k: _unpack(x) for k, x in v.items()}
    return v


def _run(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from recommendations_amd.distributed import init_from_env
        r, _, w = init_from_env(backend="gloo")
        assert (r, w) == (rank, world)
        q.put((rank, _pack(fn(rank, world))))
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
    res = {r: _unpack(v) for r, v in (q.get(timeout=120) for _ in procs)}
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


def _bucket_allreduce_overlapped(rank, world):
    """Real backward: the post-accumulate hooks launch each bucket's all-reduce during
    the backward; the result equals the rank-averaged gradient."""
    from recommendations_amd.distributed import GradBucketAllReduce
    torch.manual_seed(0)  # identical replicas
    net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 32), torch.nn.Tanh(),
                              torch.nn.Linear(32, 4))
    ar = GradBucketAllReduce(net.parameters(), bucket_bytes=1024)  # several buckets
    launched = []
    for step in range(2):
        x = torch.randn(8, 16, generator=torch.Generator().manual_seed(10 * step + rank))
        net.zero_grad(set_to_none=True)
        net(x).square().mean().backward()
        launched.append(sum(w is not None for w in ar._work))
        ar()
    grads = [p.grad.clone() for p in net.parameters()]
    # single-process reference of the last step: mean over both ranks' losses
    ref = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 32), torch.nn.Tanh(),
                              torch.nn.Linear(32, 4))
    ref.load_state_dict(net.state_dict())
    loss = sum(ref(torch.randn(8, 16, generator=torch.Generator().manual_seed(10 + r))).square().mean()
               for r in range(world)) / world
    loss.backward()
    return grads, [p.grad for p in ref.parameters()], launched, len(ar.buckets)


def test_grad_bucket_allreduce_overlaps_backward():
    for grads, ref, launched, nb in spawn(_bucket_allreduce_overlapped):
        assert nb > 1 and launched == [nb, nb]  # every bucket launched from the backward's hooks
        for g, r in zip(grads, ref):
            torch.testing.assert_close(g, r, rtol=1e-5, atol=1e-6)


def _bucket_allreduce_accumulate(rank, world):
    """Two micro-batch backward passes before ar(): with the first inside no_sync (the
    DDP pattern) and without it (hooks fire twice; the stale launch is redone)."""
    from recommendations_amd.distributed import GradBucketAllReduce
    out = []
    for use_no_sync in (True, False):
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 4))
        ar = GradBucketAllReduce(net.parameters(), bucket_bytes=512)
        for step in range(2):  # the second step checks that state was reset
            net.zero_grad(set_to_none=True)
            xs = [torch.randn(8, 16, generator=torch.Generator().manual_seed(100 * step + 10 * mb + rank))
                  for mb in range(2)]
            if use_no_sync:
                with ar.no_sync():
                    net(xs[0]).square().mean().backward()
            else:
                net(xs[0]).square().mean().backward()
            net(xs[1]).square().mean().backward()
            ar()
        ref = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 4))
        ref.load_state_dict(net.state_dict())
        loss = sum(ref(torch.randn(8, 16, generator=torch.Generator().manual_seed(100 + 10 * mb + r))).square().mean()
                   for r in range(world) for mb in range(2)) / world
        loss.backward()
        out.append(([p.grad.clone() for p in net.parameters()], [p.grad for p in ref.parameters()]))
    return out


def test_grad_bucket_allreduce_gradient_accumulation():
    for per_rank in spawn(_bucket_allreduce_accumulate):
        for grads, ref in per_rank:
            for g, r in zip(grads, ref):
                torch.testing.assert_close(g, r, rtol=1e-5, atol=1e-6)


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


def _oracle_shard_kernels():
    """The two routing kernels of the row-sharded lookup (lthm_shard_route / lthm_shard_gather)
    replaced by their CPU restatements (oracle.ref.shard_route, an index_select)."""
    import recommendations_amd.kernels as K_
    from oracle.ref import shard_route

    def route(ids, P, K, world):
        send, cnt, base, inv = shard_route(ids.numpy(), P, K, world)
        return (torch.from_numpy(send), torch.from_numpy(cnt), torch.from_numpy(base),
                torch.from_numpy(inv).view(-1, K))

    def gather(shard, rows, world, count=None):
        n = rows.numel() if count is None else int(count.reshape(-1)[0])
        return shard.index_select(0, torch.div(rows[:n], world, rounding_mode="floor"))

    K_.shard_route, K_.shard_gather = route, gather


def _sharded_lookup(rank, world):
    """Row-sharded table (r on rank r % world): every rank exchanges its own routed KShift
    rows (per-block dedup, owner-major) and gets exactly the full table's rows back."""
    import recommendations_amd.kernels as K_
    from recommendations_amd.distributed import exchange_routed
    from oracle.ref import kshift_fwd_c, kshift_rows
    _oracle_shard_kernels()
    P, D, Kk = 1000, 8, 16
    W = torch.from_numpy(np.random.default_rng(5).standard_normal((P, D)).astype(np.float32))
    shard = W[rank::world].contiguous()
    g = np.random.default_rng(40 + rank)
    ids = torch.from_numpy(g.integers(-2**63, 2**63 - 1, size=300 + 50 * rank, dtype=np.int64))
    send, cnt, base, inv = K_.shard_route(ids, P, Kk, world)
    vals = exchange_routed(send, cnt, base, shard)
    exact = torch.equal(vals, W.index_select(0, send[:int(base[-1])]))
    rows = torch.from_numpy(kshift_rows(ids.numpy(), P, Kk))
    routed = torch.equal(send[inv], rows)
    # in-order pool of the exchanged rows == the unsharded gather (oracle)
    pooled = vals[inv].sum(dim=1)
    ref = torch.from_numpy(kshift_fwd_c(ids.numpy(), W.numpy(), Kk, 2))
    return exact and routed, float((pooled - ref).abs().max())


def test_row_sharded_exchange():
    for exact, err in spawn(_sharded_lookup):
        assert exact
        assert err < 1e-5


def _oracle_local_kernels(record):
    """CPU stand-ins for the two HIP calls of the table-sharded module (the routing is
    what the gloo tests check; the kernels have their own -m gpu parity tests)."""
    from oracle.ref import kshift_bwd_c, kshift_fwd_c

    def fwd(mod, ids, gather_w):
        P, Kk, Fl = mod._num_embeddings, mod._num_shifts, mod._F
        Wn = gather_w.detach().float().numpy()
        outs = [kshift_fwd_c(ids[:, f].numpy(), Wn[f * P:(f + 1) * P], Kk, mod._mode) for f in range(Fl)]
        return torch.from_numpy(np.stack(outs, axis=1)), None

    def bwd(mod, ids, gy, out, norms):
        P, Kk, Fl = mod._num_embeddings, mod._num_shifts, mod._F
        g = np.concatenate([kshift_bwd_c(ids[:, f].numpy(), gy[:, f].float().numpy(), P, Kk, mod._mode)
                            for f in range(Fl)])
        record.append(g)

    return fwd, bwd


def _table_sharded(rank, world):
    """TableShardedKShiftEmbedding at world 2: every rank's forward equals the unsharded
    lookup of its own ids, and each owner receives exactly the rank-averaged gradient
    of its tables."""
    import recommendations_amd.commons.layers as L
    from oracle.ref import kshift_fwd_c
    F, P, D, Kk, B = 5, 40, 8, 4, 6  # 5 tables over 2 ranks: owners hold 2 and 3
    Wfull = torch.from_numpy(np.random.default_rng(3).standard_normal((F * P, D)).astype(np.float32))
    full = L.TableBatchedKShiftEmbedding(F, P, D, Kk, sparse=True, out_dtype=torch.float32)
    with torch.no_grad():
        full.weight.copy_(Wfull)
    record = []
    L._kshift_fwd_local, L._kshift_bwd_local = _oracle_local_kernels(record)
    mod = L.TableShardedKShiftEmbedding(full, rank, world)
    g = np.random.default_rng(50 + rank)
    ids = torch.from_numpy(g.integers(-2**63, 2**63 - 1, size=(B, F), dtype=np.int64))
    gy = torch.from_numpy(g.standard_normal((B, F, D)).astype(np.float32))
    out = mod(ids)
    exp = np.stack([kshift_fwd_c(ids[:, f].numpy(), Wfull[f * P:(f + 1) * P].numpy(), Kk, 0) for f in range(F)], 1)
    out.backward(gy)
    return (float(np.abs(out.detach().numpy() - exp).max()), ids, gy, record[0], mod._bounds,
            torch.equal(mod.weight.detach(), Wfull[mod._bounds[rank] * P:mod._bounds[rank + 1] * P]))


def test_table_sharded_routing_world2():
    from oracle.ref import kshift_bwd_c
    res = spawn(_table_sharded)
    F, P, Kk = 5, 40, 4
    ids_all = [r[1] for r in res]
    gy_all = [r[2] for r in res]
    for rank, (err, _, _, grad, bounds, own_ok) in enumerate(res):
        assert err == 0.0 and own_ok
        f0, f1 = bounds[rank], bounds[rank + 1]
        exp = np.concatenate([sum(kshift_bwd_c(i[:, f].numpy(), g[:, f].numpy(), P, Kk, 0) for i, g in
                                  zip(ids_all, gy_all)) / 2 for f in range(f0, f1)])
        np.testing.assert_allclose(grad, exp, rtol=1e-5, atol=1e-6)


def _row_sharded_module(rank, world):
    """RowShardedKShiftEmbedding (C3 item table) itself at world 2, its routing, gather and
    pool kernels replaced by the oracle: bit-identical to the unsharded gather of the same ids."""
    import recommendations_amd.kernels as K_
    import recommendations_amd.commons.layers as L
    from oracle.ref import kshift_fwd_c
    P, D, Kk = 1000, 8, 16
    _oracle_shard_kernels()

    def pool(rows, vals, mode, out_dtype=torch.float32):
        acc = torch.zeros(rows.shape[0], vals.shape[1], dtype=torch.float32)
        for c in range(rows.shape[1]):  # in-order f32 sum, as lthm_gather_pool
            acc += vals[rows[:, c]].float()
        return acc / math.sqrt(rows.shape[1]) if mode == K_.KSHIFT_SCALE else acc

    K_.gather_pool = pool
    Wfull = torch.from_numpy(np.random.default_rng(9).standard_normal((P, D)).astype(np.float32))
    mod = L.RowShardedKShiftEmbedding(P, D, num_shifts=Kk, rank=rank, world=world, dtype=torch.float32)
    mod.load_full_weight(Wfull)
    ids = torch.from_numpy(np.random.default_rng(70 + rank).integers(-2**63, 2**63 - 1, size=(50 + 7 * rank, 3),
                                                                     dtype=np.int64))
    out = mod(ids)
    exp = kshift_fwd_c(ids.numpy(), Wfull.numpy(), Kk, 0).reshape(out.shape)
    return float(np.abs(out.numpy() - exp).max())


def test_row_sharded_module_world2():
    for err in spawn(_row_sharded_module):
        assert err < 1e-5
