"""GPU parity: KShift / Flat gather+pool kernels vs golden vectors and the oracle."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref

pytestmark = pytest.mark.gpu


def test_rows_bit_exact(dev):
    from recommendations_amd import kernels as K
    g = golden("kshift_rows")
    ids = torch.from_numpy(g["ids"]).to(dev)
    for a, P in enumerate(g["Ps"]):
        rows = K.kshift_rows(ids, int(P), 32).cpu().numpy()
        np.testing.assert_array_equal(rows.T, g["rows"][a])


@pytest.mark.parametrize("case", range(6))
def test_kshift_golden(dev, case):
    from recommendations_amd.commons.layers import KShiftEmbedding
    g = golden(f"kshift_fwd_bwd_{case}")
    Kk, norm = int(g["K"]), bool(g["normalize"])
    m = KShiftEmbedding(int(g["P"]), int(g["D"]), num_shifts=Kk, normalize_output=norm).to(dev)
    with torch.no_grad():
        m.emb.weight.copy_(torch.from_numpy(g["weight"]))
    y = m(torch.from_numpy(g["ids"]).to(dev))
    if norm:
        np.testing.assert_allclose(y.detach().cpu().numpy(), g["out"], rtol=1e-6, atol=1e-7)
    else:
        np.testing.assert_array_equal(y.detach().cpu().numpy(), g["out"])   # bit-exact
    (y * torch.from_numpy(g["dy"]).to(dev)).sum().backward()
    np.testing.assert_allclose(m.emb.weight.grad.cpu().numpy(), g["dweight"], rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_flat_golden(dev, seed):
    from recommendations_amd.commons.layers import FlatEmbedding
    g = golden(f"flat_{seed}")
    pad = int(g["padding_idx"])
    m = FlatEmbedding(int(g["P"]), int(g["D"]), padding_idx=None if pad < 0 else pad,
                      normalize_output=bool(g["normalize"])).to(dev)
    with torch.no_grad():
        m._emb_table.weight.copy_(torch.from_numpy(g["weight"]))
    y = m(torch.from_numpy(g["ids"]).to(dev))
    np.testing.assert_allclose(y.detach().cpu().numpy(), g["out"], rtol=1e-6, atol=1e-7)
    (y * torch.from_numpy(g["dy"]).to(dev)).sum().backward()
    np.testing.assert_allclose(m._emb_table.weight.grad.cpu().numpy(), g["dweight"], rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("P,D,Kk,F,wdt", [(1_000_003, 32, 16, 1, torch.float32), (100_000, 32, 8, 4, torch.float32),
                                          (50_000, 128, 8, 1, torch.bfloat16), (4096, 4, 16, 1, torch.float32),
                                          (70_000, 256, 4, 2, torch.float32), (3000, 64, 64, 1, torch.float32)])
def test_kshift_vs_oracle_sizes(dev, P, D, Kk, F, wdt):
    """Larger/odd shapes, table-batched features, bf16 tables (fp32 accumulate)."""
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(P + D)
    n = 20000 // F
    ids = torch.randint(-(2 ** 63), 2 ** 63 - 1, (n, F), generator=g, dtype=torch.int64)
    ids[::7] = 0
    W = torch.randn(F * P, D, generator=g).to(wdt)
    out = K.kshift(ids.to(dev), W.to(dev), P, Kk, K.KSHIFT_SCALE, F=F, out_dtype=torch.float32).cpu()
    Wf = W.float().numpy()
    exp = np.stack([ref.kshift_fwd_c(ids[:, f].numpy(), Wf[f * P:(f + 1) * P], Kk, 0) for f in range(F)], 1)
    np.testing.assert_array_equal(out.numpy(), exp)  # bit-exact (bf16 upcast exact, same order)
    # backward (dense) against the C oracle
    dy = torch.randn(n, F, D, generator=g)
    Wg = W.float().to(dev).requires_grad_(True)
    y = K.kshift(ids.to(dev), Wg, P, Kk, K.KSHIFT_SCALE, F=F)
    y.backward(dy.to(dev))
    dW = Wg.grad.cpu().numpy()
    for f in range(F):
        e = ref.kshift_bwd_c(ids[:, f].numpy(), dy[:, f].numpy(), P, Kk, 0)
        np.testing.assert_allclose(dW[f * P:(f + 1) * P], e, rtol=1e-4, atol=2e-6 * np.abs(e).max() + 1e-5)


@pytest.mark.parametrize("P,D,Kk,F,wdt", [(1_000_003, 32, 16, 1, torch.bfloat16), (200_000, 128, 16, 1, torch.bfloat16),
                                          (60_000, 256, 16, 1, torch.bfloat16), (80_000, 64, 8, 3, torch.bfloat16),
                                          (90_000, 16, 4, 1, torch.float32), (50_001, 64, 16, 2, torch.float32)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_kshift_register_rows_vs_oracle(dev, P, D, Kk, F, wdt, mode):
    """The register-row gather (kshift_fwd_reg_k: 16-B lane vectors, 4 .. 32 lanes per row,
    K 4 / 8 / 16) in every output mode, ragged last wave iteration (n not a multiple of the
    items per iteration), bf16 and f32 outputs: bit-exact to the C oracle in scale / none mode
    (same in-order f32 sum), 1e-6 after the L2 normalisation."""
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(P + D + mode)
    n = 20011 // F
    ids = torch.randint(-(2 ** 63), 2 ** 63 - 1, (n, F), generator=g, dtype=torch.int64)
    ids[::5] = torch.randint(0, 2 ** 62, (len(ids[::5]), F), generator=g, dtype=torch.int64)  # non-negative too
    ids[::7] = 0
    W = torch.randn(F * P, D, generator=g).to(wdt)
    Wf = W.float().numpy()
    exp = np.stack([ref.kshift_fwd_c(ids[:, f].numpy(), Wf[f * P:(f + 1) * P], Kk, mode) for f in range(F)], 1)
    out = K.kshift(ids.to(dev), W.to(dev), P, Kk, mode, F=F, out_dtype=torch.float32).cpu().numpy()
    if mode == 1:
        np.testing.assert_allclose(out, exp, rtol=1e-6, atol=1e-7)
    else:
        np.testing.assert_array_equal(out, exp)
    ob = K.kshift(ids.to(dev), W.to(dev), P, Kk, mode, F=F, out_dtype=torch.bfloat16).float().cpu()
    if mode != 1:
        np.testing.assert_array_equal(ob.numpy(), torch.from_numpy(exp).to(torch.bfloat16).float().numpy())


def test_empty_and_errors(dev):
    from recommendations_amd import kernels as K
    W = torch.randn(10, 8, device=dev)
    out = K.kshift(torch.empty(0, dtype=torch.int64, device=dev), W, 10, 4, K.KSHIFT_SCALE)
    assert out.shape == (0, 8)
    with pytest.raises(RuntimeError):
        K.kshift(torch.zeros(3, dtype=torch.int64, device=dev), W, 10, 65, K.KSHIFT_SCALE)
    with pytest.raises(RuntimeError):
        K.kshift(torch.zeros(3, dtype=torch.int64), W.cpu(), 10, 4, K.KSHIFT_SCALE)


@pytest.mark.parametrize("normalize", [False, True])
def test_row_sharded_single_rank_bit_exact(dev, normalize):
    """RowShardedKShiftEmbedding at world 1 (exchange = local gather) equals KShiftEmbedding bit for bit."""
    from recommendations_amd.commons.layers import KShiftEmbedding, RowShardedKShiftEmbedding
    torch.manual_seed(3)
    full = KShiftEmbedding(50000, 32, num_shifts=16, normalize_output=normalize, out_dtype=torch.float32)
    full.emb.weight.data = full.emb.weight.data.to(torch.bfloat16)
    sh = RowShardedKShiftEmbedding(50000, 32, num_shifts=16, normalize_output=normalize, rank=0, world=1)
    sh.load_full_weight(full.emb.weight.data)
    full, sh = full.to(dev), sh.to(dev)
    ids = torch.randint(-2 ** 63, 2 ** 63 - 1, (4096, 8), dtype=torch.int64).to(dev)
    with torch.no_grad():
        a = full(ids)
        b = sh(ids)
    assert torch.equal(a, b)


@pytest.mark.parametrize("normalize", [False, True])
def test_qr_embedding_vs_oracle(dev, normalize):
    """QREmbedding (commons/layers.py:102-123, constructor and rounding_mode fixed, SURVEY
    §3.5 #5): Wq[(x mod d^2) // d mod d] + Wr[x mod d] (+ L2 normalise) on full-range
    int64 ids, forward and the gradients of both tables vs the torch-CPU oracle."""
    from recommendations_amd.commons.layers import QREmbedding
    torch.manual_seed(5)
    m = QREmbedding(1 << 20, 32, normalize_output=normalize)
    Wq, Wr = m.emb_q.weight.detach().clone(), m.emb_r.weight.detach().clone()
    m = m.to(dev)
    ids = torch.randint(-2 ** 63, 2 ** 63 - 1, (512, 40), dtype=torch.int64)
    ids[:, -5:] = 0
    y = m(ids.to(dev))
    wq, wr = Wq.clone().requires_grad_(True), Wr.clone().requires_grad_(True)
    yr = ref.qr_fwd(ids, wq, wr, normalize)
    if normalize:
        np.testing.assert_allclose(y.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-6, atol=1e-7)
    else:
        assert torch.equal(y.detach().cpu(), yr.detach())
    dy = torch.randn(y.shape)
    (y * dy.to(dev)).sum().backward()
    (yr * dy).sum().backward()
    # f32 scatter-adds in another order: 1e-5 of the largest row gradient
    for got, want in ((m.emb_q.weight.grad, wq.grad), (m.emb_r.weight.grad, wr.grad)):
        np.testing.assert_allclose(got.cpu().numpy(), want.numpy(), rtol=1e-5,
                                   atol=1e-5 * float(want.abs().max()))


@pytest.mark.parametrize("world,P", [(1, 100_000), (3, 1_000_003), (8, 100_000_000)])
def test_shard_route_vs_oracle(dev, world, P):
    """lthm_shard_route (the C3 row-sharded lookup's routing: per-2,048-pair LDS bitonic dedup,
    owner-major layout, device counts) against its CPU restatement oracle.ref.shard_route:
    identical per-owner counts and request multisets, and every (id, shift) pair's position
    pointing at its own KShift row (commons/layers.py:174-185) -- exact.  lthm_shard_gather
    then returns exactly the table rows, bounded by the device-side total."""
    import numpy as np
    from recommendations_amd import kernels as K
    from oracle.ref import kshift_rows, shard_route
    Kk = 16
    g = np.random.default_rng(world)
    ids = np.concatenate([g.integers(-2 ** 63, 2 ** 63 - 1, size=4000, dtype=np.int64),
                          g.integers(0, 50, size=1000, dtype=np.int64)])  # repeats: in-block duplicates
    send, cnt, base, inv = K.shard_route(torch.from_numpy(ids).to(dev), P, Kk, world)
    o_send, o_cnt, o_base, o_inv = shard_route(ids, P, Kk, world)
    assert np.array_equal(cnt.cpu().numpy(), o_cnt) and np.array_equal(base.cpu().numpy(), o_base)
    send_h = send.cpu().numpy()
    assert np.array_equal(send_h[inv.cpu().numpy()], kshift_rows(ids, P, Kk))
    for o in range(world):
        a, b = int(o_base[o]), int(o_base[o + 1])
        assert np.array_equal(np.sort(send_h[a:b]), np.sort(o_send[a:b]))
        assert (send_h[a:b] % world == o).all()
    if world == 1:
        W = torch.randn((P, 32), device=dev).to(torch.bfloat16)
        vals = K.shard_gather(W, send, 1, count=base[1:2])
        n = int(base[1])
        assert torch.equal(vals[:n], W.index_select(0, send[:n]))
