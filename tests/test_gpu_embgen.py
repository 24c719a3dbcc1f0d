"""GPU parity of the item-embedding generation loops (embedding_module_gen.py:
70-156) against a torch-CPU restatement: KShift gather/pool from the oracle
(oracle/ref.py), torch MSE / BCE-with-logits and torch.optim.Adagrad over the
whole (dense) table.  The GPU path updates only touched rows, which for
Adagrad (no decay) is the same update.  Tolerances: fp32 summation order for
the reconstruction model (relative Frobenius 1e-5 on the trained table); the
mask model's MLP runs on bf16 MFMA operands (1e-2, at lr 0.05)."""
import numpy as np
import pandas as pd
import pytest
import torch

from parity import check, relerr
import torch.nn.functional as F

from oracle import ref

pytestmark = pytest.mark.gpu




def _df(n, D, seed=0):
    g = np.random.default_rng(seed)
    return pd.DataFrame({"product_id": [str(i * 7919 + 13) for i in range(n)],
                         "embedding": list(g.standard_normal((n, D)).astype(np.float32))})


@pytest.mark.parametrize("fused", [True, False])  # lthm_kshift_adagrad_fused / the two-pass row path
def test_train_model_matches_dense_adagrad(dev, fused, monkeypatch):
    from recommendations_amd import embedding_module_gen
    from recommendations_amd.embedding_module_gen import massage_embeddings, train_model
    monkeypatch.setattr(embedding_module_gen, "_FUSED", fused)
    df = massage_embeddings(_df(3000, 32))
    torch.manual_seed(5)
    m = train_model(df, 1.15, 16, num_epochs=2, batch_size=1024, device=dev, seed=1, log=None)
    torch.manual_seed(5)
    W = torch.nn.Embedding(int(1.15 * 3000), 32).weight.detach().clone().requires_grad_(True)
    opt = torch.optim.Adagrad([W], lr=0.5)
    ids = torch.from_numpy(np.asarray(df["product_id"].values, dtype=np.int64))
    x = F.normalize(torch.from_numpy(np.stack(df["embedding"].values)), p=2.0, dim=-1)
    rng = np.random.default_rng(1)
    for _ in range(2):
        idx = np.arange(3000)
        rng.shuffle(idx)
        for b in range(0, 3000, 1024):
            it = torch.from_numpy(idx[b:b + 1024])
            y = ref.kshift_fwd_torch(ids[it], W, 16, True)
            F.mse_loss(y, x[it]).backward()
            opt.step()
            opt.zero_grad()
    check('m.emb.weight, W', relerr(m.emb.weight, W), 1e-5)


@pytest.mark.parametrize("fused", [True, False])
def test_train_mask_model_matches_dense_adagrad(dev, fused, monkeypatch):
    from recommendations_amd import embedding_module_gen
    from recommendations_amd.embedding_module_gen import massage_embeddings, train_mask_model
    monkeypatch.setattr(embedding_module_gen, "_FUSED", fused)
    df = massage_embeddings(_df(2000, 8, seed=3))
    negs = np.random.default_rng(9).integers(-2 ** 63, 2 ** 63 - 1, size=(8, 1000), dtype=np.int64)
    calls = {"i": 0}

    def negatives(k):
        v = torch.from_numpy(negs[calls["i"], :k].copy())
        calls["i"] += 1
        return v

    torch.manual_seed(11)
    # lr 0.05: at the reference's 0.5 every Adagrad step moves each weight by ~0.5 (MLP included),
    # which amplifies the bf16-level MLP gradient differences (~3e-3, tools/maskgrad_check.py) step by step
    model = train_mask_model(df, 1.15, 16, 4, num_epochs=2, batch_size=1000, device=dev, seed=2, log=None,
                             negatives=negatives, lr=0.05)
    torch.manual_seed(11)
    from recommendations_amd.commons.layers import MLP, KShiftEmbedding
    emb_c = KShiftEmbedding(int(1.15 * 2000), 4, num_shifts=16)
    mlp_c = MLP(4, 1, [64])
    W = emb_c.emb.weight.detach().clone().requires_grad_(True)
    lins = [l for l in mlp_c.model if isinstance(l, torch.nn.Linear)]
    ws = [l.weight.detach().clone().requires_grad_(True) for l in lins]
    bs = [l.bias.detach().clone().requires_grad_(True) for l in lins]
    opt = torch.optim.Adagrad([W] + ws + bs, lr=0.05)
    ids = torch.from_numpy(np.asarray(df["product_id"].values, dtype=np.int64))
    rng = np.random.default_rng(2)
    i = 0
    for _ in range(2):
        idx = np.arange(2000)
        rng.shuffle(idx)
        for b in range(0, 2000, 1000):
            pos = ids[torch.from_numpy(idx[b:b + 1000])]
            neg = torch.from_numpy(negs[i, :pos.shape[0]].copy())
            i += 1
            e = ref.kshift_fwd_torch(torch.cat([pos, neg]), W, 16, False)
            pred = ref.mlp_quickgelu(e, ws, bs).squeeze(1)
            tgt = torch.cat([torch.ones(pos.shape[0]), torch.zeros(neg.shape[0])])
            F.binary_cross_entropy_with_logits(pred, tgt).backward()
            opt.step()
            opt.zero_grad()
    # the mask MLP runs on bf16 MFMA operands (the reference's MLP is fp32): 1e-2 on the weights
    check('model[0].emb.weight, W', relerr(model[0].emb.weight, W), 1e-2)
    glins = [l for l in model[1].model if isinstance(l, torch.nn.Linear)]
    for gl, w, b in zip(glins, ws, bs):
        check('gl.weight, w', relerr(gl.weight, w), 1e-2)
        check('gl.bias, b', relerr(gl.bias, b), 1e-2)


def test_model_wrapper_forward(dev):
    from recommendations_amd.commons.layers import MLP, KShiftEmbedding
    from recommendations_amd.embedding_module_gen import ModelWrapper
    torch.manual_seed(0)
    emb = KShiftEmbedding(5000, 32, num_shifts=16, normalize_output=True)
    mask = torch.nn.Sequential(KShiftEmbedding(5000, 4, num_shifts=16), MLP(4, 1, [64]))
    w = ModelWrapper(emb, mask).to(dev)
    ids = torch.randint(-2 ** 63, 2 ** 63 - 1, (777,), dtype=torch.int64)
    with torch.no_grad():
        got = w(ids.to(dev)).cpu()
    e = ref.kshift_fwd_torch(ids, emb.emb.weight.detach().cpu(), 16, True)
    lins = [l for l in mask[1].model if isinstance(l, torch.nn.Linear)]
    mk = ref.mlp_quickgelu(ref.kshift_fwd_torch(ids, mask[0].emb.weight.detach().cpu(), 16, False),
                           [l.weight.detach().cpu() for l in lins], [l.bias.detach().cpu() for l in lins])
    exp = mk.sigmoid() * e
    check('got, exp', relerr(got, exp), 2e-2)  # the mask MLP runs on bf16 MFMA operands


def _artifact_ref(ids, sd, K, normalize, Km):
    e = ref.kshift_fwd_torch(ids, sd["model.emb.weight"].float(), K, normalize)
    m = ref.kshift_fwd_torch(ids, sd["mask_model.0.emb.weight"], Km, False)
    lg = ref.mlp_quickgelu(m, [sd["mask_model.1.model.0.weight"], sd["mask_model.1.model.2.weight"]],
                           [sd["mask_model.1.model.0.bias"], sd["mask_model.1.model.2.bias"]])
    return lg.sigmoid() * e


@pytest.mark.parametrize("D,K,Km,Dm,H1,norm,tdt", [(32, 16, 16, 4, 64, True, torch.float32),
                                                  (128, 8, 16, 8, 128, True, torch.bfloat16),
                                                  (64, 16, 4, 16, 256, False, torch.float32),
                                                  (32, 3, 5, 4, 64, True, torch.bfloat16)])
def test_item_artifact_fused_vs_oracle(dev, D, K, Km, Dm, H1, norm, tdt):
    """the fused artifact kernel (KShift pool + mask KShift pool +
    QuickGELU MLP + sigmoid gate, one launch) vs the oracle composition of the
    reference's ModelWrapper (embedding_module_gen.py:32-41).  All-f32 arithmetic
    (the table is read as stored; bf16 tables are compared on the same bf16 values):
    1e-5 relative Frobenius (exp / summation-order rounding only)."""
    from recommendations_amd.models.lthm.sequence.item_artifact import ItemEmbeddingArtifact
    torch.manual_seed(D + K)
    m = ItemEmbeddingArtifact(7001, D, K, norm, 3001, Dm, Km, H1, table_dtype=tdt)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn(p.shape).to(p.dtype))
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    ids = torch.randint(-2 ** 63, 2 ** 63 - 1, (3, 333), dtype=torch.int64)
    ids[0, :5] = torch.tensor([0, 1, -1, 2 ** 63 - 1, -2 ** 63])
    got = m(ids.to(dev)).cpu()
    assert got.shape == (3, 333, D)
    check('got, _artifact_ref(ids.view(-1), sd, K, norm, Km).view(3, 333, D)', relerr(got, _artifact_ref(ids.view(-1), sd, K, norm, Km).view(3, 333, D)), 1e-5)
    assert m(torch.empty(0, dtype=torch.int64, device=dev)).shape == (0, D)


def test_item_artifact_round_trip_and_encoder(dev, tmp_path):
    """embedding_module_gen ModelWrapper -> save_item_artifact (safetensors) ->
    load_item_artifact -> fused forward == the unfused ModelWrapper forward; the LTHM
    encoder built with product_tower.model_init_metadata uses it (encoder.py:25-29)."""
    from recommendations_amd.commons.layers import MLP, KShiftEmbedding
    from recommendations_amd.embedding_module_gen import ModelWrapper
    from recommendations_amd.models.lthm.sequence.item_artifact import (ItemEmbeddingArtifact, load_item_artifact,
                                                                      save_item_artifact)
    torch.manual_seed(1)
    w = ModelWrapper(KShiftEmbedding(5000, 32, num_shifts=16, normalize_output=True),
                     torch.nn.Sequential(KShiftEmbedding(5750, 4, num_shifts=16), MLP(4, 1, [64])))
    path = str(tmp_path / "item.safetensors")
    save_item_artifact(w, path)
    a = load_item_artifact(path, device=dev)
    w = w.to(dev)
    ids = torch.randint(-2 ** 63, 2 ** 63 - 1, (4096,), dtype=torch.int64, device=dev)
    with torch.no_grad():
        check('a(ids), w(ids)', relerr(a(ids), w(ids)), 2e-2)  # the unfused mask MLP uses bf16 MFMA operands
    sd = {k: v.detach().cpu() for k, v in w.state_dict().items()}
    check('a(ids).cpu(), _artifact_ref(ids.cpu(), sd, 16, True, 16)', relerr(a(ids).cpu(), _artifact_ref(ids.cpu(), sd, 16, True, 16)), 1e-5)

    from recommendations_amd.models.lthm.builder import LTHMModelBuilder
    from recommendations_amd.models.lthm.config import lthm_config
    from recommendations_amd.data import synthetic_lthm_batch
    cfg = lthm_config(T=32, d=64, n_layers=2, n_head=1, item_vocab=5000)
    cfg.product_tower.model_init_metadata = {"embedding_module_path": path}
    model = LTHMModelBuilder(None, cfg).build().to(dev)
    arts = [mod for mod in model.modules() if isinstance(mod, ItemEmbeddingArtifact)]
    assert len(arts) == 1
    batch = synthetic_lthm_batch(64, 32, seed=3, device=dev)
    out = model(batch)
    loss, _ = model.train_step(batch, out)
    assert torch.isfinite(loss).all()


@pytest.mark.parametrize("n,ydt", [(1, torch.float32), (1000, torch.float32), (262_144 * 4 + 3, torch.float32),
                                   (70_001, torch.bfloat16)])
def test_mse_loss_kernel(dev, n, ydt):
    """lthm_mse_fwd / _bwd (nn.MSELoss of the reconstruction model) against torch fp64."""
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(n)
    y = torch.randn(n, generator=g).to(ydt)
    x = torch.randn(n, generator=g)
    yd = y.to(dev).requires_grad_(True)
    loss = K.mse_loss(yd, x.to(dev))
    loss.backward(torch.tensor(0.5, device=dev))
    yr = y.double().requires_grad_(True)
    lr = F.mse_loss(yr, x.double())
    (0.5 * lr).backward()
    check("mse loss vs fp64", abs(float(loss) - float(lr)) / max(abs(float(lr)), 1e-30), 1e-5)
    tol = 1e-6 if ydt == torch.float32 else 8e-3  # the bf16 gradient's own rounding
    check("mse grad vs fp64", relerr(yd.grad.float(), yr.grad), tol)
