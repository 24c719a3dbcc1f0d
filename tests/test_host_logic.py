"""CPU tests of host-side logic that shapes the hot path (no GPU calls)."""
import numpy as np
import pytest
import torch


def _reference_kept(mask: torch.Tensor, span: int) -> int:
    """query_tower.py:73-86 restated: trim rule, then Python slicing x[:, trim:]."""
    T = mask.shape[1]
    mask_all_bs = mask.unsqueeze(-1).all(dim=0)
    if mask_all_bs.sum() > T - span:
        trim = T - span
    else:
        trim = int(torch.nonzero(((~mask_all_bs).cumsum(dim=0) > 0).squeeze(1)).squeeze(1)[0])
    return torch.zeros(1, T)[:, trim:].shape[1]


@pytest.mark.parametrize("T,span", [(16, 31), (32, 7), (8, 20), (128, 7), (5, 5), (9, 3)])
def test_effective_trim_matches_reference_slicing(T, span):
    from recommendations_amd.models.lthm.sequence.query_tower import effective_trim
    g = torch.Generator().manual_seed(T * 100 + span)
    for trial in range(40):
        B = int(torch.randint(1, 6, (1,), generator=g))
        lengths = torch.randint(1, T + 1, (B,), generator=g)
        mask = torch.arange(T).unsqueeze(0) < (T - lengths).unsqueeze(1)  # left padding
        if trial % 3 == 0:  # norm-threshold masks anywhere, sometimes a whole mid column
            mask |= torch.rand(B, T, generator=g) < 0.2
            mask[:, T // 2] = True
        any_col = (~mask).any(dim=0)
        first = int(torch.nonzero(any_col)[0]) if bool(any_col.any()) else T
        n_all_pad = int((~any_col).sum())
        if first == T:
            continue  # fully padded batch: the reference itself indexes an empty nonzero()
        kept = T - effective_trim(T, span, first, n_all_pad)
        assert kept == _reference_kept(mask, span), (trial, T, span)


def test_lthm_config_shapes():
    from recommendations_amd.models.lthm.config import lthm_config
    cfg = lthm_config(T=128, d=256, n_layers=4, n_head=4, cat_features=32)
    assert cfg.emb_dim == 256
    assert cfg.export_tokens == 6 and cfg.export_span == max(cfg.lookahead) + 1
    assert cfg.transformer_config.attn_config.n_head == 4


def test_item_artifact_file_round_trip(tmp_path):
    """save_item_artifact / load_item_artifact: safetensors + KShift
    metadata, reference ModelWrapper parameter names, no code executed on load."""
    from recommendations_amd.commons.layers import MLP, KShiftEmbedding
    from recommendations_amd.embedding_module_gen import ModelWrapper
    from recommendations_amd.models.lthm.sequence.item_artifact import load_item_artifact, save_item_artifact
    torch.manual_seed(0)
    w = ModelWrapper(KShiftEmbedding(300, 32, num_shifts=12, normalize_output=True),
                     torch.nn.Sequential(KShiftEmbedding(200, 4, num_shifts=7), MLP(4, 1, [64])))
    path = str(tmp_path / "a.safetensors")
    save_item_artifact(w, path)
    a = load_item_artifact(path)
    assert (a.num_shifts, a.normalize_output, a.mask_num_shifts) == (12, True, 7)
    sd = w.state_dict()
    for k, v in a.state_dict().items():
        assert torch.equal(v, sd[k]), k
    a16 = load_item_artifact(path, table_dtype=torch.bfloat16)
    assert a16.model.emb.weight.dtype == torch.bfloat16
    save_item_artifact(a, str(tmp_path / "b.safetensors"))
    assert load_item_artifact(str(tmp_path / "b.safetensors")).num_shifts == 12
    from safetensors.torch import save_file
    save_file({"x": torch.zeros(2)}, str(tmp_path / "bad.safetensors"))
    with pytest.raises(ValueError):
        load_item_artifact(str(tmp_path / "bad.safetensors"))


def test_bench_launches_n_ranks_by_itself():
    """`python bench.py --gpus 2` with no torchrun env spawns 2 ranks itself (gloo here,
    RCCL on the GPU box) and the process group reports world size 2."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--check-launch"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    out = json.loads(line)
    assert out["world"] == 2 and out["sum"] == 2.0


def test_loss_log_batches_host_syncs():
    """embedding_module_gen._LossLog: per-batch device losses reach the logger in order,
    in groups of log_every (0 = at flush / epoch end)."""
    import torch
    from recommendations_amd.embedding_module_gen import _LossLog
    seen = []
    ll = _LossLog(lambda *a: seen.append(a), "Model", 3, 2)
    for b in range(5):
        ll.add(0, b, torch.tensor(float(b)))
        assert len(seen) == (b + 1) // 2 * 2
    ll.flush()
    assert seen == [("Model", 0, 3, b, float(b)) for b in range(5)]
    seen.clear()
    ll = _LossLog(lambda *a: seen.append(a), "MASK", 1, 0)
    ll.add(0, 0, torch.tensor(1.5))
    assert seen == []
    ll.flush()
    assert seen == [("MASK", 0, 1, 0, 1.5)]
    _LossLog(None, "x", 1, 1).add(0, 0, torch.tensor(0.0))  # no logger: nothing kept


def test_unsupported_loss_width_refused_at_construction():
    """The fused loss kernels take product_emb_dim = 128 (model/lthm.yaml:22); another width
    is refused when the wrapper is built, not at the first train_step."""
    import pytest
    from recommendations_amd.models.lthm.builder import LTHMModelBuilder
    from recommendations_amd.models.lthm.config import lthm_config
    cfg = lthm_config(T=16, d=64, n_layers=1, n_head=1, cat_features=0, item_vocab=1000, log_q_buckets=1 << 10)
    cfg.product_tower.product_emb_dim = 64
    with pytest.raises(ValueError, match="product_emb_dim=64"):
        LTHMModelBuilder(None, cfg).build()


def test_na_imputation_quantile_embedding():
    """NAImputationPlusQuantileEmbedding (commons/layers.py:84-99, build-defined constructor,
    SURVEY §3.5 #6): the reference's initial table, bucketize(x, quantiles) clamped to the last
    row, na_param where (x - na_value) < eps; gradients into the hit rows and na_param."""
    from recommendations_amd.commons.layers import NAImputationPlusQuantileEmbedding
    q = [0.0, 1.0, 2.5, 4.0, 10.0]
    m = NAImputationPlusQuantileEmbedding(-1.0, q)
    assert m.emb.weight.shape == (4, 1)
    np.testing.assert_allclose(m.emb.weight[:, 0].detach().numpy(), np.arange(4) / 5 - 0.5, rtol=0, atol=1e-7)
    with torch.no_grad():
        m.na_param.fill_(7.0)
    x = torch.tensor([[-1.0, -3.0, 0.0, 0.5], [1.0, 3.0, 10.0, 99.0]])
    y = m(x)
    assert y.shape == (2, 4, 1)
    idx = np.minimum(np.searchsorted(np.array(q), x.numpy(), side="left"), 3)
    want = np.where(x.numpy() - (-1.0) < 1e-6, 7.0, m.emb.weight[:, 0].detach().numpy()[idx])
    np.testing.assert_allclose(y[..., 0].detach().numpy(), want, rtol=0, atol=1e-7)
    y.sum().backward()
    na = (x.numpy() + 1.0 < 1e-6)
    assert float(m.na_param.grad) == na.sum()
    np.testing.assert_allclose(m.emb.weight.grad[:, 0].numpy(), np.bincount(idx[~na], minlength=4))
