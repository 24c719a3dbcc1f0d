"""Ranker host logic on CPU: config defaults (BASELINE configs[3] / SURVEY §8d C4),
the module tree / parameter names the wrapper groups for its optimizers, and the
oracle composition on a tiny model (no GPU compute)."""
import torch

from oracle import ranker_ref


def test_c4_config_defaults():
    from recommendations_amd.models.ranker.config import RankerModelConfig, normal_quantiles
    cfg = RankerModelConfig()
    assert (cfg.n_dense, cfg.n_categorical, cfg.cat_vocab, cfg.cat_emb_dim) == (128, 64, 1_000_000, 32)
    assert cfg.dense_n_projs == [16] and cfg.dense_num_bins == [20] and cfg.gate_sizes == [1024, 512]
    assert cfg.emb_dim == 64 and cfg.type == "factorized_dlrm"
    q = normal_quantiles(20)
    assert len(q) == 20 and abs(q[9] + q[10]) < 1e-12 and all(a < b for a, b in zip(q, q[1:]))


def test_ranker_param_groups_and_oracle_cpu():
    from recommendations_amd.data import synthetic_ranker_batch
    from recommendations_amd.models.ranker.config import ranker_config
    cfg = ranker_config(n_dense=6, n_cat=3, cat_vocab=50, gate_sizes=(16,), emb_dim=8)
    m = cfg.get_builder().build()
    groups = m.param_groups()
    assert [p.shape for p in groups["SPARSE_ROWS"]] == [torch.Size([150, 32])]
    assert len(groups["USE_OPTIM"]) == 1 + 4  # CVE table + 2 Linear (weight, bias)
    sd = {k: v.detach().float() if v.is_floating_point() else v for k, v in m.state_dict().items()}
    batch = synthetic_ranker_batch(64, 6, 3, seed=1)
    logits = ranker_ref.ranker_forward(sd, cfg, batch)
    assert logits.shape == (64, 1) and torch.isfinite(logits).all()
    # FlatEmbedding semantics: W[x mod P] (torch.remainder: non-negative)
    W = sd["_model.cat_tables.weight"].view(3, 50, 32)
    ids = batch["categorical"][:, 1]
    assert torch.equal(W[1][torch.remainder(ids, 50)], W[1][ids % 50])
