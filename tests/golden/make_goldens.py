"""Generate golden input/output vectors by importing the reference itself.

Run ONLY in the build container, where the reference is mounted read-only:

    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py

It imports the reference's own component classes (SURVEY.md §8c lists which
ones import and run), drives them with seeded inputs on the CPU in fp32 and
writes small .npz fixtures next to this script.  Nothing of the reference's
source is copied; only the numbers it produced are kept.  The fixtures are the
parity pins for oracle/ (CPU) and for the HIP kernels (tests -m gpu).
"""
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
INT64_MIN = -(2 ** 63)
INT64_MAX = 2 ** 63 - 1


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in arrays.items()})
    print("wrote", path, sum(np.asarray(v).nbytes if not torch.is_tensor(v) else v.numel() * v.element_size()
                               for v in arrays.values()), "bytes")


def adversarial_ids(n_random, seed):
    g = torch.Generator().manual_seed(seed)
    fixed = torch.tensor([0, 1, -1, 2, -2, INT64_MIN, INT64_MAX, INT64_MIN + 1, INT64_MAX - 1,
                          2 ** 32, -(2 ** 32), 2 ** 62, -(2 ** 62), 12345, -7448648811083631205],
                         dtype=torch.int64)
    rnd = torch.randint(INT64_MIN, INT64_MAX, (n_random,), generator=g, dtype=torch.int64)
    return torch.cat([fixed, rnd])


def gen_hashing():
    from commons.feature_utils import (hash_feature_name_to_int, hash_string_to_long, pad_array,
                                       handle_categorical_history_feature)
    import pandas as pd
    names = ["product_id", "Product_ID", "customer_id", "brand", "labels", "timestamps", "", "a",
             "category_l3_name_with_a_really_long_feature_name_over_32_bytes"]
    seeds = np.array([hash_feature_name_to_int(n) for n in names], dtype=np.int64)
    strings = ["12345", "NA", "na", "", "x", "abcdefgh", "abcdefghijklmnopqrstuvwxyz0123456789ABCDEFGHIJ",
               "Ünïcödé-✓", "1234567", "123456789012345678901234567890123", "-42", "3.14159"]
    seed_list = [0, 396283771, 2 ** 32 - 1, int(seeds[1])]
    out = np.zeros((len(seed_list), len(strings), 2), dtype=np.int64)
    for i, s in enumerate(seed_list):
        for j, st in enumerate(strings):
            out[i, j, 0] = hash_string_to_long(st, s, False)
            out[i, j, 1] = hash_string_to_long(st, s, True)
    # categorical history: hash + drop label id + cap + pad (feature_utils.py:149-179)
    rng = np.random.default_rng(7)
    rows = []
    for r in range(6):
        L = int(rng.integers(0, 12))
        rows.append([str(int(x)) for x in rng.integers(0, 30, size=L)])
    label_seed = hash_feature_name_to_int("product_id")
    label = [hash_string_to_long(h[0] if h else "0", label_seed, False) for h in rows]
    df = pd.DataFrame({"product_id": label, "hist": rows})
    handle_categorical_history_feature(df, "hist", hash_ids=True, history_length=8,
                                       history_id_feature_name="product_id",
                                       remove_history_id_from_history=True)
    hist = np.stack(df["hist"].values).astype(np.int64)
    flat = [",".join(r) for r in rows]
    save("hashing", names=np.array(names), name_seeds=seeds, strings=np.array(strings),
         seed_list=np.array(seed_list, dtype=np.int64), hashes=out, hist_rows=np.array(flat),
         hist_label=np.array(label, dtype=np.int64), hist_out=hist,
         pad_in=np.array([5, -3, 7], dtype=np.int64), pad_out=pad_array([5, -3, 7], 6))


def gen_kshift():
    from commons.layers import KShiftEmbedding, FlatEmbedding
    torch.manual_seed(0)
    ids = adversarial_ids(200, 1)
    # row indices for every rotation c = 0..31 and several table sizes
    Ps = [1_000_000, 1000, 7, 2 ** 20 + 1, 1_150_000]
    rows = np.zeros((len(Ps), 32, ids.numel()), dtype=np.int64)
    for a, P in enumerate(Ps):
        m = KShiftEmbedding(P, 1, num_shifts=32)
        for c in range(32):
            rows[a, c] = m.get_row_idx(ids, c).numpy()
    save("kshift_rows", ids=ids, Ps=np.array(Ps, dtype=np.int64), rows=rows)

    cases = []
    for (P, D, K, norm, seed) in [(1000, 32, 16, False, 1), (1000, 32, 16, True, 2), (997, 32, 8, False, 3),
                                  (4096, 4, 16, False, 4), (512, 256, 8, True, 5), (300, 8, 1, False, 6)]:
        torch.manual_seed(seed)
        m = KShiftEmbedding(P, D, num_shifts=K, normalize_output=norm)
        x = adversarial_ids(300, seed + 10).reshape(-1, 5)
        y = m(x)
        g = torch.Generator().manual_seed(seed + 20)
        dy = torch.randn(y.shape, generator=g)
        (y * dy).sum().backward()
        save(f"kshift_fwd_bwd_{len(cases)}", P=P, D=D, K=K, normalize=int(norm), weight=m.emb.weight.detach(),
             ids=x, out=y, dy=dy, dweight=m.emb.weight.grad)
        cases.append(1)
    for (P, D, norm, pad, seed) in [(10_000, 16, False, None, 1), (4, 32, True, None, 2), (50, 8, False, 0, 3)]:
        torch.manual_seed(seed)
        m = FlatEmbedding(P, D, padding_idx=pad, normalize_output=norm)
        x = adversarial_ids(100, seed + 30)
        y = m(x)
        dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(seed))
        (y * dy).sum().backward()
        save(f"flat_{seed}", P=P, D=D, normalize=int(norm), padding_idx=-1 if pad is None else pad,
             weight=m._emb_table.weight.detach(), ids=x, out=y, dy=dy, dweight=m._emb_table.weight.grad)


def gen_layers():
    from commons.layers import MLP, QuickGELU, CascadedStreamingLogQCorrectionModule
    from commons.functional import cap_gradients
    torch.manual_seed(11)
    mlp = MLP(24, 5, [32, 16])
    x = torch.randn(37, 24, requires_grad=True)
    y = mlp(x)
    dy = torch.randn(y.shape)
    (y * dy).sum().backward()
    sd = {f"p_{k}": v for k, v in mlp.state_dict().items()}
    save("mlp_quickgelu", x=x.detach(), out=y.detach(), dy=dy, dx=x.grad,
         **sd, **{f"g_{n}": p.grad for n, p in mlp.named_parameters()})
    q = QuickGELU()
    xs = torch.linspace(-8, 8, 257)
    save("quickgelu", x=xs, out=q(xs))
    # cap_gradients: identity forward, g / (||g|| + 1e-6) backward
    t = torch.randn(5, 7, requires_grad=True)
    u = cap_gradients(t)
    gu = torch.randn(5, 7) * 3
    u.backward(gu)
    save("cap_gradients", x=t.detach(), out=u.detach(), dy=gu, dx=t.grad)
    # logQ forward
    m = CascadedStreamingLogQCorrectionModule(2 ** 12, [0, 34144, 7465477], alpha=0.05, p_init=0.001)
    with torch.no_grad():
        for mod in m.models:
            mod.b.copy_(torch.rand(mod.b.shape, generator=torch.Generator().manual_seed(3)) + 0.5)
    ids = adversarial_ids(60, 5).reshape(5, -1)
    save("logq", ids=ids, num_buckets=2 ** 12, offsets=np.array([0, 34144, 7465477]),
         b=torch.stack([mod.b for mod in m.models]), out=m(ids))


def gen_transformer():
    from commons.transformers.layers import (TransformerBlock, CosineVectorEmbedding, MultiQueryAttention,
                                             MoELinear, DenseMapper, QuantileMapper, SimhashVectorIndexer,
                                             LayerNorm)
    from commons.transformers.configs import TransformerConfig
    for idx, (d, H, T, B, bias, causal, pos) in enumerate([(64, 1, 17, 3, False, True, 20), (128, 2, 33, 2, True, True, 40),
                                                          (64, 2, 9, 4, False, False, None)]):
        torch.manual_seed(100 + idx)
        cfg = TransformerConfig(rotator_config={"ff_mult": 4}, is_causal=causal,
                                attn_config=dict(attn_dropout=0.0, bias=bias, dropout=0.0, n_head=H, n_embd=d,
                                                 attn_type="multi_head",
                                                 pos_bias=None if pos is None else {"context_window": pos}))
        blk = TransformerBlock(cfg, seed=idx)
        with torch.no_grad():   # non-trivial LN affine and position bias
            for n, p in blk.named_parameters():
                if "ln_" in n or "pos_bias" in n:
                    p.add_(0.1 * torch.randn(p.shape))
        x = torch.randn(B, T, d, requires_grad=True)
        y = blk(x)
        dy = torch.randn(y.shape)
        (y * dy).sum().backward()
        save(f"transformer_block_{idx}", d=d, H=H, T=T, B=B, bias=int(bias), causal=int(causal),
             context_window=-1 if pos is None else pos, x=x.detach(), out=y.detach(), dy=dy, dx=x.grad,
             **{f"p_{k}": v for k, v in blk.state_dict().items()},
             **{f"g_{n}": p.grad for n, p in blk.named_parameters()})
    # LayerNorm alone (eps 1e-5)
    torch.manual_seed(5)
    ln = LayerNorm(48, bias=True)
    with torch.no_grad():
        ln.weight.add_(torch.randn(48) * 0.2)
        ln.bias.add_(torch.randn(48) * 0.2)
    x = torch.randn(31, 48, requires_grad=True) * 3
    x.retain_grad()
    y = ln(x)
    dy = torch.randn(y.shape)
    (y * dy).sum().backward()
    save("layernorm", x=x.detach(), w=ln.weight.detach(), b=ln.bias.detach(), out=y.detach(), dy=dy, dx=x.grad,
         dw=ln.weight.grad, db=ln.bias.grad)
    # CosineVectorEmbedding (bucketize + EmbeddingBag sum)
    for nb in [2, 20]:
        torch.manual_seed(200 + nb)
        cve = CosineVectorEmbedding(32, 64, n_proj=32, num_bins=nb)
        x = torch.randn(3, 11, 32)
        x[0, 0] = 0.0
        y = cve(x)
        dy = torch.randn(y.shape)
        (y * dy).sum().backward()
        save(f"cve_{nb}", x=x, out=y.detach(), dy=dy, projection_mat=cve.projection_mat, grid=cve.grid,
             pos_offset=cve.pos_offset, weight=cve.emb.weight.detach(), dweight=cve.emb.weight.grad)
    # MultiQueryAttention (selectable in the build)
    torch.manual_seed(300)
    from types import SimpleNamespace
    acfg = SimpleNamespace(n_embd=64, n_head=4, attn_dropout=0.0, dropout=0.0, bias=True,
                           pos_bias=SimpleNamespace(context_window=16))
    mqa = MultiQueryAttention(acfg)
    with torch.no_grad():
        mqa.attn.pos_bias.bias.add_(0.3 * torch.randn(mqa.attn.pos_bias.bias.shape))
    x = torch.randn(2, 13, 64, requires_grad=True)
    L = 13
    cm = torch.ones((L, L), dtype=torch.bool).tril(0)
    mask = cm.float().masked_fill(~cm, -float("inf"))[None, None]
    y = mqa(x, mask)
    dy = torch.randn(y.shape)
    (y * dy).sum().backward()
    save("mqa", x=x.detach(), out=y.detach(), dy=dy, dx=x.grad, **{f"p_{k}": v for k, v in mqa.state_dict().items()},
         **{f"g_{n}": p.grad for n, p in mqa.named_parameters()})
    # MoELinear (top-k gating)
    torch.manual_seed(400)
    moe = MoELinear(16, 24, proj_features=32, num_experts=4, top_k=2, gate_sizes=(8,))
    x = torch.randn(5, 7, 16, requires_grad=True)
    y = moe(x)
    dy = torch.randn(y.shape)
    (y * dy).sum().backward()
    save("moe", x=x.detach(), out=y.detach(), dy=dy, dx=x.grad, **{f"p_{k}": v for k, v in moe.state_dict().items()})
    # DenseMapper / QuantileMapper
    torch.manual_seed(500)
    qs = torch.distributions.Normal(0, 1).icdf(torch.linspace(0.025, 0.975, 20)).tolist()
    stats = {f"f{i}": qs for i in range(6)}
    dm = DenseMapper(stats, emb_dim=16, n_projs=[16], num_bins=[20])
    batch = {f"f{i}": torch.randn(9, 1) for i in range(6)}
    y = dm(batch)
    save("dense_mapper", x=torch.cat([batch[f"f{i}"] for i in range(6)], 1), quantiles=np.array(qs, dtype=np.float32),
         out=y.detach(), projection_mat=dm.emb[0].projection_mat, grid=dm.emb[0].grid, weight=dm.emb[0].emb.weight.detach())
    sv = SimhashVectorIndexer(8, 16)
    x = torch.randn(10, 8)
    save("simhash", x=x, projection_mat=sv.projection_mat, out=sv(x))


def gen_transformer_mask():
    """TransformerBlock.forward(x, attn_mask) with a general additive mask
    (commons/transformers/layers.py:374, :404-408): [B, 1, T, T] random scores plus
    -inf on padded key columns (never a whole row), on top of the causal mask or not."""
    from commons.transformers.layers import TransformerBlock
    from commons.transformers.configs import TransformerConfig
    for idx, (d, H, T, B, causal) in enumerate([(64, 2, 21, 3, True), (64, 1, 12, 2, False)]):
        torch.manual_seed(600 + idx)
        cfg = TransformerConfig(rotator_config={"ff_mult": 4}, is_causal=causal,
                                attn_config=dict(attn_dropout=0.0, bias=True, dropout=0.0, n_head=H, n_embd=d,
                                                 attn_type="multi_head", pos_bias={"context_window": 32}))
        blk = TransformerBlock(cfg, seed=idx)
        with torch.no_grad():
            for n, p in blk.named_parameters():
                if "ln_" in n or "pos_bias" in n:
                    p.add_(0.1 * torch.randn(p.shape))
        mask = 0.5 * torch.randn(B, 1, T, T)
        for b in range(B):
            mask[b, :, :, T - 1 - b:] = -float("inf")  # padded keys of sequence b
            mask[b, :, :, 0] = 0.0                    # key 0 always visible
        x = torch.randn(B, T, d, requires_grad=True)
        y = blk(x, mask)
        dy = torch.randn(y.shape)
        (y * dy).sum().backward()
        save(f"transformer_block_mask_{idx}", d=d, H=H, T=T, B=B, bias=1, causal=int(causal), context_window=32,
             mask=mask, x=x.detach(), out=y.detach(), dy=dy, dx=x.grad,
             **{f"p_{k}": v for k, v in blk.state_dict().items()},
             **{f"g_{n}": p.grad for n, p in blk.named_parameters()})


def gen_vecemb():
    """CosineLinear, LearnableCosineVectorEmbedding, ProbabilityVectorEmbedding and a
    wider SimhashVectorIndexer (commons/transformers/layers.py:426-595), forward + backward."""
    from commons.transformers.layers import (CosineLinear, LearnableCosineVectorEmbedding,
                                             ProbabilityVectorEmbedding, SimhashVectorIndexer)
    torch.manual_seed(600)
    cl = CosineLinear(24, 7)
    x = torch.randn(5, 6, 24)
    x[0, 0] = 0.0
    x.requires_grad_(True)
    y = cl(x)
    dy = torch.randn(y.shape)
    (y * dy).sum().backward()
    save("cosine_linear", x=x.detach(), weight=cl.weight.detach(), out=y.detach(), dy=dy, dx=x.grad,
         dweight=cl.weight.grad)
    for tag, nb, tk in (("lcve", 20, None), ("lcve_top5", 20, 5), ("lcve_nb7", 7, 3)):
        torch.manual_seed(610 + nb + (tk or 0))
        m = LearnableCosineVectorEmbedding(24, 32, n_proj=8, num_bins=nb, sigma_inflation_factor=1.5, top_k=tk)
        x = torch.randn(3, 9, 24, requires_grad=True)
        y = m(x)
        dy = torch.randn(y.shape)
        (y * dy).sum().backward()
        save(tag, x=x.detach(), proj_weight=m.proj.weight.detach(), mean=m.mean.detach(), emb_weight=m.emb.weight.detach(),
             sigma2=np.float64(m.sigma2), top_k=np.int64(tk or 0), out=y.detach(), dy=dy, dx=x.grad,
             dproj_weight=m.proj.weight.grad, dmean=m.mean.grad, demb_weight=m.emb.weight.grad)
    for tag, nb, tk in (("pve", 10, None), ("pve_top3", 10, 3)):
        torch.manual_seed(620 + (tk or 0))
        m = ProbabilityVectorEmbedding(16, num_bins=nb, top_k=tk)
        x = torch.rand(40, 1, requires_grad=True)
        y = m(x)
        dy = torch.randn(y.shape)
        (y * dy).sum().backward()
        save(tag, x=x.detach(), mean=m.mean.detach(), emb_weight=m.emb.weight.detach(), sigma2=np.float64(m.sigma2),
             top_k=np.int64(tk or 0), out=y.detach(), dy=dy, dx=x.grad, dmean=m.mean.grad,
             demb_weight=m.emb.weight.grad)
    torch.manual_seed(630)
    sv = SimhashVectorIndexer(40, 63)
    x = torch.randn(4, 25, 40)
    save("simhash63", x=x, projection_mat=sv.projection_mat, out=sv(x))


if __name__ == "__main__":
    if not any("reference" in p for p in sys.path + os.environ.get("PYTHONPATH", "").split(":")):
        sys.exit("run with PYTHONPATH=/root/reference (build container only)")
    torch.set_num_threads(4)
    which = sys.argv[1:] or ["hashing", "kshift", "layers", "transformer"]
    for w in which:
        globals()["gen_" + w]()
