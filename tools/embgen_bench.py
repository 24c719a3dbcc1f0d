"""Item-embedding generator step time (embedding_module_gen.py:122-156 / :70-118 at the reference
sizes: batches of 2^18 ids, K = 16, P = 1.15 n), the fused dedup + Adagrad
(SparseRowAdagrad(fused=True), lthm_kshift_adagrad_fused) against the two-pass row path
(row gradients staged by the backward, then the row-wise Adagrad), each after its warm-up, on
the same seeded ids.  Prints one JSON line per (model, path).

    python tools/embgen_bench.py [--n 2000000] [--steps 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_000_000, help="catalogue size (P = 1.15 n)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    from recommendations_amd import kernels as K
    from recommendations_amd.commons.layers import MLP, KShiftEmbedding
    from recommendations_amd.optim import FusedAdagrad, SparseRowAdagrad
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    P = int(1.15 * args.n)
    catalogue = torch.randint(-2 ** 63, 2 ** 63 - 1, (args.n,), device=dev, generator=g, dtype=torch.int64)
    for model in ("reconstruction", "mask"):
        for fused in (True, False):
            torch.manual_seed(0)
            if model == "reconstruction":
                D, B = 32, 1 << 18
                emb = KShiftEmbedding(P, D, num_shifts=16, normalize_output=True, sparse=True).to(dev)
                net, extra = emb, None
                tgt = K.l2norm_rows(torch.randn(B, D, device=dev, generator=g))
            else:
                D, B = 4, 1 << 17
                emb = KShiftEmbedding(P, D, num_shifts=16, normalize_output=False, sparse=True).to(dev)
                net = torch.nn.Sequential(emb, MLP(D, 1, [D * 16])).to(dev)
                extra = FusedAdagrad(net[1].parameters(), lr=0.5)
                tgt = torch.cat([torch.ones(B, device=dev), torch.zeros(B, device=dev)])
            opt = SparseRowAdagrad([emb], lr=0.5, fused=fused)
            batches = []
            for _ in range(4):
                pos = catalogue[torch.randint(0, args.n, (B,), device=dev, generator=g)]
                if model == "mask":
                    neg = torch.randint(-2 ** 63, 2 ** 63 - 1, (B,), device=dev, generator=g, dtype=torch.int64)
                    pos = torch.cat([pos, neg])
                batches.append(pos)

            def step(i):
                ids = batches[i % len(batches)]
                if model == "reconstruction":
                    loss = K.mse_loss(net(ids), tgt)
                else:
                    loss = K.bce_with_logits(net(ids).squeeze(1).float().contiguous(), tgt)
                loss.backward()
                opt.step()
                if extra is not None:
                    extra.step()
                    extra.zero_grad(set_to_none=True)

            for i in range(args.warmup):
                step(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(args.steps):
                step(i)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.steps
            print(json.dumps({"model": model, "path": "fused" if fused else "two-pass", "ms_per_step": round(ms, 4),
                              "ids_per_step": B if model == "reconstruction" else 2 * B,
                              "P": P, "D": D, "K": 16, "steps": args.steps}), flush=True)
            del emb, net, opt, extra
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
