"""Row-wise AdamW (lthm_sparse_adamw) on the C4 table shape (64 x 1M rows x 32 f32, ~4M touched
rows a step): touched rows in first-touch (random) order vs sorted by row, and the bf16 shadow."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendations_amd import kernels as K  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    dev = torch.device("cuda")
    R, D, n = 64 * 1_000_000, 32, 4_000_000
    g = torch.Generator(device=dev).manual_seed(0)
    p = torch.randn(R, D, device=dev)
    gr = torch.zeros(R, D, device=dev)
    m = torch.zeros(R, D, device=dev)
    v = torch.zeros(R, D, device=dev)
    sh = torch.empty(R, D, dtype=torch.bfloat16, device=dev)
    flags = torch.zeros(R, dtype=torch.int32, device=dev)
    rows = torch.randperm(R, device=dev, generator=g)[:n].to(torch.int64)
    srt = torch.sort(rows).values
    cnt = torch.tensor([n], dtype=torch.int64, device=dev)
    per_row = 8 + 4 + 8 * 4 * D + 2 * D
    for name, rl in (("random", rows), ("sorted", srt)):
        for shadow in (sh, None):
            t = timeit(lambda: K.sparse_adamw_(rl, cnt, n, p, gr, m, v, flags, 1e-3, (0.9, 0.999), 1e-8, 0.0, 1,
                                               shadow=shadow))
            b = n * (per_row - (0 if shadow is not None else 2 * D))
            print(f"{name:7s} shadow={shadow is not None}: {t:.3f} ms  {b / t / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
