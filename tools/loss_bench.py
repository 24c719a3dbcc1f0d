"""Contrastive-loss kernels alone on the C2 shape (B 4096, T 128, 6 heads,
32-sequence mini-batches, tau 0.05), for per-kernel timing under
``rocprofv3 --kernel-trace --stats -- python3 tools/loss_bench.py``.
Prints the HIP-event time of one fused fwd + bwd."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main(iters=10, B=4096, T=128, NH=6, mbs=32, tau=0.05):
    from recommendations_amd.models.lthm.sequence.wrapper import ContrastiveLossFn
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    y = torch.randn((B, T + 1, NH, 128), device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    tgt = torch.randn((B, T, 128), device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    npad = torch.randint(0, T // 2, (B,), device=dev, generator=g)
    mask = (torch.arange(T, device=dev)[None, :] < npad[:, None]).to(torch.uint8)
    n_mb = (B + mbs - 1) // mbs
    offsets = torch.randint(1, 32, (n_mb, NH), device=dev, generator=g, dtype=torch.int32)
    cfg = dict(mb=mbs, tau=tau, ks=[1, 5, 10, 50, 100], flops=[1.0] * NH)

    def step():
        loss = ContrastiveLossFn.apply(y, tgt, mask, offsets, cfg)
        loss.backward()
        return loss

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        loss = step()
    e1.record()
    torch.cuda.synchronize()
    print(f"loss {float(loss):.5f}  fwd+bwd {e0.elapsed_time(e1) / iters:.3f} ms")


if __name__ == "__main__":
    main()
