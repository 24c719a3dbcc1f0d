"""Time the C2 encoder GEMMs exactly as one TransformerBlock calls them (fwd with
bias / GELU + pre-activation store / f32 residuals, dgrad with the GELU-grad
epilogue); one line per run, to A/B kernel variants selected by environment knobs
(LTHM_GEMM_PS=0 selects the one-tile-per-workgroup kernel)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendations_amd import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    M, d = 4096 * 129, 256
    tag = os.environ.get("TAG", "")
    bf = torch.bfloat16
    h = torch.randn(M, d, device=dev).to(bf)
    x = torch.randn(M, d, device=dev)
    x2 = torch.randn(M, d, device=dev)
    wqkv = (torch.randn(3 * d, d, device=dev) / 16).to(bf)
    wp = (torch.randn(d, d, device=dev) / 16).to(bf)
    w1 = (torch.randn(4 * d, d, device=dev) / 16).to(bf)
    w2 = (torch.randn(d, 4 * d, device=dev) / 32).to(bf)
    b3, b1, b = torch.randn(3 * d, device=dev), torch.randn(4 * d, device=dev), torch.randn(d, device=dev)
    pre = torch.empty(M, 4 * d, device=dev, dtype=bf)
    g = torch.randn(M, 4 * d, device=dev).to(bf)
    dy = torch.randn(M, d, device=dev).to(bf)
    dqkv = torch.randn(M, 3 * d, device=dev).to(bf)
    res = [
        ("qkv", lambda: K.linear_fwd(h, wqkv, b3)),
        ("proj", lambda: K.linear_fwd(h, wp, b, res1=x2, out_dtype=torch.float32)),
        ("fc", lambda: K.linear_fwd(h, w1, b1, act=K.ACT_GELU, aux_out=pre)),
        ("fc2", lambda: K.linear_fwd(g, w2, b, res1=x, res2=x2, out_dtype=torch.float32)),
        ("dpre", lambda: K.linear_dgrad(dy, w2, act_grad=K.ACT_GELU_GRAD, aux=pre)),
        ("dh2", lambda: K.linear_dgrad(g, w1)),
        ("do", lambda: K.linear_dgrad(dy, wp)),
        ("dh1", lambda: K.linear_dgrad(dqkv, wqkv)),
        ("dw2", lambda: K.linear_wgrad(dy, g)),
        ("dw1", lambda: K.linear_wgrad(g, h)),
        ("dwp", lambda: K.linear_wgrad(dy, h)),
        ("dwqkv", lambda: K.linear_wgrad(dqkv, h)),
    ]
    out, tot = [], 0.0
    for name, fn in res:
        t = timeit(fn)
        tot += t
        out.append(f"{name} {t:.3f}")
    print(tag, " | ".join(out), f"| sum {tot:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
