"""Break down the C2 encoder MLP GEMM forms (M = 4096 x 129 tokens, d = 256, 4d = 1024):
which part of the time is MFMA, epilogue VALU and output bytes.  One line per form with
its time, TFLOP/s and the GB/s of its algorithmic bytes; torch.matmul (hipBLASLt) of the
same shape beside it as a yardstick.  Also a pure-write and a copy probe for the box's
bandwidth ceilings."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendations_amd import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    M, d = 4096 * 129, 256
    bf = torch.bfloat16
    h = torch.randn(M, d, device=dev).to(bf)
    w1 = (torch.randn(4 * d, d, device=dev) / 16).to(bf)
    w2 = (torch.randn(d, 4 * d, device=dev) / 32).to(bf)
    b1, b = torch.randn(4 * d, device=dev), torch.randn(d, device=dev)
    pre = torch.empty(M, 4 * d, device=dev, dtype=bf)
    g = torch.randn(M, 4 * d, device=dev).to(bf)
    x, x2 = torch.randn(M, d, device=dev), torch.randn(M, d, device=dev)
    dy = torch.randn(M, d, device=dev).to(bf)
    big = torch.empty(M, 4 * d, device=dev, dtype=bf)
    fl = 2.0 * M * 4 * d * d
    H = M * 4 * d * 2  # bytes of one [M, 4d] bf16 tensor
    S = M * d * 2      # bytes of one [M, d] bf16 tensor
    forms = [
        ("fc plain bf16 out", lambda: K.linear_fwd(h, w1, b1), S + H),
        ("fc GELU (no aux)", lambda: K.linear_fwd(h, w1, b1, act=K.ACT_GELU), S + H),
        ("fc GELU + pre store", lambda: K.linear_fwd(h, w1, b1, act=K.ACT_GELU, aux_out=pre), S + 2 * H),
        ("fc GELU_D + GELU' store", lambda: K.linear_fwd(h, w1, b1, act=K.ACT_GELU_D, aux_out=pre), S + 2 * H),
        ("fc hipBLASLt bf16", lambda: torch.matmul(h, w1.T), S + H),
        ("fc2 plain f32 out", lambda: K.linear_fwd(g, w2, b, out_dtype=torch.float32), H + 2 * S),
        ("fc2 RES2 f32", lambda: K.linear_fwd(g, w2, b, res1=x, res2=x2, out_dtype=torch.float32), H + 6 * S),
        ("fc2 hipBLASLt bf16", lambda: torch.matmul(g, w2.T), H + S),
        ("dfc2 MUL_AUX", lambda: K.linear_dgrad(dy, w2, act_grad=K.ACT_MUL_AUX, aux=pre), S + 2 * H),
        ("dfc2 plain", lambda: K.linear_dgrad(dy, w2), S + H),
        ("dfc1 (K=1024)", lambda: K.linear_dgrad(g, w1), H + S),
        ("wgrad dW2", lambda: K.linear_wgrad(dy, g), H + S),
        ("wgrad dW1", lambda: K.linear_wgrad(g, h), H + S),
    ]
    for name, fn, nbytes in forms:
        t = timeit(fn)
        print(f"{name:26s} {t * 1e3:8.1f} us  {fl / t / 1e9:7.1f} TF  {nbytes / t / 1e6:7.1f} GB/s", flush=True)
    t = timeit(lambda: big.fill_(1.0))
    print(f"{'write [M,4d] bf16':26s} {t * 1e3:8.1f} us  {H / t / 1e6:7.1f} GB/s")
    t = timeit(lambda: big.copy_(g))
    print(f"{'copy [M,4d] bf16':26s} {t * 1e3:8.1f} us  {2 * H / t / 1e6:7.1f} GB/s")


if __name__ == "__main__":
    main()
