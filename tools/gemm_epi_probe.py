"""Time the C2 encoder forward GEMM forms by epilogue (csrc/gemm.hip gemm_ps_k) to separate
store bandwidth from epilogue VALU: plain bf16 C, + bias, GELU, GELU with the aux store,
GELU_D with the aux store, and the dgrad MUL_AUX form; M = 4096 x 129, K = 256."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendations_amd import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    M, Kd = 4096 * 129, 256
    for N in (768, 1024):
        a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, Kd, device=dev) / 16).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        rows = [("plain", lambda: K.linear_fwd(a, w), 1),
                ("bias", lambda: K.linear_fwd(a, w, b), 1),
                ("gelu", lambda: K.linear_fwd(a, w, b, act=K.ACT_GELU), 1),
                ("gelu+aux", lambda: K.linear_fwd(a, w, b, act=K.ACT_GELU, aux_out=aux), 2),
                ("gelu_d+aux", lambda: K.linear_fwd(a, w, b, act=K.ACT_GELU_D, aux_out=aux), 2)]
        for name, fn, nst in rows:
            t = timeit(fn)
            gb = (M * Kd * 2 + nst * M * N * 2) / 1e9
            print(f"N={N} {name:11s} {t:.3f} ms  {gb / t:.2f} TB/s (algorithmic {gb:.2f} GB)", flush=True)
    # dgrad through GELU': dpre = (dy W2) * aux, dy [M, 256], W2 [256, 1024] K-strided
    N2 = 1024
    dy = torch.randn(M, 256, device=dev).to(torch.bfloat16)
    w2 = (torch.randn(256, N2, device=dev) / 16).to(torch.bfloat16)
    aux = torch.randn(M, N2, device=dev).to(torch.bfloat16)
    t = timeit(lambda: K.linear_dgrad(dy, w2, act_grad=K.ACT_MUL_AUX, aux=aux))
    gb = (M * 256 * 2 + 2 * M * N2 * 2) / 1e9
    print(f"dgrad mul_aux {t:.3f} ms  {gb / t:.2f} TB/s", flush=True)
    t = timeit(lambda: K.linear_dgrad(dy, w2))
    gb = (M * 256 * 2 + M * N2 * 2) / 1e9
    print(f"dgrad plain   {t:.3f} ms  {gb / t:.2f} TB/s", flush=True)
    x = torch.empty(M, N2, dtype=torch.bfloat16, device=dev)
    t = timeit(lambda: x.fill_(1.0))
    print(f"torch fill    {t:.3f} ms  {M * N2 * 2 / 1e9 / t:.2f} TB/s (store-only yardstick)", flush=True)


if __name__ == "__main__":
    main()
