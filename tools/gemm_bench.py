"""Microbenchmark of the MFMA GEMM (csrc/gemm.hip) on the LTHM C2 encoder shapes,
with torch.matmul (hipBLASLt) timed beside it as a yardstick only."""
import sys
import os
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendations_amd import kernels as K  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
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
    M = 4096 * 129
    shapes = [("qkv", M, 768, 256), ("proj", M, 256, 256), ("fc", M, 1024, 256), ("fc2", M, 256, 1024)]
    if os.environ.get("GEMM_BENCH_CFG") == "c5":  # C5: B 1024 x T' 513, d 512, MQA (q 512 + kv 128)
        M = 1024 * 513
        shapes = [("qkv", M, 640, 512), ("proj", M, 512, 512), ("fc", M, 2048, 512), ("fc2", M, 512, 2048)]
    if os.environ.get("GEMM_BENCH_CFG") == "c4":  # C4 ranker MLP: 2,176 -> 1,024 -> 512 at batch 65,536
        M = 65536
        shapes = [("fc1", M, 1024, 2176), ("fc2", M, 512, 1024), ("fc1dg", M, 2176, 1024)]
    if os.environ.get("GEMM_BENCH_SQUARE"):
        shapes.append(("sq4096", 4096, 4096, 4096))
    for name, m, n, k in shapes:
        a = torch.randn(m, k, device=dev).to(torch.bfloat16)
        w = torch.randn(n, k, device=dev).to(torch.bfloat16)
        fl = 2.0 * m * n * k
        t0 = timeit(lambda: K.linear_fwd(a, w))
        t1 = timeit(lambda: K.linear_fwd(a, w, act=K.ACT_GELU, aux_out=None))
        t2 = timeit(lambda: torch.matmul(a, w.T))
        dy = torch.randn(m, n, device=dev).to(torch.bfloat16)
        t3 = timeit(lambda: K.linear_dgrad(dy, w))
        # the same dgrad product with a K-contiguous B (W^T materialised): the forward kernel form
        wt = w.t().contiguous()
        t3t = timeit(lambda: K.linear_fwd(dy, wt))
        t4 = timeit(lambda: K.linear_wgrad(dy, a), iters=5)
        t5 = timeit(lambda: torch.matmul(dy.T, a), iters=5)
        t8 = float("nan")
        if os.environ.get("GEMM_BENCH_FP8") and k % 128 == 0:
            xq, xs = K.quantize_fp8(a)
            wq, ws = K.quantize_fp8(w)
            t8 = timeit(lambda: K.linear_fwd_fp8(xq, xs, wq, ws))
        byts = 2.0 * (m * k + n * k + m * n)  # bf16 A + W + C, each once
        print(f"{name:7s} M={m} N={n} K={k}: fwd {t0:.3f} ms ({fl / t0 / 1e9:.0f} TF, "
              f"{byts / t0 / 1e6:.0f} GB/s)  +gelu {t1:.3f}  "
              f"hipblaslt {t2:.3f} ({fl / t2 / 1e9:.0f} TF) | dgrad {t3:.3f} ({fl / t3 / 1e9:.0f} TF) "
              f"via W^T {t3t:.3f} ({fl / t3t / 1e9:.0f} TF) | "
              f"wgrad {t4:.3f} ({fl / t4 / 1e9:.0f} TF) hipblaslt {t5:.3f} | fp8 fwd {t8:.3f} ({fl / t8 / 1e9:.0f} TF)",
              flush=True)


if __name__ == "__main__":
    main()
