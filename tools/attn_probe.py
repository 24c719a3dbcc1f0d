"""Time the C2 attention forward / backward (B=4096, T'=129, H=4, E=64, causal,
relative-position bias table) through the C ABI; TAG labels the variant."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendations_amd import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    # C2 by default; SHAPE=B,T,H overrides (C5: 1024,513,8)
    B, T, H = (int(v) for v in os.environ.get("SHAPE", "4096,129,4").split(","))
    E = 64
    qkv = (torch.randn(B * T, 3 * H * E, device=dev) * 0.5).to(torch.bfloat16)
    tab = torch.randn(2 * T + 1, H, device=dev) * 0.1
    out, lse = K.attn_fwd_qkv(qkv, B, T, H, E, table=tab)
    dout = torch.randn_like(out)
    tf = timeit(lambda: K.attn_fwd_qkv(qkv, B, T, H, E, table=tab))
    tb = timeit(lambda: K.attn_bwd_qkv(qkv, out, dout, lse, B, T, H, E, table=tab))
    tb0 = timeit(lambda: K.attn_bwd_qkv(qkv, out, dout, lse, B, T, H, E, table=None))
    print(os.environ.get("TAG", ""), f"fwd {tf:.3f} ms | bwd {tb:.3f} ms | bwd (no bias grad) {tb0:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
