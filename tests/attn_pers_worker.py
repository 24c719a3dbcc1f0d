"""Child process of test_gpu_encoder.py::test_attention_persistent_bwd_matches_default: runs the
attention forward + backward of the given seeded cases with the environment it was started
with (LTHM_ATTN_BWD_P=1: the persistent double-buffered backward, read once by the library)
and saves dqkv / dtable per case to an .npz.

    python tests/attn_pers_worker.py OUT.npz B,T,H,E,causal [...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def run_case(dev, B, T, H, E, causal):
    from recommendations_amd import kernels as K
    g = torch.Generator().manual_seed(B * T + H)
    C = H * E
    qkv = torch.randn(B * T, 3 * C, generator=g).to(torch.bfloat16)
    table = 0.5 * torch.randn(2 * T + 5, H, generator=g)
    dout = torch.randn(B * T, C, generator=g).to(torch.bfloat16)
    out, lse = K.attn_fwd_qkv(qkv.to(dev), B, T, H, E, table.to(dev), causal)
    dqkv, dtab = K.attn_bwd_qkv(qkv.to(dev), out, dout.to(dev), lse, B, T, H, E, table.to(dev), causal)
    return dqkv.float().cpu().numpy(), dtab.float().cpu().numpy()


def main():
    dev = torch.device("cuda:0")
    res = {}
    for spec in sys.argv[2:]:
        B, T, H, E, c = spec.split(",")
        dq, dt = run_case(dev, int(B), int(T), int(H), int(E), c == "1")
        res[f"{spec}/dqkv"], res[f"{spec}/dtab"] = dq, dt
    np.savez(sys.argv[1], **res)


if __name__ == "__main__":
    main()
