"""Fused encoder MLP vs the unfused GEMM chain at the C2 shape (M = 4096 x 129 token
rows, d = 256, hidden 1024): HIP-event time per call and the MFMA rate on the
algorithmic flops.  python tools/mlp_bench.py [--iters N] [--bwd]"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timed(fn, iters):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--M", type=int, default=4096 * 129)
    ap.add_argument("--D", type=int, default=256)
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--fused-only", action="store_true", help="time only the fused kernels (profiling)")
    args = ap.parse_args()
    from recommendations_amd import kernels as K
    dev = torch.device("cuda:0")
    M, D, HID = args.M, args.D, 4 * args.D
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    x = torch.randn(M, D, device=dev, generator=g).to(bf)
    w1 = (torch.randn(HID, D, device=dev, generator=g) / math.sqrt(D)).to(bf)
    w2 = (torch.randn(D, HID, device=dev, generator=g) / math.sqrt(HID)).to(bf)
    w2t = w2.T.contiguous()
    b1 = torch.randn(HID, device=dev, generator=g) * 0.1
    b2 = torch.randn(D, device=dev, generator=g) * 0.1
    res = torch.randn(M, D, device=dev, generator=g)
    fl = 4.0 * M * D * HID
    pre = torch.empty(M, HID, dtype=bf, device=dev)
    out = {"M": M, "D": D, "HID": HID, "nw": os.environ.get("LTHM_MLP_NW", "8")}

    def unfused():
        h = K.linear_fwd(x, w1, b1, act=K.ACT_GELU_D, aux_out=pre)
        return K.linear_fwd(h, w2, b2, res1=res, out_dtype=torch.float32)

    def fused():
        return K.mlp_fwd(x, w1, b1, w2t, b2, res)

    if not args.fused_only:
        a, b = unfused(), fused()
        out["fwd_max_abs_diff"] = float((a - b).abs().max())
    for name, fn in ((("unfused_fwd", unfused),) if not args.fused_only else ()) + (("fused_fwd", fused),):
        ms = timed(fn, args.iters)
        out[name] = {"ms": round(ms, 4), "TFLOP/s": round(fl / ms / 1e9, 1), "frac_bf16_peak": round(fl / ms / 1e9 / 2500, 4)}
    if args.bwd and hasattr(K, "mlp_bwd"):
        dy = torch.randn(M, D, device=dev, generator=g).to(bf)
        fl_b = 7.0 * 2 * M * D * HID  # executed (recompute 1 + dH 1 + dX 1 + dW 2 + recompute 2)
        ms = timed(lambda: K.mlp_bwd(x, dy, w1, b1, w2t), args.iters)
        out["fused_bwd"] = {"ms": round(ms, 4), "alg_TFLOP/s": round(8.0 * M * D * HID / ms / 1e9, 1),
                            "exec_TFLOP/s": round(fl_b / ms / 1e9, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
