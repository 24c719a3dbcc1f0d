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
    ap.add_argument("--only", default="", help="comma list of backward entries to time (profiling), e.g. bwd_dx,bwd_wgrad")
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
    only = set(filter(None, args.only.split(",")))
    for name, fn in ((((("unfused_fwd", unfused),) if not args.fused_only else ()) + (("fused_fwd", fused),))
                     if not only else ()):
        ms = timed(fn, args.iters)
        out[name] = {"ms": round(ms, 4), "TFLOP/s": round(fl / ms / 1e9, 1), "frac_bf16_peak": round(fl / ms / 1e9 / 2500, 4)}
    if (args.bwd or only) and hasattr(K, "mlp_bwd"):
        dy = torch.randn(M, D, device=dev, generator=g).to(bf)
        fl_b = 7.0 * 2 * M * D * HID  # executed (recompute 1 + dH 1 + dX 1 + dW 2 + recompute 2)
        if not only:
            ms = timed(lambda: K.mlp_bwd(x, dy, w1, b1, w2t), args.iters)
            out["fused_bwd"] = {"ms": round(ms, 4), "alg_TFLOP/s": round(8.0 * M * D * HID / ms / 1e9, 1),
                                "exec_TFLOP/s": round(fl_b / ms / 1e9, 1)}
        u = 2.0 * M * D * HID  # one unit: a [M, D] x [D, HID] product

        def chain4():  # round 4: G / dP written, dX GEMM, two weight-gradient GEMMs, db1 colsum
            dx, G, dP = K.mlp_bwd(x, dy, w1, b1, w2t)
            return dx, K.linear_wgrad(dP, x), K.linear_wgrad(dy, G), K.colsum(dP)

        def chain5():  # round 5: dX and the weight gradients by two recompute kernels, nothing in HBM
            return K.mlp_bwd_dx(x, dy, w1, b1, w2t), K.mlp_wgrad(x, dy, w1, b1, w2t)
        for name, fn, parts in (("bwd_chain_r4", chain4, None),
                                ("bwd_chain_r5", chain5, None),
                                ("bwd_hidden", lambda: K.mlp_bwd(x, dy, w1, b1, w2t, want_dx=False), 2.0),
                                ("bwd_dx", lambda: K.mlp_bwd_dx(x, dy, w1, b1, w2t), 3.0),
                                ("bwd_wgrad", lambda: K.mlp_wgrad(x, dy, w1, b1, w2t), 4.0)):
            if only and name not in only:
                continue
            ms = timed(fn, args.iters)
            e = {"ms": round(ms, 4), "alg_TFLOP/s": round(8.0 * M * D * HID / ms / 1e9, 1)}
            if parts:
                e["exec_TFLOP/s"] = round(parts * u / ms / 1e9, 1)
                e["frac_bf16_peak"] = round(parts * u / ms / 1e9 / 2500, 4)
            out[name] = e
    print(json.dumps(out))


if __name__ == "__main__":
    main()
