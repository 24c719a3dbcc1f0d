"""Phase breakdown of the fused MLP forward (mlp_fwd_k<256, 8>) at the C2 shape from the
s_memtime stamps of the LTHM_MLPF_STAMP=1 diagnostic build:

    bash tools/build_variant.sh STAMP recommendations_amd/csrc/mlp.hip "-DLTHM_MLPF_STAMP=1"
    LTHM_LIB_PATH=$PWD/recommendations_amd/liblthm_hip_STAMP.so python tools/mlp_stamp.py

Per wave (tiles after the first): cycles per chunk step in wait + barrier + DMA issue, S issue,
S completion, GELU + Y issue; cycles per tile epilogue; the kernel's cycles per wave against its
HIP-event time (the clock the kernel ran at)."""
import ctypes
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from recommendations_amd import _lib
    from recommendations_amd import kernels as K
    lib = _lib.load()
    fn = lib.lthm_debug_mlpf_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    dev = torch.device("cuda:0")
    M, D, HID = 4096 * 129, 256, 1024
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    x = torch.randn(M, D, device=dev, generator=g).to(bf)
    w1 = (torch.randn(HID, D, device=dev, generator=g) / math.sqrt(D)).to(bf)
    w2t = (torch.randn(D, HID, device=dev, generator=g) / math.sqrt(HID)).to(bf).T.contiguous()
    b1 = torch.randn(HID, device=dev, generator=g) * 0.1
    b2 = torch.randn(D, device=dev, generator=g) * 0.1
    r1 = torch.randn(M, D, device=dev, generator=g)
    r2 = torch.randn(M, D, device=dev, generator=g)
    out = {}
    for nres, res in (("res1", (r1,)), ("res1+res2", (r1, r2))):
        for _ in range(3):
            K.mlp_fwd(x, w1, b1, w2t, b2, *res)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        K.mlp_fwd(x, w1, b1, w2t, b2, *res)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        n = 2048 * 8 * 8
        buf = (ctypes.c_ulonglong * n)()
        assert fn(ctypes.cast(buf, ctypes.c_void_p), n) == 0
        rows = [list(buf[i * 8:(i + 1) * 8]) for i in range(256 * 8)]
        rows = [r for r in rows if r[4] > 0]
        steps = sum(r[4] for r in rows)
        tiles = sum(r[6] for r in rows)
        per = {k: sum(r[i] for r in rows) / steps for i, k in enumerate(
            ("wait_barrier_dma", "s_issue", "s_complete", "gelu_y_issue"))}
        per_tile_epi = sum(r[5] for r in rows) / max(tiles, 1)
        kcyc = sum(r[7] for r in rows) / len(rows)
        out[nres] = {"kernel_ms": round(ms, 4), "cycles_per_chunk_step": {k: round(v, 1) for k, v in per.items()},
                     "chunk_step_total": round(sum(per.values()), 1), "epilogue_cycles_per_tile": round(per_tile_epi, 1),
                     "kernel_cycles_per_wave": round(kcyc), "clock_GHz_est": round(kcyc / (ms * 1e6), 3),
                     "waves": len(rows), "steps_counted": steps}
    # the hidden backward (mlp_bwdp_k<256, 8>): wait + barrier + DMA, S / dH issue, their
    # completion, GELU' + strip writes, strip reads + G / dP store issue
    dy = torch.randn(M, D, device=dev, generator=g).to(bf)
    for _ in range(3):
        K.mlp_bwd(x, dy, w1, b1, w2t, want_dx=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    K.mlp_bwd(x, dy, w1, b1, w2t, want_dx=False)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    n = 2048 * 8 * 8
    buf = (ctypes.c_ulonglong * n)()
    assert fn(ctypes.cast(buf, ctypes.c_void_p), n) == 0
    rows = [list(buf[i * 8:(i + 1) * 8]) for i in range(256 * 8)]
    rows = [r for r in rows if r[4] > 0]
    steps = sum(r[4] for r in rows)
    per = {k: sum(r[i] for r in rows) / steps for i, k in ((0, "wait_barrier_dma"), (1, "s_dh_issue"),
                                                           (2, "s_dh_complete"), (3, "gelu_grad_strip"),
                                                           (5, "store_issue"))}
    kcyc = sum(r[7] for r in rows) / len(rows)
    out["bwd_hidden"] = {"kernel_ms": round(ms, 4), "cycles_per_chunk_step": {k: round(v, 1) for k, v in per.items()},
                         "chunk_step_total": round(sum(per.values()), 1), "kernel_cycles_per_wave": round(kcyc),
                         "clock_GHz_est": round(kcyc / (ms * 1e6), 3), "waves": len(rows), "steps_counted": steps}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
