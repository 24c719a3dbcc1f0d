"""Write-bandwidth ceilings of GEMM-shaped outputs (tools/write_probe.hip): 128 x 128
bf16 tiles by tile order, persistent vs one tile per workgroup, against full-row writes
and torch's fill.  Build here: python tools/write_probe.py --build; run on the box."""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "write_probe.so")

if "--build" in sys.argv:
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                           os.path.join(HERE, "write_probe.hip"), "-o", SO])
    sys.exit(0)

sys.path.insert(0, HERE)
import torch  # noqa: E402
from gemm_bench import timeit  # noqa: E402

lib = ctypes.CDLL(SO)
dev = torch.device("cuda")
s = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
M = 4096 * 128
for N in (1024, 256, 768):
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    nb = out.numel() * 2
    p = ctypes.c_void_p(out.data_ptr())
    res = []
    for name, fn in [
        ("tile row-major", lambda: lib.probe_tile(p, ctypes.c_int64(M), ctypes.c_int64(N), 0, s())),
        ("tile col-major", lambda: lib.probe_tile(p, ctypes.c_int64(M), ctypes.c_int64(N), 1, s())),
        ("persist256 row-major", lambda: lib.probe_persist(p, ctypes.c_int64(M), ctypes.c_int64(N), 0, 256, s())),
        ("persist1024 row-major", lambda: lib.probe_persist(p, ctypes.c_int64(M), ctypes.c_int64(N), 0, 1024, s())),
        ("persist256 col-major", lambda: lib.probe_persist(p, ctypes.c_int64(M), ctypes.c_int64(N), 1, 256, s())),
        ("full rows", lambda: lib.probe_rows(p, ctypes.c_int64(M), ctypes.c_int64(N), s())),
        ("torch fill", lambda: out.fill_(1.0)),
    ]:
        t = timeit(fn)
        res.append(f"{name} {nb / t / 1e6:6.0f}")
    print(f"N={N}: " + " | ".join(res) + " GB/s", flush=True)
