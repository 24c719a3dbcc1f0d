"""Build recommendations_amd/liblthm_torch_ops.so: the TORCH_LIBRARY(lthm) op layer
(lthm_ops.cpp) over liblthm_hip.so, in-tree so it travels to the GPU box with the
snapshot.  Host code only (no device code): hipcc compiles it against torch's
headers and links torch's libraries and liblthm_hip.so (rpath $ORIGIN).

    python recommendations_amd/csrc/torch_ops/build.py
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(os.path.dirname(HERE))
SRC = os.path.join(HERE, "lthm_ops.cpp")
OUT = os.path.join(PKG, "liblthm_torch_ops.so")
HEADER = os.path.join(os.path.dirname(PKG), "include", "lthm.h")


def build(force: bool = False) -> str:
    deps = [SRC, HEADER, os.path.join(PKG, "liblthm_hip.so")]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    import torch
    import torch.utils.cpp_extension as ce
    inc = sum((["-isystem", p] for p in ce.include_paths(device_type="cuda")), [])
    libdirs = ce.library_paths(device_type="cuda")
    cmd = ["/opt/rocm/bin/hipcc", "-O2", "-fPIC", "-shared", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}", *inc, SRC, "-o", OUT + ".tmp",
           *[f"-L{d}" for d in libdirs], "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
           f"-L{PKG}", "-llthm_hip", "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{libdirs[0]}"]
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
