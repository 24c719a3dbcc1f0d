"""HBM read / write / copy bandwidth probe on the GPU box: torch fill, torch copy,
the library's fill kernel and a read-only reduction, at 1-2 GB.  Prints GB/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from recommendations_amd import kernels as K
from recommendations_amd._lib import call, ptr, stream


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


def main():
    n = 1 << 28  # 1 GiB of f32
    a = torch.empty(n, dtype=torch.float32, device="cuda")
    b = torch.empty(n, dtype=torch.float32, device="cuda")
    a.normal_()
    gb = n * 4 / 1e9
    t = timed(lambda: b.zero_())
    print(f"torch zero_         write {gb / t:8.1f} GB/s")
    t = timed(lambda: call("lthm_fill_f32", ptr(b), 0.0, n, stream()))
    print(f"lthm_fill_f32       write {gb / t:8.1f} GB/s")
    t = timed(lambda: b.copy_(a))
    print(f"torch copy_   read+write {2 * gb / t:8.1f} GB/s")
    bf = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    t = timed(lambda: K.cast(a, torch.bfloat16))
    print(f"lthm_cast f32->bf16 r+w  {(gb + gb / 2) / t:8.1f} GB/s")
    acc = torch.zeros(1, dtype=torch.float32, device="cuda")
    t = timed(lambda: a.sum())
    print(f"torch sum            read {gb / t:8.1f} GB/s")


if __name__ == "__main__":
    main()
