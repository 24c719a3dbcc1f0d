"""Microbenchmark of the small-table (CVE / EmbeddingBag) backward on the C2
product-tower shape (524,288 tokens, D = 256, 6 CVE modules x 32 projections +
histogram slot) under different row-index distributions."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendations_amd import kernels as K  # noqa: E402


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def layout():
    segs, so, ro, offs = [], 0, 0, []
    for nb in (2, 4, 8, 12, 16, 20):
        rps = nb + 1
        segs += K.cve_segments(32, rps, so, ro)
        offs += [(ro + p * rps, rps) for p in range(32)]
        so += 32
        ro += rps * 32
    segs.append((so, 1, ro, 20))
    offs.append((ro, 20))
    return segs, offs, ro + 20


def main():
    dev = torch.device("cuda")
    n, D = int(os.environ.get("N", 524288)), 256
    segs, offs, R = layout()
    g = torch.Generator(device=dev).manual_seed(0)
    dy = torch.randn((n, D), device=dev, generator=g).to(torch.bfloat16)
    cases = {}
    # uniform buckets
    cols = [o + torch.randint(0, r, (n,), device=dev, generator=g) for o, r in offs]
    cases["uniform"] = torch.stack(cols, 1)
    # concentrated: 2 central buckets per slot, random order
    cols = [o + (r // 2) - torch.randint(0, 2, (n,), device=dev, generator=g).clamp(max=r - 1) for o, r in offs]
    cases["two_buckets"] = torch.stack(cols, 1)
    # one bucket per slot (all tokens identical, e.g. pads)
    cols = [torch.full((n,), o + r // 2, device=dev, dtype=torch.int64) for o, r in offs]
    cases["one_bucket"] = torch.stack(cols, 1)
    for name, rows in cases.items():
        rows16 = rows.to(torch.int32).to(torch.int16).contiguous()
        t = timeit(lambda: K.segmented_table_bwd(rows16, dy, R, segs))
        print(f"{name:12s} n={n} slots={rows.shape[1]} R={R} D={D}: {t:.3f} ms "
              f"({n * rows.shape[1] / t / 1e6:.2f} G slot-updates/s)", flush=True)
    mods, so, ro = [], 0, 0
    for nb in (2, 4, 8, 12, 16, 20):
        mods.append((so, 32, ro, nb + 1))
        so += 32
        ro += (nb + 1) * 32
    mods.append((so, 1, ro, 20))
    for name, rows in cases.items():
        rows16 = rows.to(torch.int32).to(torch.int16).contiguous()
        t = timeit(lambda: K.cve_table_bwd(rows16, dy, R, mods))
        fl = 2.0 * n * D * R
        print(f"MFMA one-hot {name:12s}: {t:.3f} ms ({fl / t / 1e9:.0f} TFLOP/s one-hot)", flush=True)
    # scaling probes: columns, tokens, segments
    rows16 = cases["uniform"].to(torch.int32).to(torch.int16).contiguous()
    for Dp in (64, 128):
        t = timeit(lambda: K.segmented_table_bwd(rows16, dy[:, :Dp].contiguous(), R, segs))
        print(f"uniform D={Dp}: {t:.3f} ms", flush=True)
    for nn in (65536, 131072):
        t = timeit(lambda: K.segmented_table_bwd(rows16[:nn].contiguous(), dy[:nn].contiguous(), R, segs))
        print(f"uniform n={nn}: {t:.3f} ms", flush=True)
    t = timeit(lambda: K.segmented_table_bwd(rows16, dy, R, segs[:1]))
    print(f"uniform first segment only {segs[0]}: {t:.3f} ms", flush=True)
    t = timeit(lambda: K.segmented_table_bwd(rows16, dy, R, segs[-1:]))
    print(f"uniform last (histogram) segment only {segs[-1]}: {t:.3f} ms", flush=True)
    dz = torch.zeros_like(dy)
    rows16 = cases["one_bucket"].to(torch.int32).to(torch.int16).contiguous()
    t = timeit(lambda: K.segmented_table_bwd(rows16, dz, R, segs))
    print(f"one_bucket, zero dY: {t:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
