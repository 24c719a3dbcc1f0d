"""Host-side issue time of the C2 training step vs its GPU time: times how long the
Python loop takes to enqueue K steps (no sync inside) and the wall time until the GPU
has finished them.  Issue time close to the GPU time means a host-bound step.
python tools/host_overhead.py [--config c2] [--steps 10]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--find-sync", action="store_true",
                    help="run one step under torch.cuda.set_sync_debug_mode('error') and print where it syncs")
    ap.add_argument("--callsites", default="",
                    help="comma-separated C-ABI names (e.g. lthm_fill_f32,lthm_cast): count their "
                         "callers (first frame outside kernels.py / _lib.py) over one step")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfgd = dict(bench.CONFIGS[args.config])
    cfg, model = bench.build(cfgd, dev)
    opts = model.optimizers_for_param_groups(model.param_groups())
    from recommendations_amd.data import synthetic_lthm_batch, synthetic_ranker_batch
    if cfgd.get("kind") == "ranker":
        batch = synthetic_ranker_batch(cfgd["B"], cfgd["n_dense"], cfgd["n_cat"], seed=1234, rank=0, device=dev)
    else:
        batch = synthetic_lthm_batch(cfgd["B"], cfgd["T"], n_cat=cfgd["n_cat"], seed=1234, rank=0, device=dev)

    def step():
        out = model(batch)
        loss, _ = model.train_step(batch, out)
        loss.backward()
        for o in opts:
            o.step()
            o.zero_grad(set_to_none=True)
        return loss

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    if args.find_sync:
        import traceback
        torch.cuda.set_sync_debug_mode("error")
        try:
            step()
            print("no synchronizing torch call in the step")
        except RuntimeError:
            traceback.print_exc(limit=12)
        finally:
            torch.cuda.set_sync_debug_mode("default")
        torch.cuda.synchronize()
    if args.callsites:
        import collections
        import traceback
        from recommendations_amd import _lib
        want = set(args.callsites.split(","))
        seen = collections.Counter()
        real = _lib.call

        def counting(name, *a, **kw):
            if name in want:
                fr = [f for f in traceback.extract_stack()[:-1]
                      if not f.filename.endswith(("kernels.py", "_lib.py"))]
                f = fr[-1]
                seen[(name, f"{os.path.relpath(f.filename)}:{f.lineno}")] += 1
            return real(name, *a, **kw)
        mods = [m for m in list(sys.modules.values()) if getattr(m, "call", None) is real]
        for m in mods:
            m.call = counting
        step()
        torch.cuda.synchronize()
        for m in mods:
            m.call = real
        for (name, site), c in seen.most_common():
            print(f"callsite {c:4d}  {name:24s} {site}")
    # host time per phase in steady state (a phase that blocks on the GPU shows up here)
    phases = {"forward": 0.0, "train_step": 0.0, "backward": 0.0, "optimizer": 0.0}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ta = time.perf_counter()
        out = model(batch)
        tb = time.perf_counter()
        loss, _ = model.train_step(batch, out)
        tc = time.perf_counter()
        loss.backward()
        td = time.perf_counter()
        for o in opts:
            o.step()
            o.zero_grad(set_to_none=True)
        te = time.perf_counter()
        phases["forward"] += tb - ta
        phases["train_step"] += tc - tb
        phases["backward"] += td - tc
        phases["optimizer"] += te - td
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    # the issue time of one step on its own, GPU idle at the start (a lower bound on the host cost)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    step()
    t_one = time.perf_counter() - t1
    torch.cuda.synchronize()
    print(json.dumps({"config": args.config, "steps": args.steps,
                      "issue_ms_per_step": round(1e3 * t_issue / args.steps, 3),
                      "wall_ms_per_step": round(1e3 * t_all / args.steps, 3),
                      "issue_ms_single_step": round(1e3 * t_one, 3),
                      "phase_ms_per_step": {k: round(1e3 * v / args.steps, 3) for k, v in phases.items()},
                      "host_cpus": os.cpu_count()}))


if __name__ == "__main__":
    main()
