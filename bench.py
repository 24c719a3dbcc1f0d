"""LTHM training-step benchmark (BASELINE.json metric: training samples/sec, LTHM
fwd+bwd, plus embedding HBM GB/s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c4x]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = the reference's inner training step (accelerate_training_strategy.py:
351-368): model(batch) -> train_step (fused contrastive loss) -> backward ->
DP gradient exchange (N > 1) -> optimizer steps (fused AdamW on dense params,
row-wise AdamW on the categorical KShift tables).  Inputs are synthetic batches
of the C2 shape already resident in HBM.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md): HBM3E 8.0 TB/s spec, bf16 dense MFMA 2.5 PF
HBM_PEAK_GBS = 8000.0
BF16_PEAK_TFLOPS = 2500.0
FP8_PEAK_TFLOPS = 5000.0  # dense e4m3 (block-scaled MFMA), MI355X_MICROARCH.md chip table

# Kernel-timer key (one C-ABI call) -> the gfx950 kernels that call launches, as
# named in the rocprofv3 PMC summary (tools/pmc_summary.py -> profiles/*_pmc_summary.json).
# the newest committed counter passes over the default (C2) bench
PMC_SUMMARY = next((p for p in (os.path.join(ROOT, "profiles", f"r0{r}_pmc_summary.json") for r in (6, 5, 4, 3))
                    if os.path.exists(p)), os.path.join(ROOT, "profiles", "r03_pmc_summary.json"))
PMC_KERNELS = {  # kernel-name prefixes (rocprofv3 short names) each C-ABI call key launches
    "cl_fr32_k": ["cl_fr32_k", "cl_fr32v_k"],
    "cl_bwd32_k": ["cl_bwd32_k<", "cl_bwd32v_k"],
    "cl_bwd_k": ["cl_bwd_k<", "cl_bwd32_k<", "cl_bwd32v_k", "cl_shift_k", "cl_vshift_k", "cl_dyscale_k<"],
    "cl_fwd_k": ["cl_diag_k", "cl_fwd_k<", "cl_fr32_k", "cl_fr32v_k", "cl_used_k", "cl_vpack_k", "cl_vgather_k",
                 "cl_stats_k", "cl_rowstats_k", "cl_wscale_k"],
    "lthm_layernorm_bwd": ["ln_bwd_v4_k<", "ln_bwd_k<"],
    "lthm_layernorm_fwd": ["ln_fwd_v4_k<", "ln_fwd_k<"],
    "attn_bwd_k": ["attn_bwd_mfma_k<", "attn_bwd32_k<", "attn_bwd_rows_win_k<", "attn_bwd_cols_win_k<",
                   "attn_delta_k<", "attn_bwd32l_k<"],
    "attn_fwd_k": ["attn_fwd_mfma_k<", "attn_fwd_win_k<", "attn_fwd32_k<"],
    "gemm_k<1,1>": ["gemm_k<true, true>", "gemm_ps_k<true, "],
    "gemm_k<1,0>": ["gemm_k<true, false>", "gemm_ps_k<false, "],
    "gemm_k<0,0>": ["gemm_k<false, false>", "gemm_wg_k", "splitk_reduce_k"],
    "cve_tab_bwd_k": ["cve_tab_bwd_k<", "seg_tab_reduce_k"],
    "lthm_product_tower_fwd": ["ptower_"],
    # the fused MLP calls (tagged enc:mlp_*): each is ONE kernel of one shape
    "mlp_fwd": ["mlp_fwd_k<", "mlp_fwd2_k<"],
    "mlp_bwd": ["mlp_bwdp_k<", "mlp_bwdp2_k<", "mlp_bwd_k<", "mlp_bwdx_k<"],
    "kshift_fwd_k": ["kshift_fwd_k<", "kshift_fwd_reg_k<", "kshift_fwd_k1_k<"],
    "mlp_wgrad": ["mlp_wgrad_k<"],
}
PMC_STEPS = 3  # tools/pmc_passes.sh profiles `bench.py --steps 2 --warmup 1 --no-kernel-timing`
# Timer keys that are NOT one kernel: C-ABI calls that launch several kernels (the loss calls:
# their main passes are timed alone as cl_fr32_k / cl_bwd32_k) and GEMM keys that pool several
# shapes / templates ("enc:" GEMM tags, untagged gemm_k forms).  The roofline object prices the
# single kernel with the largest share of the step, the rocprof-dominant kernel.  The fused MLP
# keys (enc:mlp_fwd / enc:mlp_bwd / enc:mlp_wgrad) ARE single kernels of a single shape per step
# (one launch per layer, every layer the same M x d x 4d), so they compete.
MULTI_KERNEL_KEYS = {"cl_fwd_k", "cl_bwd_k", "lthm_product_tower_fwd", "cve_tab_bwd_k", "attn_bwd_k"}
SINGLE_KERNEL_TAGGED = ("mlp_fwd", "mlp_bwd", "mlp_wgrad")
# the attention backward is ONE kernel (attn_bwd32_k, one workgroup per (b, h)) at T' <= 256 (C2,
# C3, C1); past that it is the rows / columns pair plus the delta pass.  Set from the config.
ATTN_BWD_SINGLE = [False]


def single_kernel_key(k: str) -> bool:
    if k.startswith("enc:"):
        return k.split(":")[-1] in SINGLE_KERNEL_TAGGED
    if k == "attn_bwd_k" and ATTN_BWD_SINGLE[0]:
        return True
    return not (k in MULTI_KERNEL_KEYS or k.startswith("gemm_k<") or k == "gemm_fp8")


# the KShift gather kernel the library launches for K = 16 / 8 (LTHM_KSHIFT_REG=1: the register-row form)
GATHER_KERNEL = "kshift_fwd_reg_k" if os.environ.get("LTHM_KSHIFT_REG", "0") == "1" else "kshift_fwd_k"
PROF_STEPS = 2  # untimed per-kernel profiling steps between warm-up and the timed region


def pmc_traffic(key, calls_per_step):
    """HBM bytes per call of `key` from the committed PMC summary: FETCH_SIZE x 2 +
    WRITE_SIZE (MI355X_MICROARCH.md §HBM) of every dispatch of the kernels the call
    launches, over the calls the profiled run made; None if not profiled."""
    try:
        with open(PMC_SUMMARY) as f:
            pmc = json.load(f)
    except OSError:
        return None
    prefixes = PMC_KERNELS.get(key, [key])
    tot = 0.0
    hit = False
    for name, v in pmc.items():
        if any(name.startswith(pf) for pf in prefixes) and "hbm_bytes" in v:
            tot += v["hbm_bytes"] * v.get("dispatches", 1)
            hit = True
    if not hit or calls_per_step <= 0:
        return None
    return tot / (calls_per_step * PMC_STEPS)


def embedding_generator_step(dev, n_catalogue=2_000_000, B=1 << 18, D=32, K=16, steps=10, warmup=3):
    """one step of the item-embedding generator's reconstruction model at the
    reference sizes (embedding_module_gen.py:122-156: KShiftEmbedding(1.15 n, D, K = 16,
    normalize) -> MSE -> loss.backward(); Adagrad(lr 0.5).step(); batches of 2^18 ids), with the
    tables stepped by the fused dedup + Adagrad (lthm_kshift_adagrad_fused) and by the two-pass
    row path, HIP events over `steps` steps after `warmup`."""
    from recommendations_amd import kernels as K_
    from recommendations_amd.commons.layers import KShiftEmbedding
    from recommendations_amd.optim import SparseRowAdagrad
    g = torch.Generator(device=dev).manual_seed(11)
    P = int(1.15 * n_catalogue)
    catalogue = torch.randint(-2 ** 63, 2 ** 63 - 1, (n_catalogue,), device=dev, generator=g, dtype=torch.int64)
    batches = [catalogue[torch.randint(0, n_catalogue, (B,), device=dev, generator=g)] for _ in range(4)]
    tgt = K_.l2norm_rows(torch.randn(B, D, device=dev, generator=g))
    res = {"model": f"KShiftEmbedding(P={P}, D={D}, K={K}, normalize) + MSE + Adagrad", "ids_per_step": B}
    for fused in (True, False):
        torch.manual_seed(0)
        emb = KShiftEmbedding(P, D, num_shifts=K, normalize_output=True, sparse=True).to(dev)
        opt = SparseRowAdagrad([emb], lr=0.5, fused=fused)
        for i in range(warmup + steps):
            if i == warmup:
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            K_.mse_loss(emb(batches[i % 4]), tgt).backward()
            opt.step()
        e1.record()
        torch.cuda.synchronize()
        res["fused_ms_per_step" if fused else "two_pass_ms_per_step"] = round(e0.elapsed_time(e1) / steps, 4)
        del emb, opt
    torch.cuda.empty_cache()
    return res


def embedding_gather_hbm(dev, P=16_000_000, D=128, K=16, n=524_288, iters=50):
    """SURVEY §8(d) embedding roofline: KShift gather + pool forward on a table far past
    the 256 MiB Infinity Cache (P x D bf16 = 4.1 GB), algorithmic bytes per lookup
    8 + K*D*2 + D*2 (bf16 out) over the HIP-event time of the kernel, for two id sets:
    ``reference_ids`` -- uniform over the full int64 range, as the reference's hashed ids
    (feature_utils.py:46); its arithmetic-shift quirk sends every shifted row (c >= 1) of a
    negative id to row P-1 (commons/layers.py:174-185), so ~47% of the row reads hit one
    cached row and the algorithmic rate exceeds what HBM could deliver; and
    ``spread_ids`` -- non-negative ids, whose K rows all land uniformly (8.4M reads of
    16M rows: ~77% of the reads touch a row once), the HBM-bound case the roofline is for."""
    from recommendations_amd import kernels as K_
    g = torch.Generator(device=dev).manual_seed(7)
    W = torch.randn((P, D), device=dev, generator=g).to(torch.bfloat16)
    per = 8 + K * D * 2 + D * 2
    res = {"kernel": GATHER_KERNEL, "table": f"P={P} D={D} bf16 ({P * D * 2 / 1e9:.2f} GB)", "K": K,
           "lookups": n, "bytes_per_lookup": per, "bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    for name, lo in (("spread_ids", 0), ("reference_ids", -(2 ** 63))):
        ids = torch.randint(lo, 2 ** 63 - 1, (n,), device=dev, generator=g, dtype=torch.int64)
        for _ in range(3):
            out = K_.kshift(ids, W, P, K, K_.KSHIFT_SCALE)
        torch.cuda.synchronize()
        # every launch between its own pair of events (the launches are back to back on the
        # stream): the median launch is the reported rate, the mean beside it
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
        evs[0].record()
        for i in range(iters):
            out = K_.kshift(ids, W, P, K, K_.KSHIFT_SCALE)
            evs[i + 1].record()
        torch.cuda.synchronize()
        per_ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(iters))
        ms = per_ms[iters // 2]
        mean_ms = sum(per_ms) / iters
        gbs = n * per / (ms / 1000.0) / 1e9
        res[name] = {"median_launch_ms": round(ms, 4), "mean_launch_ms": round(mean_ms, 4), "launches": iters,
                     "achieved": round(gbs, 1)}
        if name == "spread_ids":
            res[name]["frac"] = round(gbs / HBM_PEAK_GBS, 4)
        else:  # about half the row reads hit the one cached row P-1: algorithmic bytes exceed HBM's
            res[name]["note"] = ("algorithmic GB/s, not an HBM rate: the arithmetic-shift quirk sends ~47% of the "
                                 "row reads to one cached row, so no roofline fraction is given")
        del out
    del W
    res["achieved"], res["frac"] = res["spread_ids"]["achieved"], res["spread_ids"]["frac"]
    # HBM bytes per launch from the committed counter passes (tools/pmc_gather.sh): this round's
    # kernel when its summary is present, else round 2's
    res["traffic"] = None
    for src in ("r06_gather_pmc.json", "r02_gather_pmc.json"):
        try:
            with open(os.path.join(ROOT, "profiles", src)) as f:
                pmc = json.load(f)
            for name in ("spread_ids", "reference_ids"):
                res[name]["traffic"] = pmc[name]["hbm_bytes"]
            res["traffic"] = pmc["spread_ids"]["hbm_bytes"]
            res["traffic_source"] = (f"profiles/{src} (tools/pmc_gather.sh: rocprofv3 --pmc over tools/gather_bench.py;"
                                     f" kernel {pmc.get('kernel')})")
            break
        except (OSError, KeyError, ValueError):
            continue
    return res


CONFIGS = {
    # BASELINE.json configs[1]: LTHM on 1x MI355X, 32 cat x 1M vocab, seq 128, d 256, 4 layers, bf16, batch 4096
    "c2": dict(B=4096, T=128, d=256, L=4, H=4, n_cat=32, cat_vocab=1_000_000, item_vocab=1_000_000),
    # BASELINE.json configs[0] shape (tiny; plumbing)
    "c1": dict(B=128, T=32, d=64, L=2, H=1, n_cat=2, cat_vocab=10_000, item_vocab=10_000),
    # SURVEY §8 C3 per GPU: 100M-row item table row-sharded over the ranks, 64 categorical tables
    "c3": dict(B=4096, T=128, d=256, L=4, H=4, n_cat=64, cat_vocab=1_000_000, item_vocab=100_000_000,
               item_table_sharded=True),
    # BASELINE.json configs[4]: long history, fp8 encoder GEMMs; the reference
    # yaml's 32-sequence loss mini-batches (model/lthm.yaml:64): 32 x 512 = 16,384 logit rows
    "c5": dict(B=1024, T=512, d=512, L=6, H=8, n_cat=0, cat_vocab=1_000_000, item_vocab=1_000_000, fp8=True),
    # BASELINE.json configs[3]: ranker, 128 dense + 64 cat x 1M, interaction layers only
    "c4": dict(kind="ranker", B=65536, n_dense=128, n_cat=64, cat_vocab=1_000_000),
}


def build(cfgd, dev):
    from recommendations_amd.models.lthm.builder import LTHMModelBuilder
    from recommendations_amd.models.lthm.config import lthm_config
    torch.manual_seed(1234)  # identical replicas on every rank
    if cfgd.get("kind") == "ranker":
        from recommendations_amd.models.ranker.config import ranker_config
        # LTHM_C4_GATHER_BF16=1: the K = 1 tables gather from a bf16 shadow the row-wise step keeps
        # (the same bf16 outputs; round 5's default, A/B)
        cfg = ranker_config(n_dense=cfgd["n_dense"], n_cat=cfgd["n_cat"], cat_vocab=cfgd["cat_vocab"],
                            cat_gather_bf16=os.environ.get("LTHM_C4_GATHER_BF16", "0") == "1")
        with torch.device(dev):  # 64 x 1M x 32 tables drawn on the device
            model = cfg.get_builder().build()
        return cfg, model
    cfg = lthm_config(T=cfgd["T"], d=cfgd["d"], n_layers=cfgd["L"], n_head=cfgd["H"], cat_features=cfgd["n_cat"],
                      cat_vocab=cfgd["cat_vocab"], item_vocab=cfgd["item_vocab"],
                      item_table_sharded=cfgd.get("item_table_sharded", False), fp8=cfgd.get("fp8", False),
                      train_mini_batch_size=cfgd.get("mbs", 32), gradient_checkpointing=cfgd.get("ckpt", False))
    model = LTHMModelBuilder(None, cfg).build().to(dev)
    return cfg, model


def cpu_baseline(cfg, model, cfgd, B_cpu):
    """The oracle's CPU restatement of the same step (fwd + bwd + torch.optim.AdamW over
    all params, as wrapper.py:263-275 / accelerate_training_strategy.py:351-368), on a
    bounded sample of B_cpu sequences of the same workload."""
    from oracle import lthm_ref
    from recommendations_amd.data import synthetic_lthm_batch
    cores = cpu_cores()
    torch.set_num_threads(cores)
    train = {n for n, p in model.named_parameters() if p.requires_grad}
    sd = {k: (v.detach().float().cpu().clone().requires_grad_(k in train) if v.is_floating_point() else v.cpu())
          for k, v in model.state_dict().items() if not k.startswith("_log_q_calc")}
    params = [sd[n] for n in sorted(train)]  # dense AdamW over every trainable parameter (wrapper.py:263-275)
    opt = torch.optim.AdamW(params, lr=cfg.lr, weight_decay=cfg.weight_decay, betas=cfg.betas)
    batch = synthetic_lthm_batch(B_cpu, cfgd["T"], n_cat=cfgd["n_cat"], seed=99)
    n_mb = (B_cpu + cfg.train_mini_batch_size - 1) // cfg.train_mini_batch_size
    offs = np.array([[0, 3, 6, 9, 17, 25]] * n_mb, dtype=np.int32)

    def step():
        loss = lthm_ref.lthm_forward_loss(sd, cfg, batch, offs)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    dt = timed_median(step)
    return dict(value=round(B_cpu / dt, 3), unit="samples/s", cores=cores, kind="port",
                sample=f"{B_cpu} sequences of the {cfgd.get('name', 'C2')} workload per step, median of {CPU_TIMED} "
                       f"timed steps after {CPU_WARMUP} warm-up(s), {dt:.2f} s/step on {cores} threads (the job's "
                       f"CPU allotment; host: {lscpu_cores()}) (fp32 torch-CPU oracle: "
                       f"oracle/lthm_ref.py fwd + bwd + torch.optim.AdamW over every trainable parameter, "
                       f"1.1B with the 32 x 1M x 32 categorical tables, as the reference's dense optimizer)")


def cpu_baseline_ranker(cfg, model, cfgd, B_cpu):
    """The oracle's CPU restatement of the ranker step (oracle/ranker_ref.py fwd + BCE
    + bwd + torch.optim.AdamW over the dense parameters and the touched table rows'
    full tables), on a bounded sample of B_cpu rows of the C4 workload."""
    from oracle import ranker_ref
    from recommendations_amd.data import synthetic_ranker_batch
    cores = cpu_cores()
    torch.set_num_threads(cores)
    sd = {k: (v.detach().float().cpu().clone().requires_grad_(True) if v.is_floating_point() else v.cpu())
          for k, v in model.state_dict().items()}
    batch = synthetic_ranker_batch(B_cpu, cfg.n_dense, cfg.n_categorical, seed=99)
    # the sample's touched rows of the 64 tables, compacted: the same lookups, MLP and row
    # updates without materialising the dense gradient of all 64M rows (80-90 s a step)
    from types import SimpleNamespace
    F_, P_, D_ = cfg.n_categorical, cfg.cat_vocab, cfg.cat_emb_dim
    W = sd["_model.cat_tables.weight"].detach().view(F_, P_, D_)
    rows = [torch.unique(torch.remainder(batch["categorical"][:, f], P_)) for f in range(F_)]
    Pc = max(int(r.numel()) for r in rows)
    Wc = torch.zeros(F_, Pc, D_)
    cat = torch.empty_like(batch["categorical"])
    for f in range(F_):
        Wc[f, : rows[f].numel()] = W[f, rows[f]]
        cat[:, f] = torch.searchsorted(rows[f], torch.remainder(batch["categorical"][:, f], P_))
    sd["_model.cat_tables.weight"] = Wc.view(F_ * Pc, D_).requires_grad_(True)
    batch = dict(batch, categorical=cat)
    cfg = SimpleNamespace(**{**vars(cfg), "cat_vocab": Pc}) if hasattr(cfg, "__dict__") else cfg
    params = [v for k, v in sd.items() if v.is_floating_point() and ("emb.weight" in k or "interaction" in k)]
    tabs = [sd["_model.cat_tables.weight"]]
    opt = torch.optim.AdamW([p for p in params if p is not tabs[0]], lr=cfg.lr, weight_decay=cfg.weight_decay,
                            betas=cfg.betas)

    def step():
        loss = ranker_ref.ranker_loss(sd, cfg, batch)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        with torch.no_grad():  # plain SGD-style row update of the touched table rows (bounded CPU work)
            g = tabs[0].grad
            tabs[0].sub_(cfg.lr * g)
            tabs[0].grad = None

    dt = timed_median(step)
    return dict(value=round(B_cpu / dt, 3), unit="samples/s", cores=cores, kind="port",
                sample=f"{B_cpu} rows of the C4 workload per step, median of {CPU_TIMED} timed steps after "
                       f"{CPU_WARMUP} warm-up(s), {dt:.3f} s/step on {cores} threads (host: {lscpu_cores()}) "
                       f"(fp32 torch-CPU oracle: oracle/ranker_ref.py + "
                       f"torch.optim.AdamW on the dense parameters; the 64 tables compacted to the sample's "
                       f"touched rows, row update on those)")


CPU_WARMUP, CPU_TIMED = 1, 3  # BASELINE.md plans 2 + 5; at 256 sequences (~12 s a step) 1 + 3 keeps the run short


def launch_ranks(n: int) -> int:
    """Run this script as n ranks on one node (torch.distributed.run, rendezvous on
    127.0.0.1 at a free port); return the launcher's exit status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def lscpu_cores() -> str:
    """The host's core count as lscpu reports it (sockets x cores per socket), for the record."""
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = dict(l.split(":", 1) for l in out.splitlines() if ":" in l)
        sockets = int(kv.get("Socket(s)", "1").strip())
        cps = int(kv.get("Core(s) per socket", "0").strip())
        return f"{sockets * cps} physical cores ({kv.get('Model name', '?').strip()})"
    except Exception:  # lscpu absent: report nothing rather than guess
        return "lscpu unavailable"


def cpu_cores() -> int:
    """The host cores this job may use: OMP_NUM_THREADS when the launcher sets it (the GPU
    box allots 16 CPUs per GPU and exports it), else the process's CPU affinity."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def timed_median(step) -> float:
    """BASELINE.md CPU plan: 2 warm-ups, then the median of 5 timed steps (seconds)."""
    for i in range(CPU_WARMUP):
        step()
        print(f"[cpu_baseline] warm-up {i + 1}/{CPU_WARMUP}", file=sys.stderr, flush=True)
    ts = []
    for i in range(CPU_TIMED):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
        print(f"[cpu_baseline] step {i + 1}/{CPU_TIMED}: {ts[-1]:.2f} s", file=sys.stderr, flush=True)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-prefetch", action="store_true",
                    help="C3 at N > 1: look the row-sharded item table up inside each step instead of one "
                         "step ahead on a side stream")
    ap.add_argument("--batch", type=int, default=0, help="override per-GPU batch")
    ap.add_argument("--batches", type=int, default=4, help="distinct resident batches, used in turn")
    ap.add_argument("--checkpointing", action="store_true",
                    help="recompute block activations in the backward (the reference yaml's "
                         "enable_gradient_checkpointing, a memory knob; off by default: the "
                         "activations fit in 288 GB of HBM)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=0,
                    help="CPU-baseline sample (sequences); default per BASELINE.md: C2 256, C5 16, C1 the batch")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-hbm-gather", action="store_true", help="skip the 1 GB-table embedding roofline")
    ap.add_argument("--no-generator", action="store_true",
                    help="skip the item-embedding generator step (fused vs two-pass Adagrad)")
    ap.add_argument("--check-launch", action="store_true",
                    help="form the process group, print the world size it reports and exit (launcher test)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N`: this parent never touches the GPU; it starts one rank
        # per GPU through torch.distributed.run and exits with its status
        sys.exit(launch_ranks(args.gpus))

    from recommendations_amd import _lib
    from recommendations_amd.data import synthetic_lthm_batch, synthetic_ranker_batch
    from recommendations_amd.distributed import GradBucketAllReduce, init_from_env, step_flags

    rank, local, world = init_from_env()
    reported = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    if world != args.gpus or reported != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world} and the process group has {reported} ranks")
    if args.check_launch:
        if world > 1:
            t = torch.ones(1)
            torch.distributed.all_reduce(t)  # every rank joined the group
            if rank == 0:
                print(json.dumps({"world": reported, "backend": torch.distributed.get_backend(), "sum": float(t)}))
            torch.distributed.destroy_process_group()
        else:
            print(json.dumps({"world": 1, "backend": None, "sum": 1.0}))
        return
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    cfgd = dict(CONFIGS[args.config], name=args.config.upper())
    ATTN_BWD_SINGLE[0] = cfgd.get("T") is not None and cfgd["T"] + 1 <= 256
    if args.batch:
        cfgd["B"] = args.batch
    cfgd["ckpt"] = bool(args.checkpointing)
    cfg, model = build(cfgd, dev)
    B = cfgd["B"]
    ranker = cfgd.get("kind") == "ranker"
    if world > 1:
        if ranker:
            model._model.cat_tables.replicated_dp = True
        elif model._model.user_context is not None:
            # table-wise sharding of the categorical tables (all_to_all routing, no xworld
            # growth of the sparse backward / optimizer); before the optimizers are built
            model._model.user_context.shard_tables(rank, world)
    opts = model.optimizers_for_param_groups(model.param_groups())
    dense_params = [p for n, p in model.named_parameters() if p.requires_grad and not model.is_sparse(n)]
    allreduce = GradBucketAllReduce(dense_params)
    # a pool of distinct HBM-resident batches, one per step in turn (different ids, pads and
    # lengths every step: the gathers, the dedup and the sparse updates see new rows)
    nb = max(1, args.batches)
    if ranker:
        pool = [synthetic_ranker_batch(B, cfgd["n_dense"], cfgd["n_cat"], seed=1234 + 7919 * i, rank=rank, device=dev)
                for i in range(nb)]
    else:
        pool = [synthetic_lthm_batch(B, cfgd["T"], n_cat=cfgd["n_cat"], seed=1234 + 7919 * i, rank=rank, device=dev)
                for i in range(nb)]
    cursor = [0]

    # C3 on N > 1 GPUs: the row-sharded item table's lookup of the next step (routing, the
    # count exchange the host reads, two all_to_alls on a communicator of their own) runs on
    # a side stream, issued right after this step's backward has been enqueued, at the same
    # point on every rank (Encoder.prefetch): the side stream waits only for the batch's ids
    # (batch_ready), and the host's blocking read of the exchanged counts then overlaps the
    # backward already queued on the main stream.  On one GPU (and for the replicated table) the inline lookup
    # is as fast: C2 74,964 vs 74,871, C3 71,911 vs 71,185 samples/s inline vs prefetched
    # (profiles/r02_prefetch_ab.log)
    pipelined = bool(cfgd.get("item_table_sharded")) and world > 1 and not args.no_prefetch
    batch_ready = torch.cuda.Event()
    batch_ready.record()  # the synthetic batch is resident from here on
    if pipelined:
        model.prefetch(pool[0], batch_ready)

    def step():
        batch = pool[cursor[0] % nb]
        cursor[0] += 1
        out = model(batch)
        loss, _ = model.train_step(batch, out)
        loss.backward()
        if pipelined:  # after the backward is enqueued: the count read overlaps it
            model.prefetch(pool[cursor[0] % nb], batch_ready)
        allreduce()
        flags = step_flags(False, loss)
        for o in opts:
            o.step()
            o.zero_grad(set_to_none=True)
        return loss, flags

    for _ in range(args.warmup):
        loss, flags = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    prof = None
    if not args.no_kernel_timing:
        # per-kernel breakdown from untimed profiling steps (every entry point bracketed
        # by HIP events); the timed region then brackets only the dominant kernel, whose
        # live average launch time prices the roofline (events on every launch would
        # cost ~3 ms of a ~60 ms step)
        _lib.TIMER = _lib.KernelTimer()
        for _ in range(PROF_STEPS):
            loss, flags = step()
        torch.cuda.synchronize()
        prof, _lib.TIMER = _lib.TIMER.summary(), None
        dom_key = max((k for k in prof if single_kernel_key(k)), key=lambda k: prof[k]["ms"])
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        _lib.TIMER = _lib.KernelTimer(only=[dom_key])
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, flags = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    timer, _lib.TIMER = _lib.TIMER, None
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    assert float(flags[1]) == 0.0, "non-finite loss"
    samples = B * world * args.steps
    res = {
        "metric": ("training samples/sec (ranker C4 fwd+bwd)" if ranker else
                   "training samples/sec (LTHM fwd+bwd) at 1/2/4/8 MI355X; embedding HBM GB/s"),
        "value": round(samples / dt, 2),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * dt / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp8-e4m3 fwd GEMMs / bf16" if cfgd.get("fp8") else "bf16",
        "data": ("synthetic (N(0,1) dense features, uniform int64 categorical ids, Bernoulli(0.1) clicks); "
                 "random-init weights" if ranker else
                 "synthetic (seeded full-range int64 item ids with 0-padding, labels 0..3, 2023 timestamps, "
                 "uniform int64 categorical ids); random-init weights"),
        "config": {"workload": (f"ranker C4: {cfgd['n_dense']} dense -> DenseMapper(16 proj x 20 bins) + "
                                f"{cfgd['n_cat']} cat x {cfgd['cat_vocab']} FlatEmbedding D=32 -> MLP [1024, 512] -> 1, "
                                f"QuickGELU, BCE" if ranker else
                                f"LTHM {args.config.upper()}: item KShift P={cfgd['item_vocab']} D=32 K=16, "
                                f"{cfgd['n_cat']} cat x {cfgd['cat_vocab']} KShift D=32 K=8, T={cfgd['T']}, "
                                f"d={cfgd['d']}, {cfgd['L']} layers, H={cfgd['H']}, 6 lookahead heads"
                                + (", fp8 e4m3 forward encoder GEMMs" if cfgd.get("fp8") else "")
                                + (f", {cfgd['mbs']}-sequence loss mini-batches" if cfgd.get("mbs") else "")),
                   "global_batch": B * world, "per_gpu_batch": B, "seq_len": cfgd.get("T"),
                   "activation_checkpointing": cfgd["ckpt"],
                   "activation_checkpointing_note": ("the reference yaml (model/lthm.yaml:53) recomputes every block in "
                                                     "the backward; this line runs without it unless --checkpointing "
                                                     "(a memory knob the 288 GB part does not need)"),
                   "distinct_batches": nb,
                   "item_lookup": ("one step ahead on a side stream (Encoder.prefetch after the backward is "
                                   "enqueued), "
                                   "inside the timed loop"
                                   if pipelined else "inline"),
                   "parallelism": f"dp{world}" + (
                       (" (item table row-sharded, all_to_all row exchange; categorical tables table-wise "
                        "sharded, all_to_all id / row / gradient routing; dense grads bucketed all-reduce "
                        "overlapped with the backward)" if cfgd.get("item_table_sharded") else
                        " (categorical tables table-wise sharded, all_to_all id / row / gradient routing; dense "
                        "grads bucketed all-reduce overlapped with the backward)") if world > 1 else "")},
        "final_loss": round(float(loss), 5),
    }
    if timer is not None:
        summ = prof
        kern = {}
        # the sub-kernel keys (a pass inside a multi-kernel call) are not added to the total twice
        prof_ms = sum(v["ms"] for k, v in prof.items() if k not in ("cl_fr32_k", "cl_bwd32_k", "cl_fwd_main"))
        for k, s in summ.items():
            avg_ms = s["ms"] / s["calls"]
            e = {"calls_per_step": s["calls"] / PROF_STEPS, "avg_ms": round(avg_ms, 4),
                 "share": round(s["ms"] / prof_ms, 4)}
            if s.get("bytes"):
                # roofline of the form: the larger of its MFMA time and its compulsory-HBM time
                pk = FP8_PEAK_TFLOPS if "fp8" in k else BF16_PEAK_TFLOPS
                t_roof = max(s["work"] / (pk * 1e12), s["bytes"] / (HBM_PEAK_GBS * 1e9))
                e["flop_per_byte"] = round(s["work"] / s["bytes"], 1)
                e["frac_roofline"] = round(t_roof / (s["ms"] / 1000.0), 4)
            if s["work"]:
                rate = s["work"] / (s["ms"] / 1000.0)
                if s["unit"] == "byte":
                    e["GB/s"] = round(rate / 1e9, 1)
                    e["frac_hbm_peak"] = round(rate / 1e9 / HBM_PEAK_GBS, 4)
                else:
                    pk = FP8_PEAK_TFLOPS if "fp8" in k else BF16_PEAK_TFLOPS
                    e["TFLOP/s"] = round(rate / 1e12, 1)
                    e["frac_peak"] = round(rate / 1e12 / pk, 4)
                    e["peak_TFLOP/s"] = pk
            kern[k] = e
        enc = {k: v for k, v in summ.items() if k.startswith("enc:")}
        if enc:
            # north-star MFMA target: every encoder GEMM (QKV, proj, FFN; fwd, dgrad, wgrad),
            # flop-weighted: time the flops would take at each form's dense peak / time taken
            at_peak = sum(v["work"] / ((FP8_PEAK_TFLOPS if "fp8" in k else BF16_PEAK_TFLOPS) * 1e12)
                          for k, v in enc.items())
            t = sum(v["ms"] for v in enc.values()) / 1000.0
            fl = sum(v["work"] for v in enc.values())
            roof = sum(max(v["work"] / ((FP8_PEAK_TFLOPS if "fp8" in k else BF16_PEAK_TFLOPS) * 1e12),
                           v.get("bytes", 0.0) / (HBM_PEAK_GBS * 1e9)) for k, v in enc.items())
            res["encoder_gemm"] = {"bound": "mfma", "achieved": round(fl / t / 1e12, 1), "unit": "TFLOP/s",
                                   "frac": round(at_peak / t, 4),
                                   "peak": FP8_PEAK_TFLOPS if all("fp8" in k for k in enc) else BF16_PEAK_TFLOPS,
                                   "frac_roofline": round(roof / t, 4),
                                   "flop_per_step": round(fl / PROF_STEPS / 1e12, 3),
                                   "ms_per_step": round(1000 * t / PROF_STEPS, 3),
                                   "forms": sorted(enc),
                                   "note": "all TransformerBlock GEMMs (c_attn, c_proj, c_fc, mlp.c_proj; forward, "
                                           "dgrad, wgrad), algorithmic 2MNK flop over HIP-event kernel time; "
                                           "frac_roofline: per form max(flop / MFMA peak, compulsory HBM bytes / "
                                           "HBM peak) summed, over the time taken (K = 528k-row weight gradients "
                                           "sit below the ridge point)"}

            def split(pred, note):
                sub = {k: v for k, v in enc.items() if pred(k)}
                if not sub:
                    return None
                ts = sum(v["ms"] for v in sub.values()) / 1000.0
                pk_s = sum(v["work"] / ((FP8_PEAK_TFLOPS if "fp8" in k else BF16_PEAK_TFLOPS) * 1e12)
                           for k, v in sub.items())
                o = {"achieved": round(sum(v["work"] for v in sub.values()) / ts / 1e12, 1), "unit": "TFLOP/s",
                     "frac": round(pk_s / ts, 4), "ms_per_step": round(1000 * ts / PROF_STEPS, 3),
                     "flop_per_step": round(sum(v["work"] for v in sub.values()) / PROF_STEPS / 1e12, 3),
                     "forms": sorted(sub), "note": note}
                nbytes = sum(v.get("bytes", 0.0) for v in sub.values())
                if nbytes:
                    o["declared_bytes_per_step"] = round(nbytes / PROF_STEPS)
                return o
            # the MFMA fraction of the plain GEMM kernels alone, and the fused
            # forms beside it (their LayerNorm / GELU work and bytes are inside their time)
            plain = lambda k: k.split(":")[-1].startswith("gemm")  # noqa: E731
            subs = {"gemm_only": split(plain, "plain GEMM kernels (gemm_ps_k / gemm_wg_k / gemm_pp_k forms with "
                                               "bias / activation epilogues only): forward, dgrad and weight "
                                               "gradients of c_attn and c_proj, and every form the fused MLP "
                                               "does not cover"),
                    "fused_mlp": split(lambda k: k.split(":")[-1].startswith("mlp"),
                                       "mlp_fwd (c_fc -> GELU -> c_proj, hidden on chip) and mlp_bwd (hidden "
                                       "recomputed, G / dP written): their flops are the GEMMs', their time "
                                       "includes the GELU / GELU' work"),
                    "layernorm_fused": split(lambda k: k.split(":")[-1] in ("dgrad_ln", "linear_ln"),
                                             "GEMMs whose 256-column tiles finish a LayerNorm (c_fc / c_attn dgrad "
                                             "+ ln backward, c_proj + ln_2 forward): flops are the GEMMs', the "
                                             "LayerNorm's HBM bytes are declared_bytes_per_step")}
            for kk, vv in subs.items():
                if vv is not None:
                    res["encoder_gemm"][kk] = vv
        live = timer.summary()
        dom = max((k for k in live if single_kernel_key(k)), key=lambda k: live[k]["ms"])
        s = live[dom]
        avg_s = s["ms"] / s["calls"] / 1000.0
        per_launch = (s["work"] or 0.0) / s["calls"]
        pk_mfma = FP8_PEAK_TFLOPS if "fp8" in dom else BF16_PEAK_TFLOPS
        # a GEMM form declares flops AND its compulsory HBM bytes: it is priced against the
        # roof that binds it (K = 256 encoder GEMMs sit below the ridge point: HBM)
        hbm_bound_gemm = (s["unit"] != "byte" and s.get("bytes") and s["work"] and
                          s["bytes"] / (HBM_PEAK_GBS * 1e9) > s["work"] / (pk_mfma * 1e12))
        if s["unit"] == "byte" or hbm_bound_gemm:
            nb = (s["bytes"] if hbm_bound_gemm else (s["work"] or 0.0)) / s["calls"]
            ach, peak, unit, bound = nb / avg_s / 1e9, HBM_PEAK_GBS, "GB/s", "hbm"
        else:
            peak = pk_mfma
            ach, unit, bound = per_launch / avg_s / 1e12, "TFLOP/s", "mfma"
        both = {}
        if s["unit"] != "byte" and s.get("bytes") and s["work"]:
            # a kernel that declares flops AND compulsory bytes: both fractions, the binding one in `frac`
            both = {"mfma_frac": round(per_launch / avg_s / 1e12 / pk_mfma, 4),
                    "hbm_frac": round(s["bytes"] / s["calls"] / avg_s / 1e9 / HBM_PEAK_GBS, 4),
                    "flop_per_launch": per_launch, "bytes_per_launch": s["bytes"] / s["calls"]}
        if ":" in dom and prof is not None:
            # a tagged GEMM form (enc:...): the counters see the kernel, not the tag, so the
            # traffic is the form's average over all its launches (tagged or not)
            base = dom.split(":")[-1]
            fam = sum(v["calls"] for k, v in prof.items() if k.split(":")[-1] == base) / PROF_STEPS
            traffic = pmc_traffic(base, fam)
        else:
            traffic = pmc_traffic(dom, s["calls"] / args.steps)
        if args.config != "c2" or args.batch or world > 1:
            traffic = None  # the committed counter passes profile the default (C2, one GPU) run only
        res["roofline"] = {"kernel": dom, "bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit,
                           "frac": round(ach / peak, 4),
                           "traffic": round(traffic) if traffic is not None else None,
                           "traffic_unit": "bytes/launch (HBM, rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                           "traffic_source": os.path.relpath(PMC_SUMMARY, ROOT) if traffic is not None else None,
                           "avg_launch_ms": round(s["ms"] / s["calls"], 4), **both}
        if "kshift_fwd_k" in summ:
            g = summ["kshift_fwd_k"]
            res["embedding_gather_c2"] = {"kernel": GATHER_KERNEL, "bound": "hbm",
                                          "note": "C2 tables (64 MB item, 32 x 64 MB cat) are Infinity-Cache resident",
                                          "achieved": round(g["work"] / (g["ms"] / 1000) / 1e9, 1),
                                          "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                          "frac": round(g["work"] / (g["ms"] / 1000) / 1e9 / HBM_PEAK_GBS, 4)}
        if rank == 0 and not args.no_hbm_gather:
            res["embedding_gather"] = embedding_gather_hbm(dev)
        if rank == 0 and not args.no_generator and args.config == "c2":
            res["embedding_generator"] = embedding_generator_step(dev)
        res["kernels"] = kern
        res["kernels_source"] = (f"{PROF_STEPS} untimed profiling steps after warm-up (HIP events around every "
                                 f"entry point; share = fraction of the summed kernel time); the roofline kernel "
                                 f"is re-timed live inside the timed region")
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not cfgd.get("item_table_sharded"):
        cpu_b = args.cpu_batch or {"c2": 256, "c5": 16}.get(args.config, min(B, 256))
        res["cpu_baseline"] = (cpu_baseline_ranker(cfg, model, cfgd, 32768) if ranker else
                               cpu_baseline(cfg, model, cfgd, cpu_b))
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
