# Round-4 GPU pass s: SQ / TCC counters of the fused MLP forward and backward-hidden kernels (C2 shape)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04s
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/r04s/p1 -o run --output-format csv -- python3 tools/mlp_bench.py --fused-only --bwd --iters 3 > gpurun_out/r04s/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-trace -d gpurun_out/r04s/p2 -o run --output-format csv -- python3 tools/mlp_bench.py --fused-only --bwd --iters 3 > gpurun_out/r04s/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r04s/p3 -o run --output-format csv -- python3 tools/mlp_bench.py --fused-only --bwd --iters 3 > gpurun_out/r04s/p3.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/r04s/pmc.json gpurun_out/r04s/p1 gpurun_out/r04s/p2 gpurun_out/r04s/p3
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r04s/pmc.json"))
for k, v in d.items():
    if "mlp" in k or "gemm" in k:
        print(k, {c: f"{x:.3e}" for c, x in sorted(v.items())})
PY
grep -h "fused" gpurun_out/r04s/p1.log | head -3
rm -rf gpurun_out/r04s/p1 gpurun_out/r04s/p2 gpurun_out/r04s/p3
# C2 bench kernel trace (rocprof view of every kernel, for the loss auxiliaries)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04s/c2 -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/r04s/c2.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find gpurun_out/r04s/c2 -name "*.db" | head -1) 45 > gpurun_out/r04s/c2_kernel_stats.txt 2>&1 || find gpurun_out/r04s/c2 | head
head -45 gpurun_out/r04s/c2_kernel_stats.txt
find gpurun_out/r04s/c2 -name "*stats*" | head
