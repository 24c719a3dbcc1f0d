# Round-4 GPU pass u: swizzled MLP backward strips (mlp tests + microbench), then LDS bank-conflict
# and wave-cycle counters of every kernel of a C2 step
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04u
export PARITY_LOG=gpurun_out/r04u/parity.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04u/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04u/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04u/tests.log | head -20; exit 1; }
timeout -k 10 120 python -u tools/mlp_bench.py --fused-only --bwd --iters 20 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/r04u/p1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/r04u/p1.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/r04u/pmc.json gpurun_out/r04u/p1
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r04u/pmc.json"))
rows = sorted(d.items(), key=lambda kv: -kv[1].get("SQ_LDS_BANK_CONFLICT", 0) * kv[1].get("dispatches", 1))
for k, v in rows[:16]:
    n = v.get("dispatches", 1)
    print(f"{k[:60]:60s} n={n:4.0f} conflict={v.get('SQ_LDS_BANK_CONFLICT',0):.3e} busy={v.get('SQ_BUSY_CYCLES',0):.3e} ratio={v.get('SQ_LDS_BANK_CONFLICT',0)/max(v.get('SQ_BUSY_CYCLES',1),1):.3f} waitlds={v.get('SQ_WAIT_INST_LDS',0):.3e}")
PY
rm -rf gpurun_out/r04u/p1
