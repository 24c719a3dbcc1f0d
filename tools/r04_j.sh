# Round-4 GPU pass j: compact loss passes with bit-mask special tiles and the diagonal in the
# epilogue; gather computes the positive logit
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04j
export PARITY_LOG=gpurun_out/r04j/parity.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_loss_golden.py tests/test_gpu_wrapper_api.py tests/test_gpu_lthm.py tests/test_gpu_lthm_step_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04j/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04j/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04j/tests.log | head -20; exit 1; }
grep "vc \|golden" gpurun_out/r04j/tests.log | head -30
LTHM_CL_VC=1 timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r04j/lb -o run -- python3 tools/loss_bench.py > gpurun_out/r04j/lb.log 2>&1 || { tail -5 gpurun_out/r04j/lb.log; exit 1; }
echo "== $(grep fwd+bwd gpurun_out/r04j/lb.log | tail -1)"
python3 tools/rocpd_stats.py $(find gpurun_out/r04j/lb -name "*.db" | head -1) 10
rm -rf gpurun_out/r04j/lb/
n=gpurun_out/r04j/bench_c2.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
python3 - $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(d["value"], d["ms_per_step"], json.dumps(d["roofline"]))
        for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["share"])[:14]:
            print("   ", k, v["avg_ms"], v["calls_per_step"], v["share"], v.get("TFLOP/s"))
PY
