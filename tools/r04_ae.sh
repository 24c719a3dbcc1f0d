# Round-4 GPU pass ae: ragged-K wgrad, fp8 256-tile GEMM at K >= 1024, per-phase DMA issue: tests, benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ae
export PARITY_LOG=gpurun_out/r04ae/parity.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_fp8.py tests/test_gpu_lthm.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or fp8 or pad_prefix or c5" > gpurun_out/r04ae/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04ae/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04ae/tests.log | head -30; exit 1; }
for c in c5 c4 c2; do
  n=gpurun_out/r04ae/bench_$c.log
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
  python3 - $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"])
        for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["share"])[:7]:
            print("   ", k, v["avg_ms"], v["calls_per_step"], round(v["avg_ms"] * v["calls_per_step"], 3))
PY
done
