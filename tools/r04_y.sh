# Round-4 GPU pass y: packed-row attention (shared pad prefix at T' > 256): parity, attention
# regression, C5 bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04y
export PARITY_LOG=gpurun_out/r04y/parity.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_lthm.py tests/test_gpu_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pad_prefix or attention or step_vs_oracle" > gpurun_out/r04y/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04y/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04y/tests.log | head -30; exit 1; }
grep -E "pad_prefix" gpurun_out/r04y/tests.log | head -5
for c in c5; do
  n=gpurun_out/r04y/bench_$c.log
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
  python3 - $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], json.dumps(d["roofline"])[:160])
        for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["share"])[:14]:
            print("   ", k, v["avg_ms"], v["calls_per_step"], round(v["avg_ms"] * v["calls_per_step"], 3))
PY
done
