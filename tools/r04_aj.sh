# Round-4 GPU pass aj: ranker MLP input assembled in bf16 inside the MLP op: tests, C4 bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04aj
export PARITY_LOG=gpurun_out/r04aj/parity.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_ranker.py tests/test_script_ops.py tests/test_gpu_lthm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04aj/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04aj/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04aj/tests.log | head -30; exit 1; }
n=gpurun_out/r04aj/bench_c4.log
timeout -k 10 400 python -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
python3 - $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"])
        for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["share"])[:8]:
            print("   ", k, v["avg_ms"], v["calls_per_step"])
PY
