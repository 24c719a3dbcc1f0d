# Round-4 GPU pass ag: vectorized token assembly / token backward / outcome kernels: tests, C2 bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ag
export PARITY_LOG=gpurun_out/r04ag/parity.json
timeout -k 10 500 python -u -m pytest tests/test_gpu_lthm.py tests/test_gpu_lthm_step_golden.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ag/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04ag/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04ag/tests.log | head -30; exit 1; }
n=gpurun_out/r04ag/bench_c2.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
python3 - $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"])
        for k in ("lthm_tokens_fwd", "lthm_tokens_bwd", "lthm_outcome_fwd"):
            print("   ", k, d["kernels"].get(k))
PY
