# Round-4 GPU pass t: the compact gather normalises the `out` rows (no rownorm of next_token_emb):
# loss / wrapper / full-step tests, C2 bench; then the pass-s counters and C2 kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04t
export PARITY_LOG=gpurun_out/r04t/parity.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_loss_golden.py tests/test_gpu_wrapper_api.py tests/test_gpu_lthm.py tests/test_gpu_lthm_step_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04t/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04t/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04t/tests.log | head -20; exit 1; }
n=gpurun_out/r04t/bench_c2.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
python3 - $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(d["value"], d["ms_per_step"], {k: v["avg_ms"] for k, v in d["kernels"].items() if k.startswith("cl_") or "rownorm" in k or "rows_move" in k})
PY
bash tools/r04_s.sh
