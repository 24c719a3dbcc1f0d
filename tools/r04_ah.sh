# Round-4 GPU pass ah: folded residual gradient in the block backward: tests, C2 bench; sparse AdamW row order
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ah
export LTHM_LN_FOLD=1
export PARITY_LOG=gpurun_out/r04ah/parity.json
timeout -k 10 500 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_lthm.py tests/test_gpu_lthm_step_golden.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ah/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04ah/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04ah/tests.log | head -30; exit 1; }
n=gpurun_out/r04ah/bench_c2.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
python3 - $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], d["kernels"]["lthm_layernorm_bwd"])
PY
timeout -k 10 200 python -u tools/sparse_opt_bench.py > gpurun_out/r04ah/sparse.log 2>&1 || exit 1
cat gpurun_out/r04ah/sparse.log | grep -v amdgpu
