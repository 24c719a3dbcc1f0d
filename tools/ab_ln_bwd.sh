cd $GRAFT_REPO_ROOT
LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_B.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encoder.py tests/test_gpu_lthm.py -k "layernorm or block or step" > gpurun_out/r03m_tests.log 2>&1 || { tail -30 gpurun_out/r03m_tests.log; exit 1; }
tail -1 gpurun_out/r03m_tests.log
KEYS="lthm_layernorm_bwd" bash tools/ab_lib.sh || exit 1
for v in A B; do
  if [ $v = B ]; then export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_B.so; else unset LTHM_LIB_PATH; fi
  timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 2 --no-cpu-baseline --no-hbm-gather > gpurun_out/r03m_c5_$v.log 2>&1 || exit 1
  python3 - $v <<'PY'
import json, sys
v = sys.argv[1]
for l in open(f"gpurun_out/r03m_c5_{v}.log"):
    if l.startswith('{"metric"'):
        d = json.loads(l)
print("C5", v, d["value"], d["ms_per_step"], d["kernels"]["lthm_layernorm_bwd"]["avg_ms"])
PY
done
