# A/B of two builds of liblthm_hip.so on one box (B = recommendations_amd/liblthm_hip_B.so via
# LTHM_LIB_PATH), alternating C2 bench runs; KEYS = the kernel-timer keys to print
cd $GRAFT_REPO_ROOT
for v in A B A B; do
  if [ $v = B ]; then export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_B.so; else unset LTHM_LIB_PATH; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/ablib_$v.log 2>&1 || { tail -20 gpurun_out/ablib_$v.log; exit 1; }
  python3 - $v "${KEYS:-cl_fwd_k cl_bwd_k}" <<'PY'
import json, sys
for l in open(f"gpurun_out/ablib_{sys.argv[1]}.log").read().splitlines():
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], " ".join(f"{k}={d['kernels'][k]['avg_ms']}" for k in sys.argv[2].split()))
PY
done
