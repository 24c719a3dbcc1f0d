# fused forward + ROWS loss pass: the loss / golden / LTHM GPU tests, then the C2 bench A/B
# (LTHM_CL_NO_FUSED_ROWS=1: separate forward and ROWS passes)
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_loss.py tests/test_gpu_loss_golden.py tests/test_gpu_lthm.py tests/test_gpu_configs.py > gpurun_out/lf_tests.log 2>&1 || { tail -40 gpurun_out/lf_tests.log; exit 1; }
tail -2 gpurun_out/lf_tests.log
for v in 1 0; do
  LTHM_CL_NO_FUSED_ROWS=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/lf_bench_$v.log 2>&1 || { tail -30 gpurun_out/lf_bench_$v.log; exit 1; }
  python3 - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/lf_bench_{sys.argv[1]}.log").read().splitlines():
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print("no_fused_rows=" + sys.argv[1], "value", d["value"], "ms", d["ms_per_step"], "final_loss", d.get("final_loss"))
        for k in ("cl_fwd_k", "cl_bwd_k"):
            print("  ", k, d["kernels"].get(k))
        print("  roofline", d["roofline"])
PY
done
