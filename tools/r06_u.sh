# (A/B run on a since-removed switch; see DESIGN.md logQ) beta = 0 logQ update on a side stream (LTHM_LOGQ_SIDE):
# the C2 bench with the side stream off (0) and on (1), twice each
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py tests/test_gpu_loss.py tests/test_gpu_loss_golden.py tests/test_gpu_lthm.py \
  tests/test_gpu_lthm_step_golden.py tests/test_gpu_wrapper_api.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 1 0 1; do
  LTHM_LOGQ_SIDE=$v timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-hbm-gather --no-generator > $O/side$v.log 2>&1 || { tail -5 $O/side$v.log; exit 1; }
  python3 -c "
import json;s=open('$O/side$v.log').read();i=s.rfind('{\"metric\"');d=json.loads(s[i:].split(chr(10))[0])
print('side$v', d['value'], d['ms_per_step'], d['kernels']['logq_stream'], d['kernels']['cl_fwd_k']['avg_ms'], d['final_loss'])"
done
