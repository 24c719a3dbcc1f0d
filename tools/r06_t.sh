# first-touch K > 1 sparse backward (lthm_kshift_bwd_sparse_ft): GPU parity tests, then the C2
# bench's lthm_kshift_bwd_sparse with LTHM_KSHIFT_FT=0 (all-atomic) vs 1 (first touch)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kshift.py tests/test_gpu_tables.py tests/test_gpu_optim.py tests/test_gpu_lthm.py \
  tests/test_gpu_configs.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for v in 0 1 0 1; do
  LTHM_KSHIFT_FT=$v timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather --no-generator > $O/ft$v.log 2>&1 || { tail -5 $O/ft$v.log; exit 1; }
  python3 -c "
import json;s=open('$O/ft$v.log').read();i=s.rfind('{\"metric\"');d=json.loads(s[i:].split(chr(10))[0])
print('ft$v', d['value'], d['ms_per_step'], d['kernels']['lthm_kshift_bwd_sparse'], d['kernels'].get('sparse_adamw'))"
done
