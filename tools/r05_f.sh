# Round-5 GPU pass f: K = 1 table backward with first-touch stores (lthm_kshift_bwd_sparse_first):
# table / ranker / optimizer tests, then the C4 bench A/B (LTHM_KSHIFT_FIRST=1 new, 0 all-atomic)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05f
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tables.py tests/test_gpu_ranker.py tests/test_gpu_optim.py tests/test_gpu_configs.py > gpurun_out/r05f/tests.log 2>&1 || { tail -30 gpurun_out/r05f/tests.log; exit 1; }
tail -2 gpurun_out/r05f/tests.log
for v in 1 0 1 0; do
  LTHM_KSHIFT_FIRST=$v timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r05f/c4_$v.log 2>&1 || { tail -20 gpurun_out/r05f/c4_$v.log; exit 1; }
  tail -1 gpurun_out/r05f/c4_$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('FIRST=$v', d['value'], d['ms_per_step'], ' '.join(f\"{x}={k[x]['avg_ms']}x{k[x]['calls_per_step']}\" for x in sorted(k) if 'kshift' in x or 'adam' in x))"
done
