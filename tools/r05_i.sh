# Round-5 GPU pass i: K = 1 table backward with a touched-row bitmap (C4): tests, then the C4
# bench A/B (LTHM_KSHIFT_FIRST=1 bitmap + first-touch stores, 0 int32 flags + atomics)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05i
export PARITY_LOG=gpurun_out/r05i/parity.json
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tables.py tests/test_gpu_ranker.py tests/test_gpu_optim.py tests/test_gpu_configs.py tests/test_gpu_dist.py > gpurun_out/r05i/tests.log 2>&1 || { tail -30 gpurun_out/r05i/tests.log; exit 1; }
tail -2 gpurun_out/r05i/tests.log
for v in 1 0 1 0; do
  LTHM_KSHIFT_FIRST=$v timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r05i/c4_$v.log 2>&1 || { tail -20 gpurun_out/r05i/c4_$v.log; exit 1; }
  tail -1 gpurun_out/r05i/c4_$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('FIRST=$v', d['value'], d['ms_per_step'], ' '.join(f\"{x}={k[x]['avg_ms']}\" for x in sorted(k) if 'kshift' in x or 'adam' in x))"
done
