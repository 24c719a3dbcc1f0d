# Round-6 pass g: the ranker input row buffer (TablesIntoRowFn, ABI 42) -- parity and the C4 A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06g
timeout -k 10 300 python -u -m pytest tests/test_gpu_ranker.py tests/test_gpu_kshift.py tests/test_gpu_tables.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06g/tests.log 2>&1 || { grep -E "^FAILED|^E  " gpurun_out/r06g/tests.log | head -20; exit 1; }
tail -1 gpurun_out/r06g/tests.log
for a in 1 0 1 0; do
  LTHM_RANKER_INPUT_ROW=$a timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --no-hbm-gather --no-cpu-baseline > gpurun_out/r06g/c4_r$a.log 2>&1 || { tail -20 gpurun_out/r06g/c4_r$a.log; exit 1; }
  python3 - gpurun_out/r06g/c4_r$a.log r$a <<'PY'
import json, sys
s = open(sys.argv[1]).read(); j = json.loads(s[s.rfind('{"metric'):].split('\n')[0]); k = j.get('kernels', {})
print(sys.argv[2], j['ms_per_step'], {n: round(v['avg_ms'], 4) for n, v in k.items() if v['avg_ms'] * v['calls_per_step'] > 0.05})
PY
done
