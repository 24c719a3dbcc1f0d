# Round-4 GPU pass ak: K = 1 KShift forward with 8 items in flight per lane group: tests, C4 A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ak
export PARITY_LOG=gpurun_out/r04ak/parity.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_kshift.py tests/test_gpu_ranker.py tests/test_gpu_tables.py tests/test_gpu_lthm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ak/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04ak/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04ak/tests.log | head -30; exit 1; }
for v in A B A; do
  if [ $v = B ]; then export LTHM_KSHIFT_K1=0; else unset LTHM_KSHIFT_K1; fi
  n=gpurun_out/r04ak/bench_c4_$v.log
  timeout -k 10 400 python -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
  python3 - $n $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[2], d["value"], d["ms_per_step"], d["kernels"].get("kshift_fwd_k"))
PY
done
