# Round-5 GPU pass g: K = 1 table backward with first-touch stores (C4) and the dgrad GEMM fused
# with the LayerNorm backward and c_proj with ln_2's forward (C2): tests, then A/B benches (LTHM_KSHIFT_FIRST, LTHM_LN_DGRAD, LTHM_LN_LINEAR)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05g
export PARITY_LOG=gpurun_out/r05g/parity.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tables.py tests/test_gpu_ranker.py tests/test_gpu_optim.py tests/test_gpu_encoder.py tests/test_gpu_lthm_step_golden.py tests/test_gpu_lthm.py > gpurun_out/r05g/tests.log 2>&1 || { tail -30 gpurun_out/r05g/tests.log; exit 1; }
tail -2 gpurun_out/r05g/tests.log
summ() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']
print(sys.argv[2], d['value'], d['ms_per_step'], ' '.join(f\"{x}={k[x]['avg_ms']}x{k[x]['calls_per_step']}\" for x in sorted(k) if any(s in x for s in sys.argv[3].split(','))))" "$@"; }
for v in 1 0 1 0; do
  LTHM_KSHIFT_FIRST=$v timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r05g/c4_$v.log 2>&1 || { tail -20 gpurun_out/r05g/c4_$v.log; exit 1; }
  summ gpurun_out/r05g/c4_$v.log FIRST=$v kshift,adam
done
for v in 11 00 10 01 11 00; do
  LTHM_LN_DGRAD=${v:0:1} LTHM_LN_LINEAR=${v:1:1} timeout -k 10 300 python bench.py --no-cpu-baseline --no-hbm-gather --steps 10 --warmup 3 > gpurun_out/r05g/c2_$v.log 2>&1 || { tail -20 gpurun_out/r05g/c2_$v.log; exit 1; }
  summ gpurun_out/r05g/c2_$v.log LN=$v layernorm,dgrad_ln,linear_ln,gemm_k
done
