# Round-4 GPU pass ac: 64-k-stage weight-gradient kernel (gemm_wg2_k): GEMM tests, microbench on/off
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ac
export LTHM_GEMM_WG2=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/r04ac/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04ac/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04ac/tests.log | head -30; exit 1; }
for cfg in c2 c5 c4; do
  GEMM_BENCH_CFG=$cfg timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r04ac/gemm_${cfg}_wg2.log 2>&1 || exit 1
  LTHM_GEMM_WG2=0 GEMM_BENCH_CFG=$cfg timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r04ac/gemm_${cfg}_wg1.log 2>&1 || exit 1
done
for f in gpurun_out/r04ac/gemm_*.log; do echo "== $f"; grep -o "^[a-z0-9]* *M=[0-9]* N=[0-9]* K=[0-9]*\|wgrad [0-9.]* ([0-9]* TF)" $f | paste - - ; done
