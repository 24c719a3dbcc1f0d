# Round-4 GPU pass z: 256x256 GEMM kernel (gemm_pp_k): GEMM parity tests, microbench on/off
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04z
export PARITY_LOG=gpurun_out/r04z/parity.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/r04z/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04z/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04z/tests.log | head -30; exit 1; }
for cfg in c4 c5 c2; do
  GEMM_BENCH_CFG=$cfg GEMM_BENCH_SQUARE=1 timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r04z/gemm_$cfg.log 2>&1 || { tail -5 gpurun_out/r04z/gemm_$cfg.log; exit 1; }
  LTHM_GEMM_PP=0 GEMM_BENCH_CFG=$cfg GEMM_BENCH_SQUARE=1 timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r04z/gemm_${cfg}_off.log 2>&1 || exit 1
  echo "== $cfg pp"; grep -v amdgpu.ids gpurun_out/r04z/gemm_$cfg.log
  echo "== $cfg off"; grep -v amdgpu.ids gpurun_out/r04z/gemm_${cfg}_off.log
done
