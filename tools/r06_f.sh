# Round-6 pass f: the software-pipelined one-wave-per-SIMD MLP forward (mlp_fwd_pipe_k, its
# D = 128 GELU coverage fixed, fragment reads 2 steps ahead) -- parity and A/B; the ranker tests
# with the fp32-master gather
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06f
R=$GRAFT_REPO_ROOT/recommendations_amd
LTHM_MLP_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 200 --timeout-method thread -k "fwd" > gpurun_out/r06f/tests_pipe.log 2>&1
rc=$?; tail -3 gpurun_out/r06f/tests_pipe.log; grep -E "^FAILED|^E  " gpurun_out/r06f/tests_pipe.log | head -10
timeout -k 10 300 python -u -m pytest tests/test_gpu_ranker.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06f/tests_ranker.log 2>&1 || { grep -E "^FAILED|^E  " gpurun_out/r06f/tests_ranker.log | head -10; exit 1; }
tail -1 gpurun_out/r06f/tests_ranker.log
for v in base pipe pipe1 base pipe pipe1; do
  case $v in base) E="LTHM_X=1"; L=$R/liblthm_hip.so;; pipe) E="LTHM_MLP_PIPE=1"; L=$R/liblthm_hip.so;; pipe1) E="LTHM_MLP_PIPE=1"; L=$R/liblthm_hip_PP1.so;; esac
  echo -n "$v " >> gpurun_out/r06f/mlp_ab.log
  env $E LTHM_LIB_PATH=$L timeout -k 10 120 python tools/mlp_bench.py --fused-only --iters 20 2>/dev/null >> gpurun_out/r06f/mlp_ab.log || exit 1
done
cat gpurun_out/r06f/mlp_ab.log
