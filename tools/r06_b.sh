# Round-6 pass b: GPU parity of the round-6 paths (all switched on: the register-row gather, the
# two-workgroup MLP forward / hidden backward, the keep-grad row-wise step, the 8-row LN-GEMM
# epilogue library), the advisor-driven test changes, kernel A/Bs, the row-wise AdamW layout probe
# and the gather PMC passes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06b
export NEW="LTHM_KSHIFT_REG=1 LTHM_MLP_FWD2=1 LTHM_MLP_BWDP2=1 LTHM_SPARSE_KEEP_GRAD=1 LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_EPR8.so"
env $NEW timeout -k 10 500 python -u -m pytest tests/test_gpu_kshift.py tests/test_gpu_encoder.py tests/test_gpu_mlp.py tests/test_gpu_optim.py tests/test_gpu_tables.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06b/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06b/tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r06b/tests.log | head -30; exit $rc; }
env $NEW timeout -k 10 300 python -u -m pytest tests/test_gpu_wrapper_api.py tests/test_gpu_lthm_step_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06b/tests2.log 2>&1 || { grep -E "^FAILED|^E " gpurun_out/r06b/tests2.log | head -20; exit 1; }
tail -1 gpurun_out/r06b/tests2.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_loss_golden.py -q -s --timeout 200 --timeout-method thread > gpurun_out/r06b/tests_loss.log 2>&1
rc=$?; tail -2 gpurun_out/r06b/tests_loss.log; grep -E "NaN|^FAILED" gpurun_out/r06b/tests_loss.log | head; [ $rc -le 1 ] || exit $rc
for v in 1 0 1 0; do
  echo -n "FWD2=$v " >> gpurun_out/r06b/mlp_ab.log
  LTHM_MLP_FWD2=$v timeout -k 10 120 python tools/mlp_bench.py --fused-only --iters 20 2>/dev/null >> gpurun_out/r06b/mlp_ab.log || exit 1
  echo -n "BWDP2=$v " >> gpurun_out/r06b/mlp_ab.log
  LTHM_MLP_BWDP2=$v timeout -k 10 120 python tools/mlp_bench.py --only bwd_hidden --iters 20 2>/dev/null >> gpurun_out/r06b/mlp_ab.log || exit 1
done
echo -n "FWD2=1 PF2 " >> gpurun_out/r06b/mlp_ab.log
LTHM_MLP_FWD2=1 LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_PF2.so timeout -k 10 120 python tools/mlp_bench.py --fused-only --iters 20 2>/dev/null >> gpurun_out/r06b/mlp_ab.log || exit 1
cat gpurun_out/r06b/mlp_ab.log
LTHM_KSHIFT_REG=1 timeout -k 10 200 python tools/gather_bench.py > gpurun_out/r06b/gather.json 2>gpurun_out/r06b/gather.err || { tail gpurun_out/r06b/gather.err; exit 1; }
cat gpurun_out/r06b/gather.json
timeout -k 10 200 python tools/gather_bench.py > gpurun_out/r06b/gather_old.json 2>/dev/null || exit 1
cat gpurun_out/r06b/gather_old.json
timeout -k 10 120 ./tools/probes/sparse_layout_probe > gpurun_out/r06b/sparse_probe.log 2>&1 || { cat gpurun_out/r06b/sparse_probe.log; exit 1; }
cat gpurun_out/r06b/sparse_probe.log
LTHM_KSHIFT_REG=1 bash tools/pmc_gather.sh || exit 1
cat gpurun_out/pmc_gather/summary.txt
