# attention A/B of two library builds (B = liblthm_hip_B.so): encoder GPU tests on B, then
# the probe at the C2 and C5 shapes on A and B alternately
cd $GRAFT_REPO_ROOT
LB=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_B.so
LTHM_LIB_PATH=$LB timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encoder.py > gpurun_out/abal_tests.log 2>&1 || { tail -40 gpurun_out/abal_tests.log; exit 1; }
tail -2 gpurun_out/abal_tests.log
for sh in 4096,129,4 1024,513,8; do
  for v in A B A B; do
    if [ $v = B ]; then export LTHM_LIB_PATH=$LB; else unset LTHM_LIB_PATH; fi
    SHAPE=$sh TAG="shape=$sh lib=$v" timeout -k 10 120 python3 tools/attn_probe.py || exit 1
  done
done
