# long-T' attention backward (32x32x16 rows / columns kernels) vs the windowed kernels:
# encoder GPU tests, then the probe at the C5 shape with LTHM_ATTN_BWD_OLD=1 / 0
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encoder.py > gpurun_out/abl_tests.log 2>&1 || { tail -40 gpurun_out/abl_tests.log; exit 1; }
tail -2 gpurun_out/abl_tests.log
for sh in 1024,513,8 4096,129,4; do
  for v in 1 0; do SHAPE=$sh TAG="shape=$sh bwd_old=$v" LTHM_ATTN_BWD_OLD=$v timeout -k 10 120 python3 tools/attn_probe.py || exit 1; done
done
