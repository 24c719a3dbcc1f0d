# Round-5 GPU pass j: attention backward with the wider gradient stores: encoder tests (both the
# per-(b, h) kernel and, LTHM_ATTN_BWD_P=1, the persistent one), then the C2 / C5 probe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05j
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_encoder.py > gpurun_out/r05j/tests.log 2>&1 || { tail -30 gpurun_out/r05j/tests.log; exit 1; }
tail -1 gpurun_out/r05j/tests.log
LTHM_ATTN_BWD_P=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_encoder.py -k "attention" > gpurun_out/r05j/tests_p.log 2>&1 || { tail -30 gpurun_out/r05j/tests_p.log; exit 1; }
tail -1 gpurun_out/r05j/tests_p.log
for sh in 4096,129,4 1024,513,8; do
  for rep in 1 2; do
    SHAPE=$sh TAG="shape=$sh" timeout -k 10 120 python3 tools/attn_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
