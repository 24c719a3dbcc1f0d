# attention backward: GPU encoder tests, then the C2-shape probe old / new
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encoder.py > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
for v in 1 0; do TAG=old$v LTHM_ATTN_BWD_OLD=$v timeout -k 10 120 python3 tools/attn_probe.py || exit 1; done
