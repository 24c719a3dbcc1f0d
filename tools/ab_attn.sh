# attention backward: GPU encoder tests, then the C2-shape probe: old 16x16x32 kernel,
# one-shot 32x32x16 kernel, persistent double-buffered 32x32x16 kernel
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encoder.py > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
TAG=old LTHM_ATTN_BWD_OLD=1 timeout -k 10 120 python3 tools/attn_probe.py || exit 1
TAG=oneshot LTHM_ATTN_BWD_ONESHOT=1 timeout -k 10 120 python3 tools/attn_probe.py || exit 1
TAG=persistent timeout -k 10 120 python3 tools/attn_probe.py || exit 1
