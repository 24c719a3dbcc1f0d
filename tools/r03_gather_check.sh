# KShift gather: parity tests, then the 4.1 GB gather leg under rocprofv3 kernel-trace
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kshift.py > gpurun_out/${TAG}_kshift_tests.log 2>&1 || { tail -5 gpurun_out/${TAG}_kshift_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_kshift_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_gather -o run -- python3 tools/gather_bench.py > gpurun_out/${TAG}_gather.log 2>&1 || exit 1
tail -c 400 gpurun_out/${TAG}_gather.log; echo
python3 tools/rocpd_dispatches.py $(find gpurun_out/${TAG}_gather -name "*.db" | head -1) kshift_fwd_k 2 1
