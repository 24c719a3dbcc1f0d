# One GPU call: the whole -m gpu suite, the default bench (C2), and a kernel-trace of the
# 4.1 GB gather leg; outputs under gpurun_out/ (TAG names the files)
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03}
export PARITY_LOG=gpurun_out/${TAG}_parity.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_c2.log 2>&1 || exit 1
tail -c 600 gpurun_out/${TAG}_bench_c2.log; echo
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_gather -o run -- python3 tools/gather_bench.py > gpurun_out/${TAG}_gather.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find gpurun_out/${TAG}_gather -name "*.db" | head -1) 5 > gpurun_out/${TAG}_gather_stats.txt
cat gpurun_out/${TAG}_gather_stats.txt
