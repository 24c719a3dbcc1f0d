# One GPU call: the -m gpu suite, smoke, the default bench (C2), C5, and a rocprofv3
# kernel-trace summary of the C2 step (TAG names the files under gpurun_out/)
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03c}
export PARITY_LOG=gpurun_out/${TAG}_parity.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_c2.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c2.log; exit 1; }
tail -c 700 gpurun_out/${TAG}_bench_c2.log; echo
timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-gather > gpurun_out/${TAG}_bench_c5.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c5.log; exit 1; }
tail -c 400 gpurun_out/${TAG}_bench_c5.log; echo
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_c2prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/${TAG}_c2prof.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find gpurun_out/${TAG}_c2prof -name "*.db" | head -1) 40 > gpurun_out/${TAG}_c2_kernel_stats.txt
head -12 gpurun_out/${TAG}_c2_kernel_stats.txt
