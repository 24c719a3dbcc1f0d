# Round-5 final GPU pass: the whole -m gpu suite (parity log), smoke, the default bench (C2, with
# cpu_baseline), C4 with its cpu_baseline, C5, and a rocprofv3 --kernel-trace --stats summary of
# the C2 bench.  Steps chained: the first failure ends the script.
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05z}
mkdir -p gpurun_out/keep
export PARITY_LOG=gpurun_out/${TAG}_parity.json
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/${TAG}_gpu_tests.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench_c2.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c2.log; exit 1; }
tail -c 600 gpurun_out/${TAG}_bench_c2.log; echo
timeout -k 10 500 python bench.py --config c4 --steps 20 --warmup 5 --no-hbm-gather > gpurun_out/${TAG}_bench_c4.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c4.log; exit 1; }
tail -c 400 gpurun_out/${TAG}_bench_c4.log; echo
timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 2 --no-hbm-gather --no-cpu-baseline > gpurun_out/${TAG}_bench_c5.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c5.log; exit 1; }
tail -c 300 gpurun_out/${TAG}_bench_c5.log; echo
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c2prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/${TAG}_c2prof.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find gpurun_out/${TAG}_c2prof -name "*.db" | head -1) 45 > gpurun_out/${TAG}_c2_kernel_stats.txt 2>&1
find gpurun_out/${TAG}_c2prof -name "*stats*.csv" -exec cp {} gpurun_out/keep/${TAG}_c2_kernel_stats.csv \;
head -16 gpurun_out/${TAG}_c2_kernel_stats.txt
rm -rf gpurun_out/${TAG}_c2prof
