# Round-4 end evidence in one GPU call: the -m gpu suite, smoke, PMC passes over the C2 bench
# (profiles/r04_pmc_summary.json, read by bench.py for roofline.traffic), the default bench (C2)
# with its cpu_baseline, C3 / C4 / C5 lines and a rocprofv3 --kernel-trace --stats summary of
# the C2 bench command
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r04f}
mkdir -p gpurun_out/keep
export PARITY_LOG=gpurun_out/${TAG}_parity.json
if [ "${STAGE:-1}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/${TAG}_gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
exit 0
fi
bash tools/pmc_passes.sh || exit 1
cp gpurun_out/pmc/summary.json gpurun_out/keep/${TAG}_pmc_summary.json && cp gpurun_out/pmc/summary.txt gpurun_out/keep/${TAG}_pmc_summary.txt
cp gpurun_out/pmc/summary.json profiles/r04_pmc_summary.json
rm -rf gpurun_out/pmc/fetch gpurun_out/pmc/write gpurun_out/pmc/sq
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_c2.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c2.log; exit 1; }
tail -c 600 gpurun_out/${TAG}_bench_c2.log; echo
for c in c3 c4 c5; do
  timeout -k 10 500 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-gather > gpurun_out/${TAG}_bench_$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_$c.log; exit 1; }
  tail -c 300 gpurun_out/${TAG}_bench_$c.log; echo
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c2prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/${TAG}_c2prof.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find gpurun_out/${TAG}_c2prof -name "*.db" | head -1) 45 > gpurun_out/${TAG}_c2_kernel_stats.txt 2>&1
find gpurun_out/${TAG}_c2prof -name "*stats*.csv" -exec cp {} gpurun_out/keep/${TAG}_c2_kernel_stats.csv \;
head -12 gpurun_out/${TAG}_c2_kernel_stats.txt
rm -rf gpurun_out/${TAG}_c2prof
