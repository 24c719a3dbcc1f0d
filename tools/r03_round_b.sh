# One GPU call: the -m gpu suite, the default bench (C2), then the PMC passes over the C2
# bench (tools/pmc_passes.sh) whose summary bench.py reads for roofline.traffic
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03b}
export PARITY_LOG=gpurun_out/${TAG}_parity.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/pmc_passes.sh || exit 1
tail -25 gpurun_out/pmc/summary.txt
mkdir -p gpurun_out/keep && cp gpurun_out/pmc/summary.json gpurun_out/keep/${TAG}_pmc_summary.json && cp gpurun_out/pmc/summary.json profiles/r03_pmc_summary.json
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_c2.log 2>&1 || exit 1
tail -c 1500 gpurun_out/${TAG}_bench_c2.log; echo
