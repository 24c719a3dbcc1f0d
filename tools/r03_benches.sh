# Round-3 bench lines for C3 / C4 / C5 and a rocprofv3 kernel-trace summary of the C2 step
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03g}
for c in c4 c5 c3; do
  timeout -k 10 500 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-gather > gpurun_out/${TAG}_bench_$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_$c.log; exit 1; }
  tail -c 400 gpurun_out/${TAG}_bench_$c.log; echo
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_c2prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/${TAG}_c2prof.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find gpurun_out/${TAG}_c2prof -name "*.db" | head -1) 40 > gpurun_out/${TAG}_c2_kernel_stats.txt
head -30 gpurun_out/${TAG}_c2_kernel_stats.txt
