# kernel summary of the generator step (fused path) after the round-6 tuning
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/embgen_bench.py --steps 10 --warmup 2 > $O/prof.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find $O/prof -name "*.db" | head -1) 40 > $O/kernel_stats.txt 2>&1
head -30 $O/kernel_stats.txt
rm -rf $O/prof
