# kernel breakdown of the attention forward / backward at the C5 shape (T' = 513)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
SHAPE=1024,513,8 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run -- python3 tools/attn_probe.py > gpurun_out/prof_c5.log 2>&1 || { tail -30 gpurun_out/prof_c5.log; exit 1; }
f=$(ls gpurun_out/prof_c5/*/run_kernel_stats.csv | head -1); cut -d, -f1-4 "$f" | head -14
