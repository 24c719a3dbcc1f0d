# Round-4 GPU pass ai: rocprofv3 --kernel-trace --stats summaries of the C5 and C4 bench commands
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ai
for c in c5 c4; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04ai/$c -o run -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-gather > gpurun_out/r04ai/$c.log 2>&1 || { tail -5 gpurun_out/r04ai/$c.log; exit 1; }
  python3 tools/rocpd_stats.py $(find gpurun_out/r04ai/$c -name "*.db" | head -1) 40 > gpurun_out/r04ai/${c}_kernel_stats.txt 2>&1
  rm -rf gpurun_out/r04ai/$c
  head -12 gpurun_out/r04ai/${c}_kernel_stats.txt
done
