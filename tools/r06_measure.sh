# Round-6 measurement pass over the current tree.  Steps (each under its own time limit, chained:
# the first failure ends the script):
#   TESTS=1  the whole -m gpu suite (parity log) + smoke
#   BENCH=1  default bench (C2, with cpu_baseline), C4 with its cpu_baseline, C5
#   PROF=1   rocprofv3 --kernel-trace --stats summary of the C2 bench
#   PMC=1    FETCH_SIZE / WRITE_SIZE / SQ passes over the C2 bench (separate runs)
#   LADDER=1 the mlp_fwd_k cost ladder (liblthm_hip_M{1..4}.so, tools/build_variant.sh)
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r06a}
mkdir -p gpurun_out/keep
if [ "${TESTS:-0}" = 1 ]; then
  export PARITY_LOG=gpurun_out/${TAG}_parity.json
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.log
  [ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/${TAG}_gpu_tests.log | head -30; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench_c2.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c2.log; exit 1; }
  tail -c 600 gpurun_out/${TAG}_bench_c2.log; echo
  timeout -k 10 500 python bench.py --config c4 --steps 20 --warmup 5 --no-hbm-gather > gpurun_out/${TAG}_bench_c4.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c4.log; exit 1; }
  tail -c 400 gpurun_out/${TAG}_bench_c4.log; echo
  timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 2 --no-hbm-gather --no-cpu-baseline > gpurun_out/${TAG}_bench_c5.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c5.log; exit 1; }
  tail -c 300 gpurun_out/${TAG}_bench_c5.log; echo
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c2prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/${TAG}_c2prof.log 2>&1 || exit 1
  python3 tools/rocpd_stats.py $(find gpurun_out/${TAG}_c2prof -name "*.db" | head -1) 45 > gpurun_out/${TAG}_c2_kernel_stats.txt 2>&1
  find gpurun_out/${TAG}_c2prof -name "*stats*.csv" -exec cp {} gpurun_out/keep/${TAG}_c2_kernel_stats.csv \;
  head -16 gpurun_out/${TAG}_c2_kernel_stats.txt
  rm -rf gpurun_out/${TAG}_c2prof
fi
if [ "${PMC:-0}" = 1 ]; then
  P=gpurun_out/${TAG}_pmc
  mkdir -p $P
  B="--steps 2 --warmup 1 --no-cpu-baseline --no-hbm-gather --no-kernel-timing"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch -o run --output-format csv -- python3 bench.py $B > $P/fetch.log 2>&1 || exit 1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write -o run --output-format csv -- python3 bench.py $B > $P/write.log 2>&1 || exit 1
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --kernel-trace -d $P/sq -o run --output-format csv -- python3 bench.py $B > $P/sq.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $P/summary.json $P/fetch $P/write $P/sq > $P/summary.txt 2>&1
  head -12 $P/summary.txt | cut -c1-200
  rm -rf $P/fetch $P/write $P/sq
fi
if [ "${LADDER:-0}" = 1 ]; then
  L=gpurun_out/${TAG}_ladder.log
  for rep in 1 2; do
    for v in base M1 M2 M3 M4; do
      if [ $v = base ]; then unset LTHM_LIB_PATH; else export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_$v.so; fi
      echo -n "$v " >> $L
      timeout -k 10 120 python3 tools/mlp_bench.py --fused-only --iters 20 > $L.tmp 2>&1 || { cat $L.tmp; exit 1; }
      grep -v amdgpu.ids $L.tmp >> $L
    done
  done
  unset LTHM_LIB_PATH
  cat $L
fi
if [ "${GATHER:-0}" = 1 ]; then
  bash tools/pmc_gather.sh || exit 1
  cp gpurun_out/pmc_gather/gather_pmc.json gpurun_out/${TAG}_gather_pmc.json
  cat gpurun_out/pmc_gather/summary.txt | head -30
fi
if [ "${C4PROF:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c4prof -o run -- python3 bench.py --config c4 --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/${TAG}_c4prof.log 2>&1 || exit 1
  python3 tools/rocpd_stats.py $(find gpurun_out/${TAG}_c4prof -name "*.db" | head -1) 30 > gpurun_out/${TAG}_c4_kernel_stats.txt 2>&1
  head -12 gpurun_out/${TAG}_c4_kernel_stats.txt
  rm -rf gpurun_out/${TAG}_c4prof
fi
if [ "${C5PROF:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c5prof -o run -- python3 bench.py --config c5 --steps 3 --warmup 2 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/${TAG}_c5prof.log 2>&1 || exit 1
  python3 tools/rocpd_stats.py $(find gpurun_out/${TAG}_c5prof -name "*.db" | head -1) 30 > gpurun_out/${TAG}_c5_kernel_stats.txt 2>&1
  head -12 gpurun_out/${TAG}_c5_kernel_stats.txt
  rm -rf gpurun_out/${TAG}_c5prof
fi
