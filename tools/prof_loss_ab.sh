# loss kernels alone (tools/loss_bench.py) under rocprofv3 --kernel-trace for backward variants:
# old = round-2 16x16x32 per-head kernels (LTHM_CL_BWD_OLD=1); new = the 32x32x16 all-heads kernels
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-old new}; do
  if [ $v = old ]; then export LTHM_CL_BWD_OLD=1; else export LTHM_CL_BWD_OLD=0; fi

  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/prof_$v -o run -- python3 tools/loss_bench.py > gpurun_out/loss_$v.log 2>&1 || exit 1
  echo "== $v $(grep fwd+bwd gpurun_out/loss_$v.log | tail -1)"
  python3 tools/rocpd_stats.py $(find gpurun_out/prof_$v -name "*.db" | head -1) 3
done
