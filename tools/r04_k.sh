# Round-4 GPU pass k: software-pipelined compact fused pass (S of step i+1 beside step i's
# exp / sums / P.img), with two sched_group_barrier interleaves (CL_SGB=1/2) for A/B; parity on the default
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04k
export PARITY_LOG=gpurun_out/r04k/parity.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_loss_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04k/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04k/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04k/tests.log | head -20; exit 1; }
for v in base sgb1 sgb2; do
  if [ $v = base ]; then export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip.so
  else export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r04k/lb_$v -o run -- python3 tools/loss_bench.py > gpurun_out/r04k/lb_$v.log 2>&1 || { tail -5 gpurun_out/r04k/lb_$v.log; exit 1; }
  echo "== $v $(grep fwd+bwd gpurun_out/r04k/lb_$v.log | tail -1)"
  python3 tools/rocpd_stats.py $(find gpurun_out/r04k/lb_$v -name "*.db" | head -1) 3
done
unset LTHM_LIB_PATH
rm -rf gpurun_out/r04k/lb_*/
