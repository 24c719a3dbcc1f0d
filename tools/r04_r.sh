# Round-4 GPU pass r: hand-scheduled clean tiles of the compact fused pass (CL_HS) vs default:
# loss tests on the variant, loss bench alternating
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04r
export PARITY_LOG=gpurun_out/r04r/parity.json
LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_hs.so timeout -k 10 300 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_loss_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04r/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04r/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04r/tests.log | head -20; exit 1; }
for rep in 1 2; do for v in base hs; do
  if [ $v = base ]; then export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip.so
  else export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r04r/lb_$v -o run -- python3 tools/loss_bench.py > gpurun_out/r04r/lb_$v.log 2>&1 || { tail -5 gpurun_out/r04r/lb_$v.log; exit 1; }
  echo "== $v $(grep fwd+bwd gpurun_out/r04r/lb_$v.log | tail -1) $(python3 tools/rocpd_stats.py $(find gpurun_out/r04r/lb_$v -name '*.db' | head -1) 20 | grep fr32v)"
  rm -rf gpurun_out/r04r/lb_$v/
done; done
