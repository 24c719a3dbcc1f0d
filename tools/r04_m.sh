# Round-4 GPU pass m: compact fused pass block order A/B: LTHM_CL_FR_XCD = 0 (plain), 1 (XCD-contiguous),
# 2 (clean tiles rotated per row block), 3 (both), alternating twice
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04m
for rep in 1 2; do for v in 0 1 2 3; do
  LTHM_CL_FR_XCD=$v timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r04m/lb_$v -o run -- python3 tools/loss_bench.py > gpurun_out/r04m/lb_$v.log 2>&1 || { tail -5 gpurun_out/r04m/lb_$v.log; exit 1; }
  echo "== xcd=$v $(grep fwd+bwd gpurun_out/r04m/lb_$v.log | tail -1) $(python3 tools/rocpd_stats.py $(find gpurun_out/r04m/lb_$v -name '*.db' | head -1) 20 | grep fr32v)"
  rm -rf gpurun_out/r04m/lb_$v/
done; done
