# Round-5 GPU pass k: cost ladder of the fused MLP forward (mlp_fwd_k, C2 shape): the normal build
# against builds without the DMA waits (M1), the GELU (M2), the per-chunk barrier (M3) or the
# S MFMAs (M4)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05k
for rep in 1 2; do
  for v in base M1 M2 M3 M4; do
    if [ $v = base ]; then unset LTHM_LIB_PATH; else export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_$v.so; fi
    echo -n "$v " >> gpurun_out/r05k/ladder.log
    timeout -k 10 120 python3 tools/mlp_bench.py --fused-only --iters 20 2>&1 | grep -v amdgpu.ids >> gpurun_out/r05k/ladder.log || exit 1
  done
done
unset LTHM_LIB_PATH
cat gpurun_out/r05k/ladder.log
