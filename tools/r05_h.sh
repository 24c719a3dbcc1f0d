# Round-5 GPU pass h: cost ladder of the C2 attention backward (attn_bwd32_k): the normal build
# against builds that skip the units (X1), the staging loads (X2) or the gradient stores (X3)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05h
for rep in 1 2; do
  for v in base X1 X2 X3; do
    if [ $v = base ]; then unset LTHM_LIB_PATH; else export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_$v.so; fi
    TAG="$v" timeout -k 10 120 python3 tools/attn_probe.py >> gpurun_out/r05h/ladder.log 2>&1 || { tail -20 gpurun_out/r05h/ladder.log; exit 1; }
  done
done
unset LTHM_LIB_PATH
grep -v amdgpu.ids gpurun_out/r05h/ladder.log
