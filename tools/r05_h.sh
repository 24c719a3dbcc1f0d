# Round-5 GPU pass h: the C2 attention backward (attn_bwd32_k and its persistent double-buffered
# form attn_bwd32p_k): the encoder tests, then a cost ladder against builds that skip the units
# (X1), the staging loads (X2) or the gradient stores (X3), for both kernels
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05h
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_encoder.py -k "attention or block" > gpurun_out/r05h/tests.log 2>&1 || { tail -30 gpurun_out/r05h/tests.log; exit 1; }
tail -2 gpurun_out/r05h/tests.log
for rep in 1 2; do
  for p in 1 0; do
    for v in base X1 X2 X3; do
      if [ $v = base ]; then unset LTHM_LIB_PATH; else export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_$v.so; fi
      LTHM_ATTN_BWD_P=$p TAG="pers=$p $v" timeout -k 10 120 python3 tools/attn_probe.py >> gpurun_out/r05h/ladder.log 2>&1 || { tail -20 gpurun_out/r05h/ladder.log; exit 1; }
    done
  done
done
unset LTHM_LIB_PATH
grep -v amdgpu.ids gpurun_out/r05h/ladder.log
