# Round-4 GPU pass al: C2 attention backward with 8 waves per (b, h) (B) vs 4 (A); parity of B first
cd $GRAFT_REPO_ROOT
export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_B.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r04al_tests_B.log 2>&1
rc=$?; echo "B tests rc=$rc"; tail -1 gpurun_out/r04al_tests_B.log
[ $rc -eq 0 ] || exit 1
unset LTHM_LIB_PATH
KEYS="attn_bwd_k attn_fwd_k" bash tools/ab_lib.sh
