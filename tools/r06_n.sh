# 8-wave persistent attention backward (LTHM_ATTN_BWD_P=8): encoder tests under it, then the C2
# probe alternating default / P=1 / P=8
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06n
mkdir -p $O
LTHM_ATTN_BWD_P=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encoder.py -k "attention and not persistent" > $O/tests_p8.log 2>&1 || { tail -30 $O/tests_p8.log; exit 1; }
tail -2 $O/tests_p8.log
for rep in 1 2; do
  for v in 0 1 8; do
    LTHM_ATTN_BWD_P=$v TAG="P=$v" timeout -k 10 120 python3 tools/attn_probe.py >> $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
  done
done
grep "P=" $O/probe.log
