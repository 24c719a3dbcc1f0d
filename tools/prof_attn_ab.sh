# attention backward A/B: encoder/attention GPU tests, then the C2 bench under
# rocprofv3 --kernel-trace with the round-2 16x16x32 kernel (old) and the 32x32x16 one (new)
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encoder.py > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -3 gpurun_out/attn_tests.log
for v in ${VARIANTS:-old new}; do
  if [ $v = old ]; then export LTHM_ATTN_BWD_OLD=1; else export LTHM_ATTN_BWD_OLD=0; fi
  timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/aprof_$v -o run -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/abench_$v.log 2>&1 || exit 1
  echo "== $v $(tail -1 gpurun_out/abench_$v.log | cut -c1-200)"
  python3 tools/rocpd_stats.py $(find gpurun_out/aprof_$v -name "*.db" | head -1) 12
done
