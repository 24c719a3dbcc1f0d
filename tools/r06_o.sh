# fused generator Adagrad: parity tests and the step A/B after the packed prep kernel
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kshift_adagrad.py tests/test_gpu_embgen.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/tests.log | head -40; exit $rc; }
timeout -k 10 300 python tools/embgen_bench.py > $O/embgen_bench.log 2>&1 || { tail -20 $O/embgen_bench.log; exit 1; }
grep model $O/embgen_bench.log
