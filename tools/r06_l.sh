# new parity cases: C5 at full depth, the persistent attention backward vs the default; the fused
# generator Adagrad tests and step A/B after the pipelined pair loads
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06l
mkdir -p $O
export PARITY_LOG=$O/parity.json
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread "tests/test_gpu_lthm.py::test_lthm_c5_all_layers_fp8_vs_oracle" "tests/test_gpu_encoder.py::test_attention_persistent_bwd_matches_default" tests/test_gpu_kshift_adagrad.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "6 layers|persistent" $O/tests.log | sort -g | tail -8
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/tests.log | head -40; exit $rc; }
timeout -k 10 300 python tools/embgen_bench.py > $O/embgen_bench.log 2>&1 || { tail -20 $O/embgen_bench.log; exit 1; }
grep model $O/embgen_bench.log
