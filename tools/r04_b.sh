# Round-4 GPU pass b: new / changed parity tests, the loss-kernel experiment variants, a short C2 bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PARITY_LOG=gpurun_out/r04b_parity.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm_bigk.py tests/test_gpu_mlp.py tests/test_gpu_encoder.py tests/test_gpu_wrapper_api.py tests/test_gpu_lthm_step_golden.py tests/test_gpu_loss.py tests/test_gpu_loss_golden.py tests/test_gpu_lthm.py -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04b_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
[ $rc -eq 1 ] && grep -E "^FAILED|Error" gpurun_out/r04b_tests.log | head -20
VARIANTS="base exp2 exp3 exp4 exp5 l3 sp2" bash tools/r04_loss_exp.sh || exit 1
LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_sp2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_loss_golden.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r04b_sp2_golden.log 2>&1; echo "sp2 goldens rc=$?"; tail -1 gpurun_out/r04b_sp2_golden.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/r04b_bench.log 2>&1 || { tail -20 gpurun_out/r04b_bench.log; exit 1; }
tail -c 1500 gpurun_out/r04b_bench.log; echo
LTHM_MLP_TRAIN=0 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/r04b_bench_nomlp.log 2>&1 || { tail -20 gpurun_out/r04b_bench_nomlp.log; exit 1; }
tail -c 300 gpurun_out/r04b_bench_nomlp.log; echo
