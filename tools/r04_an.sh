# Round-4 GPU pass an: shape-dependent DMA issue placement in the 256x256 GEMM: tests, C2 bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04an
export PARITY_LOG=gpurun_out/r04an/parity.json
timeout -k 10 500 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_lthm.py tests/test_gpu_lthm_step_golden.py tests/test_gpu_ranker.py tests/test_gpu_fp8.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04an/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04an/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04an/tests.log | head -30; exit 1; }
n=gpurun_out/r04an/bench_c2.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
grep -o '"value": [0-9.]*, "unit": "samples/s", "n_gpus": 1, "steps": 10, "warmup": 3, "ms_per_step": [0-9.]*' $n
