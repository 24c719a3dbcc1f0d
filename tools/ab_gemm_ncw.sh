# persistent GEMM variants: loader waves through registers (LTHM_GEMM_PS_RL=1) with 4 or 8
# compute waves vs LDS-DMA: GEMM / fp8 / encoder GPU tests under RL, then the epilogue probe
cd $GRAFT_REPO_ROOT
for n in 4 8; do
LTHM_GEMM_PS_RL=1 LTHM_GEMM_PS_NCW=$n timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_encoder.py > gpurun_out/ncw_tests_$n.log 2>&1 || { tail -40 gpurun_out/ncw_tests_$n.log; exit 1; }
tail -1 gpurun_out/ncw_tests_$n.log
done
for v in "0 4" "1 4" "1 8"; do set -- $v; echo "RL=$1 NCW=$2"; LTHM_GEMM_PS_RL=$1 LTHM_GEMM_PS_NCW=$2 timeout -k 10 100 python3 tools/gemm_epi_probe.py || exit 1; done
