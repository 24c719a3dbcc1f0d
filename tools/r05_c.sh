# Round-5 GPU pass c: MLP tests + microbench only (iterating on mlp_wgrad_k / mlp_bwd_dx)
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05c}
mkdir -p gpurun_out
export PARITY_LOG=gpurun_out/${TAG}_mlp_parity.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_mlp_tests.log 2>&1
rc=$?; echo "mlp tests rc=$rc"; tail -2 gpurun_out/${TAG}_mlp_tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/${TAG}_mlp_tests.log | head -30; exit $rc; }
timeout -k 10 200 python tools/mlp_bench.py --bwd --fused-only --iters 10 > gpurun_out/${TAG}_mlp_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_mlp_bench.log; exit 1; }
cat gpurun_out/${TAG}_mlp_bench.log
