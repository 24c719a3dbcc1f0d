# Round-4 GPU pass x: GEMM microbench (C4 ranker, C2 encoder, square) against hipBLASLt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04x
GEMM_BENCH_CFG=c4 GEMM_BENCH_SQUARE=1 timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r04x/gemm_c4.log 2>&1 || { tail -20 gpurun_out/r04x/gemm_c4.log; exit 1; }
cat gpurun_out/r04x/gemm_c4.log
timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r04x/gemm_c2.log 2>&1 || { tail -20 gpurun_out/r04x/gemm_c2.log; exit 1; }
cat gpurun_out/r04x/gemm_c2.log
