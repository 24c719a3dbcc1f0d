# Round-4 GPU pass p: GEMM microbench (C2, C4 shapes) with hipBLASLt as a yardstick
cd $GRAFT_REPO_ROOT
for c in c2 c4; do echo "== $c"; GEMM_BENCH_CFG=$c timeout -k 10 200 python -u tools/gemm_bench.py || exit 1; done
