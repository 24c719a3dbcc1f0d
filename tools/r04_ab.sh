# Round-4 GPU pass ab: fp8 form of the 256x256 GEMM: fp8 tests, microbench on/off, C5 bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ab
export LTHM_GEMM_PP_F8=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ab/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04ab/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04ab/tests.log | head -30; exit 1; }
GEMM_BENCH_FP8=1 GEMM_BENCH_CFG=c5 GEMM_BENCH_SQUARE=1 timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r04ab/gemm_c5.log 2>&1 || exit 1
LTHM_GEMM_PP_F8=0 LTHM_GEMM_PP=0 GEMM_BENCH_FP8=1 GEMM_BENCH_CFG=c5 GEMM_BENCH_SQUARE=1 timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r04ab/gemm_c5_off.log 2>&1 || exit 1
for m in 2 3 4; do
  LTHM_GEMM_PP=$m GEMM_BENCH_FP8=1 GEMM_BENCH_CFG=c5 GEMM_BENCH_SQUARE=1 timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r04ab/gemm_c5_m$m.log 2>&1 || exit 1
done
for m in 1 2 3 4; do
  LTHM_GEMM_PP=$m GEMM_BENCH_CFG=c4 timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r04ab/gemm_c4_m$m.log 2>&1 || exit 1
done
python3 tools/gemm_ab_table.py gpurun_out/r04ab
n=gpurun_out/r04ab/bench_c5_f8off.log
LTHM_GEMM_PP_F8=0 timeout -k 10 400 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
grep -o '"value": [0-9.]*, "unit": "samples/s", "n_gpus": 1, "steps": 10, "warmup": 3, "ms_per_step": [0-9.]*' $n
n=gpurun_out/r04ab/bench_c5.log
timeout -k 10 400 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
python3 - $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"])
        for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["share"])[:8]:
            print("   ", k, v["avg_ms"], v["calls_per_step"], round(v["avg_ms"] * v["calls_per_step"], 3))
PY
