# Round-4 GPU pass c: the tests that failed in pass b, then the C2 bench with the fused MLP
# (default) and without it (LTHM_MLP_TRAIN=0), and a rocprof kernel summary of the default bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PARITY_LOG=gpurun_out/r04c_parity.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_lthm.py tests/test_gpu_wrapper_api.py tests/test_gpu_mlp.py tests/test_gpu_fp8.py tests/test_gpu_gemm_bigk.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04c_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/r04c_bench.log 2>&1 || { tail -20 gpurun_out/r04c_bench.log; exit 1; }
LTHM_MLP_TRAIN=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/r04c_bench_nomlp.log 2>&1 || { tail -20 gpurun_out/r04c_bench_nomlp.log; exit 1; }
python3 - <<'PY'
import json
for f in ["gpurun_out/r04c_bench.log", "gpurun_out/r04c_bench_nomlp.log"]:
    for l in open(f):
        if l.startswith('{"metric"'):
            d = json.loads(l)
            print(f, d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"], d.get("encoder_gemm", {}).get("frac"))
            for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["share"])[:14]:
                print("   ", k, v["avg_ms"], v["calls_per_step"], v["share"], v.get("TFLOP/s"))
PY
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r04c_prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/r04c_prof.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find gpurun_out/r04c_prof -name "*.db" | head -1) 40 > gpurun_out/r04c_kernel_stats.txt
head -25 gpurun_out/r04c_kernel_stats.txt
VARIANTS="base pf sp2 pfsp2 exp5 pfexp5 exp6 pfexp6" bash tools/r04_loss_exp.sh > gpurun_out/r04c_lossexp.log 2>&1; echo "lossexp rc=$?"
grep -E "^==|cl_fr32|cl_bwd32" gpurun_out/r04c_lossexp.log
LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_pfsp2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_loss_golden.py tests/test_gpu_loss.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r04c_pfsp2_golden.log 2>&1; echo "pfsp2 goldens rc=$?"; tail -1 gpurun_out/r04c_pfsp2_golden.log
