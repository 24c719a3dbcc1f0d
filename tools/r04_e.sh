# Round-4 GPU pass e: fused MLP forward with the half-chunk lag of waves 4-7 (LTHM_MLP_STAG=1):
# parity, timing A/B, SQ counters of both forms; C2 step A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04e
export PARITY_LOG=gpurun_out/r04e/parity.json
LTHM_MLP_STAG=1 timeout -k 10 240 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_encoder.py tests/test_gpu_tables.py tests/test_gpu_lthm.py tests/test_gpu_lthm_step_golden.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r04e/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04e/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED" gpurun_out/r04e/tests.log | head; exit 1; }
LTHM_MLP_PIPE=1 timeout -k 10 240 python -u -m pytest tests/test_gpu_mlp.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r04e/tests_pipe.log 2>&1
rc=$?; echo "pipe tests rc=$rc"; tail -2 gpurun_out/r04e/tests_pipe.log
[ $rc -eq 0 ] || { grep -E "^FAILED" gpurun_out/r04e/tests_pipe.log | head; exit 1; }
for st in 0 1; do LTHM_MLP_STAG=$st timeout -k 10 120 python -u tools/mlp_bench.py --fused-only --bwd --iters 20 || exit 1; done
LTHM_MLP_PIPE=1 timeout -k 10 120 python -u tools/mlp_bench.py --fused-only --iters 20 || exit 1
for c in c4 c5; do for bt in 0 1; do echo "gemm $c bt=$bt"; GEMM_BENCH_CFG=$c LTHM_GEMM_BT=$bt timeout -k 10 200 python -u tools/gemm_bench.py || exit 1; done; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for st in 0 1; do
  export LTHM_MLP_STAG=$st
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/r04e/pmc_sq_$st -o run --output-format csv -- python3 tools/mlp_bench.py --fused-only --iters 3 > gpurun_out/r04e/pmc_sq_$st.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/r04e/pmc_sq2_$st -o run --output-format csv -- python3 tools/mlp_bench.py --fused-only --iters 3 > gpurun_out/r04e/pmc_sq2_$st.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/r04e/pmc_$st.json gpurun_out/r04e/pmc_sq_$st gpurun_out/r04e/pmc_sq2_$st && grep -A12 '"mlp_fwd_k' gpurun_out/r04e/pmc_$st.json | head -16
done
unset LTHM_MLP_STAG
rm -rf gpurun_out/r04e/pmc_sq_* gpurun_out/r04e/pmc_sq2_*
for st in "LTHM_MLP_STAG=1" "LTHM_MLP_PIPE=1" "LTHM_MLP_STAG=0"; do
  n=gpurun_out/r04e/bench_c2_${st//=/}.log
  env $st timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
  python3 - $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], {k: v["avg_ms"] for k, v in d["kernels"].items() if k.startswith("enc:mlp")})
PY
done
