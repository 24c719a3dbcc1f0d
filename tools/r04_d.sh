# Round-4 GPU pass d: A/B of the MLP LayerNorm prologue and the big-tile GEMM on C2 / C4 / C5,
# plus the loss tests on the SP2 + PF default build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PARITY_LOG=gpurun_out/r04d_parity.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_bigk.py tests/test_gpu_loss_golden.py tests/test_gpu_loss.py tests/test_gpu_encoder.py tests/test_gpu_mlp.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04d_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ $rc -eq 1 ] && grep -E "^FAILED" gpurun_out/r04d_tests.log | head
for t in 1 0; do LTHM_ATTN_TAIL=$t TAG=tail$t timeout -k 10 120 python -u tools/attn_probe.py || exit 1; done
summ() {
python3 - "$1" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"], d.get("encoder_gemm", {}).get("frac"))
        for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["share"])[:10]:
            print("   ", k, v["avg_ms"], v["calls_per_step"], v["share"], v.get("TFLOP/s"))
PY
}
for v in "c2 LTHM_MLP_LN=1" "c2 LTHM_MLP_LN=0" "c2 LTHM_MLP_NS=2" "c4 LTHM_GEMM_BT=1" "c4 LTHM_GEMM_BT=0" "c5 LTHM_GEMM_BT=1" "c5 LTHM_GEMM_BT=0"; do
  set -- $v
  n=gpurun_out/r04d_bench_$1_${2//=/}.log
  env $2 timeout -k 10 300 python -u bench.py --config $1 --steps 8 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
  summ $n
done
