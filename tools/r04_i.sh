# Round-4 GPU pass i: valid-row compaction of the training loss passes: parity (loss tests,
# goldens, wrapper API, full steps), loss-kernel timing (compact vs full), C2 bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04i
export PARITY_LOG=gpurun_out/r04i/parity.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_loss_golden.py tests/test_gpu_wrapper_api.py tests/test_gpu_lthm.py tests/test_gpu_lthm_step_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04i/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04i/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r04i/tests.log | head -20; exit 1; }
grep "vc " gpurun_out/r04i/tests.log | head
for v in 1 0; do
  LTHM_CL_VC=$v timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r04i/lb_$v -o run -- python3 tools/loss_bench.py > gpurun_out/r04i/lb_$v.log 2>&1 || { tail -5 gpurun_out/r04i/lb_$v.log; exit 1; }
  echo "== vc=$v $(grep fwd+bwd gpurun_out/r04i/lb_$v.log | tail -1)"
  python3 tools/rocpd_stats.py $(find gpurun_out/r04i/lb_$v -name "*.db" | head -1) 8
done
rm -rf gpurun_out/r04i/lb_*/
n=gpurun_out/r04i/bench_c2.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
python3 - $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(d["value"], d["ms_per_step"], json.dumps(d["roofline"]))
        for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["share"])[:12]:
            print("   ", k, v["avg_ms"], v["calls_per_step"], v["share"], v.get("TFLOP/s"))
PY
