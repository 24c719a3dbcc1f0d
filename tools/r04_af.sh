# Round-4 GPU pass af: C2 A/B of the weight-gradient kernel on any row count (A) vs K % 32 == 0 only (B)
cd $GRAFT_REPO_ROOT
for v in A B A B; do
  if [ $v = B ]; then export LTHM_WG_RAGGED=0; else unset LTHM_WG_RAGGED; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/abwg_$v.log 2>&1 || { tail -20 gpurun_out/abwg_$v.log; exit 1; }
  python3 - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/abwg_{sys.argv[1]}.log").read().splitlines():
    if l.startswith('{"metric"'):
        d = json.loads(l)
        ks = ["enc:gemm_k<0,0>", "gemm_k<0,0>", "enc:gemm_k<1,1>", "gemm_k<1,1>"]
        print(sys.argv[1], d["value"], d["ms_per_step"], " ".join(f"{k}={d['kernels'][k]['avg_ms']}x{d['kernels'][k]['calls_per_step']}" for k in ks if k in d["kernels"]))
PY
done
