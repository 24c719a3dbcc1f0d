# Round-4 GPU pass am: C2 env A/B: per-phase DMA issue in the 256x256 GEMM (A, default) vs all behind the barrier (B)
cd $GRAFT_REPO_ROOT
for v in A B A B; do
  if [ $v = B ]; then export LTHM_GEMM_PP=2; else unset LTHM_GEMM_PP; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/abpp_$v.log 2>&1 || { tail -20 gpurun_out/abpp_$v.log; exit 1; }
  python3 - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/abpp_{sys.argv[1]}.log").read().splitlines():
    if l.startswith('{"metric"'):
        d = json.loads(l)
        ks = ["enc:gemm_k<1,1>", "enc:mlp_bwd"]
        print(sys.argv[1], d["value"], d["ms_per_step"], " ".join(f"{k}={d['kernels'][k]['avg_ms']}" for k in ks))
PY
done
