# Round-4 GPU pass ao: C2 env A/B: fused MLP forward with 4 waves per workgroup (B) vs 8 (A)
cd $GRAFT_REPO_ROOT
for v in A B A B; do
  if [ $v = B ]; then export LTHM_MLP_NW=4; else unset LTHM_MLP_NW; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/abnw_$v.log 2>&1 || { tail -20 gpurun_out/abnw_$v.log; exit 1; }
  python3 - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/abnw_{sys.argv[1]}.log").read().splitlines():
    if l.startswith('{"metric"'):
        d = json.loads(l)
        ks = ["enc:mlp_fwd", "enc:mlp_bwd"]
        print(sys.argv[1], d["value"], d["ms_per_step"], " ".join(f"{k}={d['kernels'][k]['avg_ms']}" for k in ks))
PY
done
