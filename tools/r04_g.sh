# Round-4 GPU pass g: STAG A/B timing of the fused MLP forward (parity of STAG=1 green in pass f)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04g
for st in 0 1; do LTHM_MLP_STAG=$st timeout -k 10 120 python -u tools/mlp_bench.py --fused-only --bwd --iters 20 || exit 1; done
for st in "LTHM_MLP_STAG=1" "LTHM_MLP_STAG=0"; do
  n=gpurun_out/r04g/bench_c2_${st//=/}.log
  env $st timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
  python3 - $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], {k: v["avg_ms"] for k, v in d["kernels"].items() if k.startswith("enc:mlp")})
PY
done
