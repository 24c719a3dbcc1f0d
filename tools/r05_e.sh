# Round-5 GPU pass e: C2 bench A/B of the MLP backward (LTHM_MLP_WG=1: lthm_mlp_bwd_dx +
# lthm_mlp_wgrad; 0: the round-4 chain), alternating, two runs each
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05e
for v in 1 0 1 0; do
  LTHM_MLP_WG=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-hbm-gather --steps 10 --warmup 3 > gpurun_out/r05e/ab_$v.log 2>&1 || { tail -20 gpurun_out/r05e/ab_$v.log; exit 1; }
  tail -1 gpurun_out/r05e/ab_$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
mk=[x for x in k if 'mlp' in x or x.startswith('enc:gemm')]
print('WG=$v', d['value'], d['ms_per_step'], ' '.join(f\"{x}={k[x]['avg_ms']}x{k[x]['calls_per_step']}\" for x in sorted(mk)), 'roof', d['roofline']['kernel'], d['roofline']['frac'])"
done
