# A/B: dgrad GEMMs on the K-strided W (default) vs a K-contiguous W^T copy (LTHM_DGRAD_WT=1),
# C2 and C5 bench lines alternating on one box
cd $GRAFT_REPO_ROOT
for c in c5 c2; do
  for m in 0 1 0 1; do
    LTHM_DGRAD_WT=$m timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-gather > gpurun_out/r03f_ab_${c}_$m.log 2>&1 || { tail -5 gpurun_out/r03f_ab_${c}_$m.log; exit 1; }
    python3 -c "
import json,sys
for l in open('gpurun_out/r03f_ab_${c}_$m.log'):
    if l.startswith('{\"metric\"'): d=json.loads(l)
k=d['kernels']; e=[v for n,v in k.items() if n.endswith('gemm_k<1,0>') or n.endswith('gemm_k<1,1>')]
print('$c WT=$m', d['value'], d['ms_per_step'], {n:(v['calls_per_step'],v['avg_ms']) for n,v in k.items() if 'gemm_k<1' in n})"
  done
done
