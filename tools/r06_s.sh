# cost ladder of the KShift sparse backward (C2 bench timer lthm_kshift_bwd_sparse): default,
# no bitonic sort (KSB1), no row atomics (KSB2) -- timing only
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s
mkdir -p $O
for v in base KSB1 KSB2; do
  if [ $v = base ]; then unset LTHM_LIB_PATH; else export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_$v.so; fi
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-gather --no-generator > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  python3 -c "
import json;s=open('$O/$v.log').read();i=s.rfind('{\"metric\"');d=json.loads(s[i:].split(chr(10))[0])
print('$v', d['kernels']['lthm_kshift_bwd_sparse'])"
done
