# Round-6 pass c: C2 step A/B of the round-6 kernels, one bench process per arm (the switches
# are read once per process): default / LTHM_MLP_FWD2=0 / LTHM_MLP_BWDP2=0 / the EPR=4 gemm
# library; then C4 with the keep-grad row-wise AdamW and its A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06c
B="--steps 20 --warmup 5 --no-cpu-baseline --no-hbm-gather"
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py $B > gpurun_out/r06c/$tag.log 2>&1 || { tail -20 gpurun_out/r06c/$tag.log; return 1; }
  python3 - gpurun_out/r06c/$tag.log $tag <<'PY'
import json, sys
s = open(sys.argv[1]).read(); j = json.loads(s[s.rfind('{"metric'):].split('\n')[0]); k = j.get('kernels', {})
f = lambda n: (round(k[n]['avg_ms'], 4) if n in k else None)
print(sys.argv[2], j['ms_per_step'], 'mlp_fwd', f('enc:mlp_fwd'), 'mlp_bwd', f('enc:mlp_bwd'), 'dgrad_ln', f('enc:dgrad_ln'),
      'linear_ln', f('enc:linear_ln'), 'logq', f('logq_stream'), 'kshift_fwd', f('kshift_fwd_k'))
PY
}
L8=LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_EPR8.so
run base LTHM_X=1 || exit 1
run fwd2 LTHM_MLP_FWD2=1 || exit 1
run bwdp2 LTHM_MLP_BWDP2=1 || exit 1
run epr8 $L8 || exit 1
run all LTHM_MLP_FWD2=1 LTHM_MLP_BWDP2=1 LTHM_KSHIFT_REG=1 $L8 || exit 1
run base2 LTHM_X=1 || exit 1
LTHM_SPARSE_KEEP_GRAD=1 timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --no-hbm-gather --no-cpu-baseline > gpurun_out/r06c/c4.log 2>&1 || { tail -20 gpurun_out/r06c/c4.log; exit 1; }
tail -c 300 gpurun_out/r06c/c4.log; echo
LTHM_SPARSE_KEEP_GRAD=0 timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --no-hbm-gather --no-cpu-baseline > gpurun_out/r06c/c4_zg.log 2>&1 || { tail -20 gpurun_out/r06c/c4_zg.log; exit 1; }
tail -c 300 gpurun_out/r06c/c4_zg.log; echo
for f in c4 c4_zg; do python3 - gpurun_out/r06c/$f.log $f <<'PY'
import json, sys
s = open(sys.argv[1]).read(); j = json.loads(s[s.rfind('{"metric'):].split('\n')[0]); k = j.get('kernels', {})
print(sys.argv[2], j['ms_per_step'], {n: round(v['avg_ms'], 4) for n, v in k.items() if v['avg_ms'] * v['calls_per_step'] > 0.05})
PY
done
