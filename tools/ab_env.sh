# A/B a kernel-variant environment switch on the C2 bench: bash tools/ab_env.sh VAR "v1 v2 ..." [kernel-key]
VAR=$1; VALS=$2; KEY=${3:-cl_bwd_k}
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/ab_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels'].get('$KEY', {}); print('$VAR=$v', d['value'], d['ms_per_step'], k.get('avg_ms'))"
done
