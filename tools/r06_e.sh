# Round-6 pass e: W2T prefetch (TRPF) A/B of the fused MLP forward + its phase stamps; C4 with the
# K = 1 tables gathered from the fp32 master (no bf16 shadow) A/B; C4 kernel summary
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06e
R=$GRAFT_REPO_ROOT/recommendations_amd
for v in base TRPF base TRPF; do
  if [ $v = base ]; then L=$R/liblthm_hip.so; else L=$R/liblthm_hip_$v.so; fi
  echo -n "$v " >> gpurun_out/r06e/mlp_ab.log
  LTHM_LIB_PATH=$L timeout -k 10 120 python tools/mlp_bench.py --fused-only --iters 20 2>/dev/null >> gpurun_out/r06e/mlp_ab.log || exit 1
done
cat gpurun_out/r06e/mlp_ab.log
LTHM_LIB_PATH=$R/liblthm_hip_TRPFST.so timeout -k 10 120 python tools/mlp_stamp.py > gpurun_out/r06e/stamp_trpf.json 2> gpurun_out/r06e/stamp.err || { tail -20 gpurun_out/r06e/stamp.err; exit 1; }
cat gpurun_out/r06e/stamp_trpf.json
for a in 1 0 1 0; do
  LTHM_C4_GATHER_BF16=$a timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --no-hbm-gather --no-cpu-baseline > gpurun_out/r06e/c4_g$a.log 2>&1 || { tail -20 gpurun_out/r06e/c4_g$a.log; exit 1; }
  python3 - gpurun_out/r06e/c4_g$a.log g$a <<'PY'
import json, sys
s = open(sys.argv[1]).read(); j = json.loads(s[s.rfind('{"metric'):].split('\n')[0]); k = j.get('kernels', {})
print(sys.argv[2], j['ms_per_step'], {n: round(v['avg_ms'], 4) for n, v in k.items() if v['avg_ms'] * v['calls_per_step'] > 0.05})
PY
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06e/c4prof -o run -- python3 bench.py --config c4 --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/r06e/c4prof.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find gpurun_out/r06e/c4prof -name "*.db" | head -1) 30 > gpurun_out/r06e/c4_kernel_stats.txt 2>&1
head -20 gpurun_out/r06e/c4_kernel_stats.txt
rm -rf gpurun_out/r06e/c4prof
