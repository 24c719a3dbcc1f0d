# Loss-kernel variants (tools/build_variant.sh) timed alone under rocprofv3 --kernel-trace:
# VARIANTS="base exp2 ..." -> per variant the fwd+bwd event time and the top loss kernels
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_$v.so
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/lexp_$v -o run -- python3 tools/loss_bench.py > gpurun_out/lexp_$v.log 2>&1 || { tail -5 gpurun_out/lexp_$v.log; exit 1; }
  echo "== $v $(grep fwd+bwd gpurun_out/lexp_$v.log | tail -1)"
  python3 tools/rocpd_stats.py $(find gpurun_out/lexp_$v -name "*.db" | head -1) 4
done
