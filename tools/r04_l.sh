# Round-4 GPU pass l: cost ladder of the compact fused pass (CL_VX 1: no staging / waits /
# barriers in the clean loop, 2: no element work, 3: both) and SQ counters of the default build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04l
for v in base vx1 vx2 vx3; do
  if [ $v = base ]; then export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip.so
  else export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r04l/lb_$v -o run -- python3 tools/loss_bench.py > gpurun_out/r04l/lb_$v.log 2>&1 || { tail -5 gpurun_out/r04l/lb_$v.log; exit 1; }
  echo "== $v $(grep fwd+bwd gpurun_out/r04l/lb_$v.log | tail -1)"
  python3 tools/rocpd_stats.py $(find gpurun_out/r04l/lb_$v -name "*.db" | head -1) 2
done
unset LTHM_LIB_PATH
rm -rf gpurun_out/r04l/lb_*/
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/r04l/pmc1 -o run --output-format csv -- python3 tools/loss_bench.py > gpurun_out/r04l/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-trace -d gpurun_out/r04l/pmc2 -o run --output-format csv -- python3 tools/loss_bench.py > gpurun_out/r04l/pmc2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_INSTS_SMEM --kernel-trace -d gpurun_out/r04l/pmc3 -o run --output-format csv -- python3 tools/loss_bench.py > gpurun_out/r04l/pmc3.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/r04l/pmc.json gpurun_out/r04l/pmc1 gpurun_out/r04l/pmc2 gpurun_out/r04l/pmc3
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r04l/pmc.json"))
for k, v in d.items():
    if k.startswith("cl_fr32v") or k.startswith("cl_bwd32v") or k.startswith("cl_vgather"):
        print(k, {c: f"{x:.3e}" for c, x in sorted(v.items())})
PY
rm -rf gpurun_out/r04l/pmc1 gpurun_out/r04l/pmc2 gpurun_out/r04l/pmc3
