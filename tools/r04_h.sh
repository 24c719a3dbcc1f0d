# Round-4 GPU pass h: loss-kernel cost ladder (CL_EXP 2..6 variants of the default SP2+PF build,
# each timed alone under --kernel-trace) and two SQ counter passes of the default build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04h
for v in base exp2 exp3 exp4 exp5 exp6; do
  if [ $v = base ]; then export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip.so
  else export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r04h/lexp_$v -o run -- python3 tools/loss_bench.py > gpurun_out/r04h/lexp_$v.log 2>&1 || { tail -5 gpurun_out/r04h/lexp_$v.log; exit 1; }
  echo "== $v $(grep fwd+bwd gpurun_out/r04h/lexp_$v.log | tail -1)"
  python3 tools/rocpd_stats.py $(find gpurun_out/r04h/lexp_$v -name "*.db" | head -1) 4
done
unset LTHM_LIB_PATH
rm -rf gpurun_out/r04h/lexp_*/
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/r04h/pmc1 -o run --output-format csv -- python3 tools/loss_bench.py > gpurun_out/r04h/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-trace -d gpurun_out/r04h/pmc2 -o run --output-format csv -- python3 tools/loss_bench.py > gpurun_out/r04h/pmc2.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/r04h/pmc.json gpurun_out/r04h/pmc1 gpurun_out/r04h/pmc2
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r04h/pmc.json"))
for k, v in d.items():
    if k.startswith("cl_"):
        print(k, {c: f"{x:.3e}" for c, x in sorted(v.items())})
PY
rm -rf gpurun_out/r04h/pmc1 gpurun_out/r04h/pmc2
