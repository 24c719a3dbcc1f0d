# SQ counters of the loss kernels (tools/loss_bench.py), old vs 32x32x16 backward; one pass each
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_loss
for v in old new; do
  if [ $v = old ]; then export LTHM_CL_BWD_OLD=1; else export LTHM_CL_BWD_OLD=0; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc_loss/$v -o run --output-format csv -- python3 tools/loss_bench.py > gpurun_out/pmc_loss/$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for v in ("old", "new"):
    f = glob.glob(f"gpurun_out/pmc_loss/{v}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(v, "no csv", glob.glob(f"gpurun_out/pmc_loss/{v}/**/*", recursive=True)[:10]); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "cl_bwd" not in k and "cl_fwd" not in k: continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        calls = max(n[(k, c)] for c in d)
        print(v, k[:40], "calls", calls, {c: f"{val / calls:.3e}" for c, val in sorted(d.items())})
PY
