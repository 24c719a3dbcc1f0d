# fused loss pass block order A/B on C2 (LTHM_CL_FR_XCD=1: XCD-remapped), alternating, with kernel trace
cd $GRAFT_REPO_ROOT
for v in 0 1 0 1; do
  LTHM_CL_FR_XCD=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/frx_$v.log 2>&1 || exit 1
  python3 - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/frx_{sys.argv[1]}.log").read().splitlines():
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print("xcd=" + sys.argv[1], d["value"], d["ms_per_step"], "cl_fwd_k", d["kernels"]["cl_fwd_k"]["avg_ms"])
PY
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1; do
  LTHM_CL_FR_XCD=$v timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/frx_pmc$v -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/frx_pmc$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for v in (0, 1):
    f = glob.glob(f"gpurun_out/frx_pmc{v}/**/*counter_collection.csv", recursive=True)[0]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "cl_fr32_k" in r["Kernel_Name"]]
    print("xcd", v, "cl_fr32_k FETCH_SIZE KiB per dispatch", sum(vals) / max(len(vals), 1), len(vals))
PY
