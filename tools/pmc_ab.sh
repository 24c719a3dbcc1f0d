# SQ / TCC counters of the kernels matching $FILTER while running $PROG, per variant of
# the A/B switch $SWITCH (variants: old = $SWITCH=1, new = $SWITCH=0); one --pmc pass each
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
out=gpurun_out/pmc_ab
mkdir -p $out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for v in ${VARIANTS:-old new}; do
  if [ $v = old ]; then export $SWITCH=1; else export $SWITCH=0; fi
  for p in 1 2 3 4; do
    eval cs=\$P$p
    timeout -s KILL 120 rocprofv3 --pmc $cs --kernel-trace -d $out/$v$p -o run --output-format csv -- python3 $PROG > $out/$v$p.log 2>&1 || exit 1
  done
done
python3 - <<PY
import csv, glob, collections
for v in "${VARIANTS:-old new}".split():
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for p in (1, 2, 3, 4):
        f = glob.glob(f"$out/{v}{p}/**/*counter_collection.csv", recursive=True)
        if not f:
            print(v, p, "no csv"); continue
        for r in csv.DictReader(open(f[0])):
            k = r["Kernel_Name"]
            if "$FILTER" not in k: continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        print(v, k[:60])
        for c, val in sorted(d.items()):
            print(f"    {c:28s} {val / n[(k, c)]:.4e}")
PY
