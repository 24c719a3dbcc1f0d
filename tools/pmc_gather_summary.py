"""HBM bytes per launch of the embedding-gather roofline leg (tools/gather_bench.py under
tools/pmc_gather.sh), split into its two id sets: the kshift dispatches run in order, the first
half on the spread ids and the second half on the reference ids (bench.py embedding_gather_hbm).

usage: python tools/pmc_gather_summary.py OUT.json FETCH_DIR WRITE_DIR

hbm_bytes = 1024 x (2 x FETCH_SIZE + WRITE_SIZE) per dispatch, the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md (FETCH_SIZE counts half of a 16-B-per-lane streaming read)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

N, P, D, K = 524_288, 16_000_000, 128, 16
ALGO = N * (8 + K * D * 2 + D * 2)


def per_dispatch(d, counter):
    vals = defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter or "kshift_fwd" not in row.get("Kernel_Name", ""):
                    continue
                key = int(row.get("Dispatch_Id", row.get("Correlation_Id", 0)))
                vals[key] += float(row["Counter_Value"])
                names[key] = row["Kernel_Name"].split("(")[0].replace("void ", "")
    ids = sorted(vals)
    return [vals[i] for i in ids], [names[i] for i in ids]


def main():
    out, fdir, wdir = sys.argv[1:4]
    fetch, names = per_dispatch(fdir, "FETCH_SIZE")
    write, _ = per_dispatch(wdir, "WRITE_SIZE")
    n = min(len(fetch), len(write))
    half = n // 2
    res = {"kernel": names[0] if names else None,
           "recipe": "tools/pmc_gather.sh (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over "
                     "tools/gather_bench.py); dispatches split in order: first half spread ids, second half "
                     "reference ids",
           "correction": "hbm_bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), MI355X_MICROARCH.md HBM section: "
                         "gfx950 FETCH_SIZE counts half of a 16-B-per-lane streaming read",
           "dispatches_per_set": half}
    for name, sl in (("spread_ids", slice(0, half)), ("reference_ids", slice(half, 2 * half))):
        fs, ws = fetch[sl], write[sl]
        fk, wk = sum(fs) / len(fs), sum(ws) / len(ws)
        hb = 1024.0 * (2.0 * fk + wk)
        res[name] = {"FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk, "hbm_bytes": hb, "algorithmic_bytes": ALGO,
                     "traffic_over_algorithmic": round(hb / ALGO, 4)}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
