"""Aggregate rocprofv3 --pmc counter CSVs into per-kernel means per dispatch.

usage: python tools/pmc_summary.py OUT.json DIR [DIR ...]

Each DIR is one rocprofv3 pass (``-d DIR --output-format csv``).  Counters are
averaged over the dispatches of each kernel (name shortened to the symbol
before the argument list).  HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md
§HBM: FETCH_SIZE (KiB) is doubled on gfx950 for wide coalesced reads,
WRITE_SIZE (KiB) is taken as is; ``hbm_bytes`` = 1024 * (2 * FETCH_SIZE + WRITE_SIZE).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    name = name.split("(")[0]
    return name.replace("lthm::", "")


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", ""))
                    acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_bytes"] = 1024.0 * (2.0 * m["FETCH_SIZE"] + m["WRITE_SIZE"])
        res[k] = m
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    top = sorted(res.items(), key=lambda kv: -kv[1].get("hbm_bytes", 0.0))[:20]
    for k, m in top:
        print(f"{k[:60]:60s} " + " ".join(f"{c}={v:.4g}" for c, v in sorted(m.items()) if c != "dispatches"))


if __name__ == "__main__":
    main()
