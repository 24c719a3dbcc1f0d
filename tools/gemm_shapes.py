"""Per-dispatch GEMM durations of one C2 training step from a rocprofv3 kernel trace
(python3 tools/gemm_shapes.py gpurun_out/<dir>/run_kernel_trace.csv): grid size ->
(tiles, batch, splits) and duration, grouped by kernel and grid."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"]
    if "gemm_" not in k and "splitk" not in k:
        continue
    key = (k.split("(")[0].replace("void lthm::", ""), r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"],
           r.get("LDS_Block_Size", ""))
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
for key, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    print(f"{key[0]:28s} grid=({key[1]},{key[2]},{key[3]}) n={len(v):4d} avg={sum(v) / len(v):8.1f} us "
          f"total={sum(v) / 1e3:8.2f} ms")
print(f"total {tot / 1e3:.2f} ms")
