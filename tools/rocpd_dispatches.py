"""Per-dispatch durations of one kernel from a rocprofv3 rocpd SQLite database, split into
equal consecutive groups (e.g. the gather leg's spread-id and reference-id launches):
    python3 tools/rocpd_dispatches.py DB KERNEL_SUBSTRING GROUPS [skip_first_of_each_group]"""
import sqlite3
import sys


def durations(path, name):
    con = sqlite3.connect(path)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    rows = cur.execute(f"select d.end - d.start from {disp} d join {sym} s on d.kernel_id = s.id "
                       f"where s.kernel_name like ? order by d.start", (f"%{name}%",)).fetchall()
    return [r[0] / 1e6 for r in rows]


if __name__ == "__main__":
    ms = durations(sys.argv[1], sys.argv[2])
    groups = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    per = len(ms) // groups
    for g in range(groups):
        part = ms[g * per + skip:(g + 1) * per]
        print(f"group {g}: {len(part)} dispatches, mean {sum(part) / len(part):.4f} ms, "
              f"min {min(part):.4f}, max {max(part):.4f}")
