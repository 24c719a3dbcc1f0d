"""Per-kernel stats (calls, average / total ms) from a rocprofv3 rocpd SQLite database
(the default output of `rocprofv3 --kernel-trace` on ROCm 7.2):
    python3 tools/rocpd_stats.py gpurun_out/prof_x/run_results.db [top]"""
import sqlite3
import sys


def stats(path, top=20):
    con = sqlite3.connect(path)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    rows = cur.execute(f"select s.kernel_name, count(*), avg(d.end - d.start), sum(d.end - d.start) "
                       f"from {disp} d join {sym} s on d.kernel_id = s.id group by s.kernel_name "
                       f"order by sum(d.end - d.start) desc").fetchall()
    out = []
    for name, n, avg, tot in rows[:top]:
        out.append((name, n, avg / 1e6, tot / 1e6))
    return out


if __name__ == "__main__":
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    for name, n, avg, tot in stats(sys.argv[1], top):
        print(f"{tot:10.3f} ms {n:6d} x {avg:8.4f} ms  {name[:110]}")
