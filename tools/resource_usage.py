"""Print VGPR / scratch / occupancy of every gfx950 kernel in csrc/ (hipcc -Rpass-analysis)."""
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    files = sys.argv[1:] or sorted(glob.glob(os.path.join(ROOT, "recommendations_amd", "csrc", "*.hip")))
    for f in files:
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
                            "-c", f, "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
        cur = None
        for line in r.stderr.splitlines():
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                cur = {"name": m.group(1)}
                continue
            for key in ("VGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
                m = re.search(key + r": (\d+)", line)
                if m and cur is not None:
                    cur[key.split()[0]] = int(m.group(1))
            if cur is not None and "LDS" in cur:
                flag = " <-- SCRATCH" if cur.get("ScratchSize", 0) else ""
                print(f"{os.path.basename(f):14s} {cur['name'][:70]:70s} vgpr={cur.get('VGPRs')} "
                      f"scratch={cur.get('ScratchSize')} occ={cur.get('Occupancy')} lds={cur['LDS']}{flag}")
                cur = None


if __name__ == "__main__":
    main()
