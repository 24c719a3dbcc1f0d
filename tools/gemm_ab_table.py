"""Condense tools/gemm_bench.py logs of one directory into fwd / dgrad-via-W^T / fp8 columns."""
import glob
import os
import re
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "gemm_*.log"))):
    for line in open(f):
        m = re.match(r"(\S+)\s+M=.*?fwd ([\d.]+) ms.*?via W\^T ([\d.]+).*?fp8 fwd ([\d.na]+)", line)
        if m:
            print(f"{os.path.basename(f):22s} {m.group(1):7s} fwd {m.group(2)}  dgradT {m.group(3)}  fp8 {m.group(4)}")
