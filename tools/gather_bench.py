"""Embedding gather roofline leg on its own (bench.py embedding_gather_hbm), for the
rocprofv3 counter passes of tools/pmc_passes.sh:

    rocprofv3 --pmc FETCH_SIZE -- python tools/gather_bench.py
    rocprofv3 --pmc WRITE_SIZE -- python tools/gather_bench.py

Prints the bench's JSON for the gather (4.1 GB bf16 table, 524,288 ids, K = 16; the
spread and the reference id sets, 10 timed launches each after one warm-up)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import embedding_gather_hbm  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(embedding_gather_hbm(torch.device("cuda:0"))))
