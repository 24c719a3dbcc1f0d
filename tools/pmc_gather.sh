#!/bin/bash
# HBM counter passes over the embedding-gather roofline leg alone (tools/gather_bench.py:
# 4.1 GB bf16 table, 524,288 ids, K = 16, spread and reference id sets): FETCH_SIZE and
# WRITE_SIZE in separate passes (MI355X_MICROARCH.md §HBM / PMC slots), split per id set by
# tools/pmc_gather_summary.py into gpurun_out/pmc_gather/gather_pmc.json.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_gather
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_gather/fetch -o run --output-format csv \
  -- python3 tools/gather_bench.py > gpurun_out/pmc_gather/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_gather/write -o run --output-format csv \
  -- python3 tools/gather_bench.py > gpurun_out/pmc_gather/write.log 2>&1
python3 tools/pmc_gather_summary.py gpurun_out/pmc_gather/gather_pmc.json gpurun_out/pmc_gather/fetch \
  gpurun_out/pmc_gather/write > gpurun_out/pmc_gather/summary.txt 2>&1
rm -rf gpurun_out/pmc_gather/fetch gpurun_out/pmc_gather/write
