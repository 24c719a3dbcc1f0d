set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-gather --no-kernel-timing"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc/fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/pmc/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc/write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/pmc/write.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc/sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-hbm-gather --no-kernel-timing > gpurun_out/pmc/sq.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc/summary.json gpurun_out/pmc/fetch gpurun_out/pmc/write gpurun_out/pmc/sq > gpurun_out/pmc/summary.txt 2>&1
