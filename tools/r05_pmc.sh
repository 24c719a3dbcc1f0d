# Round-5 PMC passes over the default (C2) bench: FETCH_SIZE, WRITE_SIZE and the SQ counters in
# separate runs (MI355X_MICROARCH.md HBM section), summarised per kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc5
B="--steps 2 --warmup 1 --no-cpu-baseline --no-hbm-gather --no-kernel-timing"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc5/fetch -o run --output-format csv -- python3 bench.py $B > gpurun_out/pmc5/fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc5/write -o run --output-format csv -- python3 bench.py $B > gpurun_out/pmc5/write.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc5/sq -o run --output-format csv -- python3 bench.py $B > gpurun_out/pmc5/sq.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc5/summary.json gpurun_out/pmc5/fetch gpurun_out/pmc5/write gpurun_out/pmc5/sq > gpurun_out/pmc5/summary.txt 2>&1
head -12 gpurun_out/pmc5/summary.txt | cut -c1-200
rm -rf gpurun_out/pmc5/fetch gpurun_out/pmc5/write gpurun_out/pmc5/sq
