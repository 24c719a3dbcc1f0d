set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_mlp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/pmc_mlp/sq -o run --output-format csv -- python3 tools/mlp_bench.py --fused-only --iters 3 > gpurun_out/pmc_mlp/sq.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_mlp/sq2 -o run --output-format csv -- python3 tools/mlp_bench.py --fused-only --iters 3 > gpurun_out/pmc_mlp/sq2.log 2>&1
