# Round-5 GPU pass d: PMC counters of the two round-5 MLP backward kernels (mlp_bwdx_k, mlp_wgrad_k)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_mlp5
B="tools/mlp_bench.py --only bwd_dx,bwd_wgrad --iters 3"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/pmc_mlp5/sq -o run --output-format csv -- python3 $B > gpurun_out/pmc_mlp5/sq.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_mlp5/sq2 -o run --output-format csv -- python3 $B > gpurun_out/pmc_mlp5/sq2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY --kernel-trace -d gpurun_out/pmc_mlp5/sq3 -o run --output-format csv -- python3 $B > gpurun_out/pmc_mlp5/sq3.log 2>&1 || true
python3 tools/pmc_summary.py gpurun_out/pmc_mlp5/summary.json gpurun_out/pmc_mlp5/sq gpurun_out/pmc_mlp5/sq2 gpurun_out/pmc_mlp5/sq3 > gpurun_out/pmc_mlp5/summary.txt 2>&1
grep -E "mlp_bwdx|mlp_wgrad_k" gpurun_out/pmc_mlp5/summary.txt
rm -rf gpurun_out/pmc_mlp5/sq gpurun_out/pmc_mlp5/sq2 gpurun_out/pmc_mlp5/sq3
