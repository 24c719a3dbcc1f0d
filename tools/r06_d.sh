# Round-6 pass d: phase stamps of the fused MLP forward (diagnostic build, tools/mlp_stamp.py)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06d
LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_STAMP.so timeout -k 10 120 python tools/mlp_stamp.py > gpurun_out/r06d/stamp.json 2> gpurun_out/r06d/stamp.err || { tail -20 gpurun_out/r06d/stamp.err; exit 1; }
cat gpurun_out/r06d/stamp.json
