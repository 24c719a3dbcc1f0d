# phase stamps of the fused MLP forward and hidden backward (STAMP build)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06k
mkdir -p $O
LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_STAMP.so timeout -k 10 200 python tools/mlp_stamp.py > $O/stamp.json 2> $O/stamp.err || { tail -20 $O/stamp.err; exit 1; }
cat $O/stamp.json
