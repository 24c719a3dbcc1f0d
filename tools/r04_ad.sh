# Round-4 GPU pass ad: r04_ab (fp8 256-tile GEMM, schedule variants, C5 bench) then r04_ac (wgrad kernel)
cd $GRAFT_REPO_ROOT
bash tools/r04_ab.sh || exit 1
bash tools/r04_ac.sh || exit 1
