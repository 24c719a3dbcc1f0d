# Round-4 GPU pass f (re-entry check): whole GPU suite on the default build, then pass e's A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04f
export PARITY_LOG=gpurun_out/r04f/parity.json
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r04f/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 gpurun_out/r04f/suite.log
[ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/r04f/suite.log | head; exit 1; }
bash tools/r04_e.sh
