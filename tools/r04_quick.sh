# Round-4 quick GPU pass: the given test files, then a short C2 bench (no CPU baseline).
# Usage: TAG=x bash tools/r04_quick.sh tests/test_a.py tests/test_b.py
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r04q}
mkdir -p gpurun_out
export PARITY_LOG=gpurun_out/${TAG}_parity.json
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.log | head -30; exit $rc; }
if [ -z "$NOBENCH" ]; then
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -c 600 gpurun_out/${TAG}_bench.log; echo
fi
