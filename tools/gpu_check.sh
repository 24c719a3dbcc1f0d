#!/bin/bash
# One GPU-box pass: parity tests, smoke, the C2 bench line and a rocprofv3 kernel-stats
# summary of the same bench command.  Usage (from the repo root, on the GPU box):
#   bash tools/gpu_check.sh TAG [tests|bench|prof ...]   (default: all three)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}; shift || true
STAGES=${*:-tests bench prof}
mkdir -p gpurun_out
for s in $STAGES; do
  case $s in
    tests)
      # exit status 1 = assertion failures only: go on; anything else (fault, abort, time limit): stop
      rc=0
      PARITY_LOG=gpurun_out/${TAG}_parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -v \
        --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || rc=$?
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
      [ $rc -eq 1 ] && echo "TESTS FAILED (assertions)"
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 ;;
    bench)
      timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 ;;
    bench3)
      timeout -k 10 400 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/${TAG}_bench_c3.log 2>&1 ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv \
        -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 ;;
    pmc)
      bash tools/pmc_passes.sh ;;
  esac
done
echo "gpu_check $TAG done: $STAGES"
