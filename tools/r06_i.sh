# fused dedup + Adagrad: diagnostics, parity tests, generator step A/B, kernel summary
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 300 python tools/kag_diag.py > $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
grep -v amdgpu.ids $O/diag.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kshift_adagrad.py tests/test_gpu_embgen.py tests/test_gpu_optim.py tests/test_gpu_kshift.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/tests.log | head -40; exit $rc; }
timeout -k 10 300 python tools/embgen_bench.py > $O/embgen_bench.log 2>&1 || { tail -20 $O/embgen_bench.log; exit 1; }
grep model $O/embgen_bench.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/embgen_bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find $O/prof -name "*.db" | head -1) 40 > $O/kernel_stats.txt 2>&1
head -40 $O/kernel_stats.txt
rm -rf $O/prof
