# KShift dense/sparse backward: touched-row flag atomics issued side by side; tests + C2 bench
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kshift.py tests/test_gpu_tables.py tests/test_gpu_optim.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/tests.log | head -40; exit $rc; }
timeout -k 10 400 python bench.py --no-cpu-baseline --no-hbm-gather --no-generator > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
python3 -c "
import json;s=open('$O/bench_c2.log').read();i=s.rfind('{\"metric\"');d=json.loads(s[i:].split(chr(10))[0])
print('value',d['value'],'ms',d['ms_per_step']);k=d['kernels'];print({x:k[x] for x in k if 'kshift' in x or 'sparse' in x})"
