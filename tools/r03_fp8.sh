# fp8 path after the fused-amax change: fp8 / encoder GPU tests, the C5 LTHM step test, then the C5 bench
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03k}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_encoder.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lthm.py -k c5 > gpurun_out/${TAG}_c5test.log 2>&1 || { tail -40 gpurun_out/${TAG}_c5test.log; exit 1; }
tail -1 gpurun_out/${TAG}_c5test.log
timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-gather > gpurun_out/${TAG}_bench_c5.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c5.log; exit 1; }
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('c5',d['value'],d['ms_per_step']);k=d.get('kernels',{});[print(n,v) for n,v in k.items() if 'quant' in n or 'amax' in n]" gpurun_out/${TAG}_bench_c5.log
