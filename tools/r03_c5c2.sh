# C5 and C2 bench lines (no CPU baseline) after an attention change; TAG names the logs
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03j}
timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-gather > gpurun_out/${TAG}_bench_c5.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c5.log; exit 1; }
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('c5',d['value'],d['ms_per_step'])" gpurun_out/${TAG}_bench_c5.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/${TAG}_bench_c2.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c2.log; exit 1; }
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('c2',d['value'],d['ms_per_step'])" gpurun_out/${TAG}_bench_c2.log
