# CVE / product-tower kernels: their GPU tests, then the C2 bench's per-kernel timing
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tables.py tests/test_gpu_lthm.py tests/test_gpu_vecemb.py > gpurun_out/cve_tests.log 2>&1 || { tail -30 gpurun_out/cve_tests.log; exit 1; }
tail -2 gpurun_out/cve_tests.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-gather > gpurun_out/cve_bench.log 2>&1 || { tail -30 gpurun_out/cve_bench.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/cve_bench.log").read().splitlines():
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print("value", d["value"], "ms", d["ms_per_step"])
        for k in ("cve_tab_bwd_k", "lthm_product_tower_fwd", "table_bwd_mfma_k", "cl_bwd_k", "attn_bwd_k"):
            print(k, d["kernels"].get(k))
PY
