# Round-4 GPU pass n: C2 and C5 benches on the compact loss passes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04n
summ() {
python3 - "$1" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], json.dumps(d["roofline"])[:200])
        for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["share"])[:16]:
            print("   ", k, v["avg_ms"], v["calls_per_step"], round(v["avg_ms"] * v["calls_per_step"], 3), v.get("TFLOP/s"))
PY
}
for c in c2 c5; do
  n=gpurun_out/r04n/bench_$c.log
  timeout -k 10 400 python -u bench.py --config $c --steps 8 --warmup 3 --no-cpu-baseline --no-hbm-gather > $n 2>&1 || { tail -20 $n; exit 1; }
  summ $n
done
