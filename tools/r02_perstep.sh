set -u
OUT=${OUT:-gpurun_out/r02_perstep}; mkdir -p $OUT
for c in 3 2 4; do
timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --per-step --steps 10 --warmup 3 > $OUT/bench_$c.log 2>&1 || { echo fail $c; tail -5 $OUT/bench_$c.log; exit 1; }
grep '^{"metric"' $OUT/bench_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['ms_per_step'], d['value'], json.dumps(d.get('per_step_api')))"
done
