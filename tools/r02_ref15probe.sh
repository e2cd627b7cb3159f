set -u
OUT=gpurun_out/r02_ref15probe; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --config ref15 --no-cpu-baseline > $OUT/bench_ref15.log 2>&1 || { echo fail; tail -5 $OUT/bench_ref15.log; exit 1; }
grep '^{"metric"' $OUT/bench_ref15.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], json.dumps(d['roofline']))"
