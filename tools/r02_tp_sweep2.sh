set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_tp2
for c in ${*:-12288 16384}; do
  KFMI_STREAM_CHUNKS=$c timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/r02_tp2/prof_$c -o run --output-format csv -- python3 bench.py --config 1 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r02_tp2/bench_$c.log 2>&1 || exit 1
  f=$(find gpurun_out/r02_tp2/prof_$c -name "run_kernel_trace.csv" | head -1)
  echo "== $c"; python tools/step_timeline.py $f | head -10
done
