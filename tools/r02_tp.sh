set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_timeparallel.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_tp_pytest.log 2>&1 || exit 1
for c in 4096 8192 16384; do
  KFMI_STREAM_CHUNKS=$c timeout -k 10 120 python bench.py --config 1 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r02_tp_c$c.json 2>/dev/null || exit 1
done
for c in 8192 16384; do
  KFMI_STREAM_CHUNKS=$c timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp_$c -o run --output-format csv -- python3 bench.py --config 1 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/prof_tp_$c.json 2>/dev/null || exit 1
done
