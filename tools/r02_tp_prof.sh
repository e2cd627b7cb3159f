set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in 4096 8192; do
  KFMI_STREAM_CHUNKS=$c timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp_$c -o run --output-format csv -- python3 bench.py --config 1 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/prof_tp_$c.json 2>/dev/null || exit 1
done
