#!/bin/bash
# GPU-box session for the SURVEY 8f rows and config 1: one bench line each (with CPU
# baseline) plus the same bench command under rocprofv3 kernel-stats, whose own JSON line is
# kept as bench_<c>_profiled.json: HBM placement differs per process, so the
# HIP-event kernel time and the rocprof average are compared within that one process.
#   gpurun -- bash tools/gpu_rows.sh TAG [config ...]        (default configs: 1 ref15 bf)
# Stops at the first step that ends in anything but success (timeouts, aborts, faults).
set -u
TAG=${1:-rows}; shift || true
CONFIGS=${*:-1 ref15 bf}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a "$OUT/steps.txt"
  if [ "$rc" != 0 ]; then echo "stopping after $name (rc=$rc)"; tail -20 "$OUT/$name.log"; exit "$rc"; fi
}
for c in $CONFIGS; do
  cd "$ROOT"
  step "bench_$c" 600 python bench.py --config "$c"
  tail -1 "$OUT/bench_$c.log" > "$OUT/bench_$c.json"
  cd /tmp
  step "rocprof_$c" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o kt -- \
       python3 "$ROOT/bench.py" --config "$c" --no-cpu-baseline
  grep '^{"metric"' "$OUT/rocprof_$c.log" | tail -1 > "$OUT/bench_${c}_profiled.json"
done
cd "$ROOT"
for c in $CONFIGS; do python3 -c "import json,sys; r=json.load(open('$OUT/bench_$c.json')); print('$c', r['value'], r['ms_per_step'], r['roofline'].get('frac'), (r.get('cpu_baseline') or {}).get('value'))"; done
