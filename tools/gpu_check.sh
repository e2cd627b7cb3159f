#!/bin/bash
# GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
#   gpurun -- bash tools/gpu_check.sh TAG [bench args...]
# Stops at the first step that ends in anything but success or an ordinary test failure
# (timeouts, aborts, segfaults, signals), so a fault never leads to further GPU work.
set -u
TAG=${1:-run}; shift || true
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
  case $rc in
    0|1) return 0 ;;
    *) echo "stopping after $name (rc=$rc)"; tail -20 "$OUT/$name.log"; exit "$rc" ;;
  esac
}
cd "$ROOT"
rocm-smi --showproductname > "$OUT/device.txt" 2>&1 || true
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py "$@"
cd /tmp
# the bench command itself under rocprof: its JSON line (bench_profiled.json) and the kernel
# stats come from one process, so they see the same HBM placement
step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o kt -- python3 "$ROOT/bench.py" --no-cpu-baseline "$@"
cd "$ROOT"
grep '^{"metric"' "$OUT/rocprof_stats.log" | tail -1 > "$OUT/bench_profiled.json" || true
tail -3 "$OUT/pytest_gpu.log"; cat "$OUT/bench.log" | tail -2
