#!/bin/bash
# Run a list of GPU steps on the box, each under its own time limit, stopping at the first
# failure other than an ordinary test failure (rc 1).  Each step's output: gpurun_out/TAG/NAME.log
#   gpurun -- bash tools/gpu_steps.sh TAG "name|seconds|command" ...
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; lim=${rest%%|*}; cmd=${rest#*|}
  t0=$(date +%s)
  timeout -k 10 "$lim" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a "$OUT/steps.txt"
  case $rc in
    0|1) ;;
    *) echo "stopping after $name (rc=$rc)"; tail -20 "$OUT/$name.log"; exit "$rc" ;;
  esac
done
