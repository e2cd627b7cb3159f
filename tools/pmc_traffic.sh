#!/bin/bash
# HBM traffic of cv_run_kernel from rocprofv3 PMC counters (gpurun -- bash tools/pmc_traffic.sh TAG "CFG...").
# One counter per pass (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950), --pmc only
# (no sys/hip trace domains).  The bandwidth probe's soa_read / soa_write kernels (known byte
# counts, 8 B per lane like the fp64 engine) are profiled in the same way for calibration.
set -u
TAG=$1; CFGS=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/probe_$ctr" -o p -- "$ROOT/tools/probes/bw_probe" 1048576 64 > "$OUT/probe_$ctr.log" 2>&1 || { echo "probe $ctr failed"; tail "$OUT/probe_$ctr.log"; exit 1; }
  for c in $CFGS; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/cfg${c}_$ctr" -o k -- python3 "$ROOT/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/cfg${c}_$ctr.log" 2>&1 || { echo "cfg $c $ctr failed"; tail "$OUT/cfg${c}_$ctr.log"; exit 1; }
  done
done
cd "$ROOT"
python3 tools/pmc_traffic.py "$OUT" $CFGS
