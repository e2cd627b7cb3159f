#!/bin/bash
# HBM traffic of each config's dominant kernel from rocprofv3 PMC counters
# (gpurun -- bash tools/pmc_traffic.sh TAG "CFG..." ["SETS"]).
# One counter set per pass (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950), --pmc only
# (no sys/hip trace domains).  SETS (default "FETCH_SIZE WRITE_SIZE RDSIZED"): RDSIZED is the L2's
# memory-side read requests by size (32 / 64 / 128 B, and their total: the 4 TCC slots), which
# counts gathered reads exactly where FETCH_SIZE's 64-B tally needs a per-pattern calibration.
# The bandwidth probe's soa_read / soa_write kernels (known byte counts, 8 B per lane like the
# fp64 engine) are profiled in the same way for calibration.  PMC_BENCH_ARGS: extra bench.py
# arguments for every config run (diagnostics, e.g. "--sched-rates 10,20").
set -u
TAG=$1; CFGS=$2; SETS=${3:-"FETCH_SIZE WRITE_SIZE RDSIZED"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for set in $SETS; do
  if [ "$set" = RDSIZED ]; then
    ctrs="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
  else
    ctrs=$set
  fi
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/probe_$set" -o p -- "$ROOT/tools/probes/bw_probe" 1048576 64 > "$OUT/probe_$set.log" 2>&1 || { echo "probe $set failed"; tail "$OUT/probe_$set.log"; exit 1; }
  for c in $CFGS; do
    timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/cfg${c}_$set" -o k -- python3 "$ROOT/bench.py" --config $c ${PMC_STEPS:---steps 3 --warmup 1} --no-cpu-baseline ${PMC_BENCH_ARGS:-} > "$OUT/cfg${c}_$set.log" 2>&1 || { echo "cfg $c $set failed"; tail "$OUT/cfg${c}_$set.log"; exit 1; }
  done
done
cd "$ROOT"
python3 tools/pmc_traffic.py "$OUT" $CFGS
