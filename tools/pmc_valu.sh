#!/bin/bash
# VALU issue of the bench kernels from rocprofv3 SQ counters ("also report the
# VALU fraction").  One --pmc pass per config (8 SQ + 1 GRBM counter, within gfx950's slots),
# --pmc only (no trace domains).   gpurun -- bash tools/pmc_valu.sh TAG "3 4 2 5 ref15"
set -u
TAG=$1; CFGS=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
cd /tmp
for c in $CFGS; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/cfg$c" -o k -- python3 "$ROOT/bench.py" --config $c ${PMC_STEPS:---steps 3 --warmup 1} --no-cpu-baseline > "$OUT/cfg$c.log" 2>&1 || { echo "cfg $c failed"; tail "$OUT/cfg$c.log"; exit 1; }
  # per-kernel durations of the same command (configs with more than one kernel per step)
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt$c" -o k -- python3 "$ROOT/bench.py" --config $c ${PMC_STEPS:---steps 3 --warmup 1} --no-cpu-baseline > "$OUT/kt$c.log" 2>&1 || { echo "kt $c failed"; tail "$OUT/kt$c.log"; exit 1; }
  echo "cfg $c ok"
done
cd "$ROOT"
python3 tools/pmc_valu.py "$OUT" $CFGS
