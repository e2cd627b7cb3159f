#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/mix1; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p1" -o k -- python3 "$ROOT/bench.py" --config 1 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/p1.log" 2>&1 || { tail "$OUT/p1.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_MFMA --output-format csv -d "$OUT/p2" -o k -- python3 "$ROOT/bench.py" --config 1 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/p2.log" 2>&1 || { tail "$OUT/p2.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o k -- python3 "$ROOT/bench.py" --config 1 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/kt.log" 2>&1 || { tail "$OUT/kt.log"; exit 1; }
echo done
