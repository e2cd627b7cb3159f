#!/bin/bash
# Occupancy sweep: gpurun -- bash tools/gpu_occ.sh TAG "CFG..." "K..."   (K = workgroups per CU cap, 0 = none)
set -u
TAG=$1; CFGS=$2; KS=$3; ROUNDS=${ROUNDS:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for r in $(seq 1 "$ROUNDS"); do for c in $CFGS; do for k in $KS; do
  KFMI_BLOCKS_PER_CU=$k timeout -k 10 300 python bench.py --config "$c" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/tmp.json" 2> "$OUT/err.log"
  rc=$?; if [ $rc -ne 0 ]; then echo "cfg=$c k=$k rc=$rc"; tail -5 "$OUT/err.log"; exit $rc; fi
  python3 -c "import json; d=json.load(open('$OUT/tmp.json')); print('round=$r cfg=$c blocks_per_cu=$k', f\"value={d['value']:.4e} kern_ms={d['roofline']['kernel_ms']:.3f} GB/s={d['roofline']['achieved']:.0f} frac={d['roofline']['frac']:.3f}\")" | tee -a "$OUT/occ.txt"
done; done; done
