#!/bin/bash
# Ablation sweep: gpurun -- bash tools/gpu_ablate.sh TAG "CFG..."
set -u
TAG=$1; CFGS=$2; ROUNDS=${ROUNDS:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for r in $(seq 1 "$ROUNDS"); do for c in $CFGS; do for ab in none no-logdet no-traj no-traj-no-logdet; do
  timeout -k 10 300 python bench.py --config "$c" --steps 10 --warmup 2 --no-cpu-baseline --ablate $ab > "$OUT/tmp.json" 2> "$OUT/err.log"
  rc=$?; if [ $rc -ne 0 ]; then echo "cfg=$c ab=$ab rc=$rc"; tail -5 "$OUT/err.log"; exit $rc; fi
  python3 -c "import json; d=json.load(open('$OUT/tmp.json')); print('round=$r cfg=$c ablate=$ab', f\"kern_ms={d['roofline']['kernel_ms']:.3f}\")" | tee -a "$OUT/ablate.txt"
done; done; done
