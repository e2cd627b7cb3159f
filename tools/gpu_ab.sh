#!/bin/bash
# A/B bench sweep on the GPU box:  gpurun -- bash tools/gpu_ab.sh TAG "LIB1 LIB2 ..." "CFG1 CFG2 ..."
# Runs bench.py for each (library, config) pair, interleaved over ROUNDS rounds, one line each.
# A LIB entry of the form NAME=VALUE is a handle option of the default library instead
# (bench.py --opt, e.g. "cv_kernel=general cv_kernel=auto").
set -u
TAG=$1; LIBS=$2; CFGS=$3; ROUNDS=${ROUNDS:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd "$ROOT"
for r in $(seq 1 "$ROUNDS"); do
  for lib in $LIBS; do
    for c in $CFGS; do
      if [[ "$lib" == *=* ]]; then
        timeout -k 10 300 python bench.py --opt "$lib" --config "$c" --steps 20 --warmup 10 --no-cpu-baseline > "$OUT/tmp.json" 2> "$OUT/err_${c}.log"
      else
        KFMI_LIB=$lib timeout -k 10 300 python bench.py --config "$c" --steps 20 --warmup 10 --no-cpu-baseline > "$OUT/tmp.json" 2> "$OUT/err_${c}.log"
      fi
      rc=$?
      if [ $rc -ne 0 ]; then echo "lib=$lib cfg=$c rc=$rc"; tail -5 "$OUT/err_${c}.log"; exit $rc; fi
      python3 -c "import json,sys; d=json.load(open('$OUT/tmp.json')); print('round=$r lib=$lib cfg=$c', f\"value={d['value']:.4e} kern_ms={d['roofline']['kernel_ms']:.3f} GB/s={d['roofline']['achieved']:.0f} frac={d['roofline']['frac']:.3f} bad={d['failed_filters']}\")" | tee -a "$OUT/ab.txt"
    done
  done
done
