#!/bin/bash
# Config 3 in N fresh processes (default 8): the per-process HBM placement spread of the headline
# (DESIGN.md §4).   gpurun -- bash tools/placement_series.sh TAG [N]
set -u
TAG=${1:-placement}; N=${2:-8}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd "$ROOT"
# the box's clocks and partition modes beside the series (read-only queries)
(rocm-smi --showclocks; rocm-smi --showcomputepartition --showmemorypartition) > "$OUT/smi.txt" 2>&1 || true
for i in $(seq 1 "$N"); do
  timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/run_$i.log" 2>&1 || { echo "run $i failed"; tail -5 "$OUT/run_$i.log"; exit 1; }
  grep '^{"metric"' "$OUT/run_$i.log" | tail -1 >> "$OUT/lines.jsonl"
  python3 -c "import json; r=json.loads(open('$OUT/lines.jsonl').read().splitlines()[-1]); print($i, round(r['ms_per_step'],3), round(r['roofline']['frac'],3), round(r['roofline']['pattern_ceiling']['frac'],3), round(r['roofline']['pattern_ceiling']['achieved']))" | tee -a "$OUT/summary.txt"
done
