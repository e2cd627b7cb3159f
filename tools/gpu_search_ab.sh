#!/bin/bash
# kf_search_combos A/B on the GPU box: search parity tests, then the bf bench per kernel choice
# (KFMI_SEARCH_KERNEL), interleaved, then kernel trace + stats of the default.
#   gpurun -- bash tools/gpu_search_ab.sh TAG
set -u
TAG=${1:-srch}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ref15.py -x -v --timeout 120 --timeout-method thread -k "search or brute" -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -n 5 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for v in auto cm pm; do
    kk=$v
    KFMI_SEARCH_KERNEL=$kk timeout -k 10 200 python bench.py --config bf --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bf_$v.$r.log 2>&1 || exit 3
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/bf_$v.$r.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --config bf --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || exit 4
