#!/bin/bash
# GPU-box session for the time-parallel single-filter path (kf_run_stream): its tests (plus the
# other chain-kernel users), the config 1 bench line, a warm-up / chunk sweep, and rocprofv3
# kernel stats of the bench command.   gpurun -- bash tools/gpu_tp.sh TAG
set -u
TAG=${1:-tp}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_timeparallel.py tests/test_gpu_refmodels.py tests/test_gpu_ingest.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python bench.py --config 1 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/b1.log 2>&1 || { tail -20 $OUT/b1.log; exit 1; }
tail -1 $OUT/b1.log | cut -c1-300
timeout -k 10 300 python tools/stream_sweep.py ${SWEEP_ARGS:-} > $OUT/sweep.log 2>&1 || { tail -20 $OUT/sweep.log; exit 1; }
grep '^{' $OUT/sweep.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o kt -- python3 $ROOT/bench.py --config 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
echo done
