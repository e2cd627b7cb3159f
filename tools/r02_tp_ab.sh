set -u
OUT=gpurun_out/r02_tp_ab; mkdir -p $OUT
export TMPDIR=/tmp
if [ "${2:-}" = "test" ]; then
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_timeparallel.py > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u tools/ab_inproc.py --config 1 --arms "$1" --rounds 8 --launches 10 > $OUT/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; tail -3 $OUT/ab.log
