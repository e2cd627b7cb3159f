set -u
OUT=gpurun_out/r02_sched_ab; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_ref15.py tests/test_gpu_compat.py -k "sched or sampling or score" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_inproc.py --config sched --arms "$1" --rounds 4 --launches 3 > $OUT/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; tail -3 $OUT/ab.log
