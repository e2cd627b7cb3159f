set -u
OUT=gpurun_out/r02_bf; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_ref15.py -k "search or brute" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_inproc.py --config bf --arms build/ab/base.so,default --rounds 6 --launches 5 > $OUT/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; tail -12 $OUT/ab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config bf > $OUT/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-400
