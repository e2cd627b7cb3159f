set -u
OUT=gpurun_out/r02_ref15_ab; mkdir -p $OUT
export TMPDIR=/tmp
KFMI_REF_IMAGES=3 timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_ref15.py tests/test_gpu_refmodels.py -k "not search and not brute and not combo" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_inproc.py --config ref15 --arms "$1" --rounds 6 --launches 5 > $OUT/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; tail -3 $OUT/ab.log
