set -u
OUT=gpurun_out/r02_perstep2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_compat.py > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
OUT=$OUT bash tools/r02_perstep.sh
