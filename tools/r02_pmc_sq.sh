set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_WAIT_INST_ANY SQ_INSTS_VALU_TRANS_F64"
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_sq_ref15 -o run --output-format csv -- python3 bench.py --config ref15 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_sq_ref15.json 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_sq_c1 -o run --output-format csv -- python3 bench.py --config 1 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_sq_c1.json 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_timeparallel.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_tp_pytest.log 2>&1 || exit 1
