set -u
OUT=gpurun_out/r02_bf_prof; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 bench.py --config bf --no-cpu-baseline --steps 2 --warmup 1 > $OUT/kt.log 2>&1 || exit 1
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_WAIT_INST_ANY SQ_INSTS_VALU_TRANS_F64"
timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc -o run --output-format csv -- python3 bench.py --config bf --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pmc.log 2>&1 || exit 1
C2="SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU_MUL_F64"
timeout -s KILL 120 rocprofv3 --pmc $C2 -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py --config bf --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pmc2.log 2>&1 || exit 1
