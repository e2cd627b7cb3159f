set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_c1_pmc_chunks; mkdir -p $OUT
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"
for c in 8192 16384; do
  KFMI_STREAM_CHUNKS=$c timeout -s KILL 120 rocprofv3 --pmc $C1 -d $OUT/p$c -o run --output-format csv -- python3 bench.py --config 1 --no-cpu-baseline --steps 3 --warmup 1 > $OUT/p$c.log 2>&1 || { echo "pass $c failed"; tail -5 $OUT/p$c.log; exit 1; }
done
echo done
