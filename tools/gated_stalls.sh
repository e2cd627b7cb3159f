#!/bin/bash
# Where the one-filter gated kernels' issue slots go (diagnostic, DESIGN.md §3
# ref_chain_gated_kernel): the SQ counter passes of tools/search_stalls.sh over
# tools/gated_kernel_ab.py at one threshold (both kernels, one round), reduced per kernel.
#   gpurun -- bash tools/gated_stalls.sh TAG [THRESHOLD]
set -u
TAG=$1; THR=${2:--36.4}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F64"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
P3="SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_BUSY_CYCLES SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"
cd /tmp
i=0
for C in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o k -- python3 "$ROOT/tools/gated_kernel_ab.py" --thr=$THR --rounds 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o k -- python3 "$ROOT/tools/gated_kernel_ab.py" --thr=$THR --rounds 1 > "$OUT/kt.log" 2>&1 || { echo "kt failed"; exit 1; }
cd "$ROOT"
python3 tools/search_stalls.py "$OUT" '(ref_chain(?:_gated)?)_kernel<([^>]*)>'
