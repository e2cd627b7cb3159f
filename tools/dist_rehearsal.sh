#!/bin/bash
# One-GPU rehearsal of bench.py's N>1 path (shards, max-over-ranks timing, the final all-gather
# and its reassembly check): N ranks share the box's one GPU over gloo, since RCCL refuses two
# ranks on one device.  The numbers are NOT scaling results (the ranks split one GPU's HBM).
#   gpurun -- bash tools/dist_rehearsal.sh TAG
set -u
TAG=${1:-dist}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
for cfg in 3 ref15 sched bf 1; do
  for n in 2 4; do
    [ "$n" = 4 ] && [ "$cfg" != 3 ] && [ "$cfg" != ref15 ] && continue  # the §8f rows and config 1 at N = 2
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 3 --warmup 1 \
      --config $cfg $([ "$cfg" = bf ] || [ "$cfg" = 1 ] || echo --batch 262144) --dist-backend gloo \
      --no-cpu-baseline > "$OUT/c${cfg}_n$n.log" 2>&1
    rc=$?
    echo "config $cfg n=$n rc=$rc" | tee -a "$OUT/steps.txt"
    grep '^{"metric"' "$OUT/c${cfg}_n$n.log" | tail -1 >> "$OUT/lines.jsonl" || true
    [ $rc -eq 0 ] || { tail -30 "$OUT/c${cfg}_n$n.log"; exit $rc; }
  done
done
# the self-launching form (the BENCH command's own: no launcher; bench.py starts its ranks as
# a child torch.distributed.run and relays rank 0's line)
timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --config 3 --batch 262144 \
  --dist-backend gloo --gather-traj-every 8 > "$OUT/self_launch_n2.log" 2>&1
rc=$?
echo "self-launch config 3 n=2 rc=$rc" | tee -a "$OUT/steps.txt"
grep '^{"metric"' "$OUT/self_launch_n2.log" | tail -1 >> "$OUT/lines.jsonl" || true
[ $rc -eq 0 ] || { tail -30 "$OUT/self_launch_n2.log"; exit $rc; }
