set -u
O=gpurun_out/r03_sched; mkdir -p $O
for arm in "auto:" "fused:--opt sched_kernel=fused" "auto_rb1:--rate-block 1" "fused_rb1:--rate-block 1 --opt sched_kernel=fused"; do
  n=${arm%%:*}; a=${arm#*:}
  timeout -k 10 200 python bench.py --config sched --steps 20 --warmup 5 $a > $O/bench_$n.json 2> $O/bench_$n.err || exit 1
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$n.json)"
done
R=$GRAFT_REPO_ROOT; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/bench.py --config sched --steps 10 --warmup 3 --no-cpu-baseline > $R/$O/bench_profiled.json 2> $R/$O/kt.log || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pmc_cache -o k -- python3 $R/bench.py --config sched --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/pmc_cache.log 2>&1 || exit 1
cd $R
timeout -k 10 600 bash tools/pmc_valu.sh r03_sched_valu sched > $O/pmc_valu.txt 2>&1 || { tail $O/pmc_valu.txt; exit 1; }
echo ok
