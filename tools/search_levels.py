"""Per-level durations of the kf_search_combos kernels in a rocprofv3 kernel trace (the last
search call's n level launches).   python tools/search_levels.py <kt_kernel_trace.csv> [n]"""
import csv
import math
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = [r for r in csv.DictReader(open(path)) if 'ref15_search' in r['Kernel_Name']]
# levels without stored parents (k = n) are scored by the previous launch and not launched
nl = sum(1 for k in range(1, n + 1) if k == 1 or math.comb(n - 2, k - 1) > 0)
last = rows[-nl:]
tot = 0.0
for k, r in enumerate(last, 1):
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot += d
    kind = 'cm' if 'cm_kernel' in r['Kernel_Name'] else 'pm'
    print(f'{k:3d} {kind} {d:9.1f} us  subsets {math.comb(n, k):9d}  parents {math.comb(n - 2, k - 1) if k > 1 else 1:9d}')
span = (int(last[-1]['End_Timestamp']) - int(last[0]['Start_Timestamp'])) / 1e3
print(f'kernels {tot:.1f} us, span {span:.1f} us')
