"""Print the kernel timeline of the last bench step from a rocprofv3 kernel_trace.csv: one line
per kernel (start offset, duration in us), from the step's first kernel (dt_kernel) on.
Diagnostic tool.   python tools/step_timeline.py <run_kernel_trace.csv> [first_kernel_substring]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else 'dt_kernel'
rows.sort(key=lambda r: int(r['Start_Timestamp']))
starts = [i for i, r in enumerate(rows) if first in r['Kernel_Name']]
i0 = starts[-1]
t0 = int(rows[i0]['Start_Timestamp'])
for r in rows[i0:]:
    name = re.sub(r'kfmi::\(anonymous namespace\)::', '', r['Kernel_Name'])
    name = re.sub(r'\(.*$', '', name)[:90]
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f'{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name}')
