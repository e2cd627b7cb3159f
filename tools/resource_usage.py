"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage output: python tools/resource_usage.py FILE"""
import re
import subprocess
import sys

rows, cur = {}, None
for line in open(sys.argv[1]):
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r':\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\w+) \[-Rpass', line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    name = subprocess.run(['c++filt', k], capture_output=True, text=True).stdout.strip()
    name = name.replace('kfmi::(anonymous namespace)::', '').replace('(kfmi::CvArgs)', '').replace('(kfmi::SynthArgs)', '')
    print(f"{name[:48]:48s} VGPR={v.get('VGPRs'):>4} SGPR={v.get('TotalSGPRs'):>3} "
          f"scratch={v.get('ScratchSize')} spill={v.get('VGPRs Spill')} waves/SIMD={v.get('Occupancy')}")
