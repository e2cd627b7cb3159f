"""Reduce tools/search_stalls.sh's passes: per search kernel, the SQ counters summed over its
dispatches, per 64 subsets where that is meaningful, and the shares of the wave cycles.

usage: python tools/search_stalls.py OUTDIR [KERNEL_REGEX]   -> prints and writes OUTDIR/search_stalls.json
(KERNEL_REGEX: group 1 the kernel's stem, group 2 its template arguments; default the search
kernels; tools/gated_stalls.sh passes the chain and look-ahead kernels')
"""
import collections
import csv
import glob
import json
import os
import re
import sys


KERNELS = r'(ref15_search_\w+?)_kernel<([^>]*)>'


def sums(d):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                m = re.search(KERNELS, r['Kernel_Name'])
                if m:
                    out[f'{m.group(1)}<{m.group(2)}>'][r['Counter_Name']] += float(r['Counter_Value'])
    return out


def main():
    global KERNELS
    d = sys.argv[1]
    if len(sys.argv) > 2:
        KERNELS = sys.argv[2]
    tot = collections.defaultdict(dict)
    for p in ('p1', 'p2', 'p3'):
        for k, cs in sums(os.path.join(d, p)).items():
            tot[k].update(cs)
    kt = {}
    for f in glob.glob(os.path.join(d, 'kt', '**', '*kernel_stats.csv'), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                m = re.search(KERNELS, r['Name'])
                if m:
                    kt[f'{m.group(1)}<{m.group(2)}>'] = float(r['TotalDurationNs']) * 1e-6
    rep = {}
    for k, c in sorted(tot.items()):
        wc = c.get('SQ_WAVE_CYCLES') or 1.0
        ms = kt.get(k)
        r = {'ms_total': ms, 'counters': c,
             'share_of_wave_cycles': {n: round(c.get(n, 0) / wc, 4) for n in
                                      ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_WAIT_INST_LDS', 'SQ_ACTIVE_INST_VALU',
                                       'SQ_ACTIVE_INST_SCA', 'SQ_ACTIVE_INST_LDS', 'SQ_ACTIVE_INST_MISC')},
             'per_valu': {n: round(c.get(n, 0) / max(c.get('SQ_INSTS_VALU', 1), 1), 4) for n in
                          ('SQ_INSTS_SALU', 'SQ_INSTS_SMEM', 'SQ_INSTS_LDS', 'SQ_INSTS_BRANCH', 'SQ_INSTS_VMEM_WR',
                           'SQ_INSTS_VALU_TRANS_F64', 'SQ_INSTS_VALU_FMA_F64', 'SQ_INSTS_VALU_MUL_F64',
                           'SQ_INSTS_VALU_ADD_F64', 'SQ_INSTS_VALU_INT32', 'SQ_LDS_BANK_CONFLICT')}}
        if ms:
            r['valu_issue_frac'] = round(c.get('SQ_INSTS_VALU', 0) * 4 / (ms * 1e-3 * 2.4e9 * 1024), 4)
        rep[k] = r
        print(k, json.dumps({x: r[x] for x in r if x != 'counters'}))
    with open(os.path.join(d, 'search_stalls.json'), 'w') as f:
        json.dump(rep, f, indent=1)


if __name__ == '__main__':
    main()
