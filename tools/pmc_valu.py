"""Reduce tools/pmc_valu.sh's SQ counters to VALU issue per launch of each config's dominant kernel.

usage: python tools/pmc_valu.py OUTDIR CFG [CFG ...]   -> writes OUTDIR/pmc_valu.json

valu_issue_frac = SQ_INSTS_VALU x 4 cycles / (kernel time x 2.4 GHz x 1024 SIMDs): the share of
the chip's VALU issue slots the kernel's wave instructions fill (a wave64 VALU instruction
occupies its 16-lane SIMD 4 cycles; fp64 FMA is full rate on gfx950, 78.6 TFLOP/s; transcendental
and f64 rcp instructions take longer, so this is a floor on the VALU busy share).  The kernel
time is the HIP-event time of the same profiled process (its bench JSON line).
"""
import json
import os
import sys

from pmc_traffic import per_kernel, pick

CLK, SIMDS, CYC = 2.4e9, 1024, 4
COUNTERS = ['SQ_WAVES', 'SQ_INSTS_VALU', 'SQ_ACTIVE_INST_VALU', 'SQ_WAVE_CYCLES', 'SQ_BUSY_CYCLES', 'SQ_WAIT_ANY',
            'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'GRBM_GUI_ACTIVE']


def bench_line(path):
    with open(path) as f:
        for line in f:
            if line.startswith('{"metric"'):
                rec = json.loads(line)
    return rec


def kernel_trace_ms(out_dir, c, kern):
    """Average duration (ms) of the kernel matching `kern` in pmc_valu.sh's kernel-trace pass."""
    import csv
    import glob
    for f in glob.glob(os.path.join(out_dir, f'kt{c}', '**', '*kernel_stats.csv'), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kern in r['Name']:
                    return float(r['AverageNs']) * 1e-6
    raise SystemExit(f'no kernel-trace row for {kern!r} under {out_dir}/kt{c}')


def search_valu(out_dir, rec, c):
    """bf / bf40: one search = its launches (every ref15_search_* dispatch: one kf_search_combos
    call, or one per class), counters and kernel-trace durations summed per search; a unit is one
    subset."""
    import csv
    import glob
    d = os.path.join(out_dir, f'cfg{c}')
    classes = rec['config'].get('classes', 1)
    searches = len(pick(per_kernel(d, 'SQ_WAVES'), 'ref15_search_head')) / classes
    vals = {ctr: sum(v for k, vs in per_kernel(d, ctr).items() if 'ref15_search' in k for v in vs) / searches
            for ctr in COUNTERS}
    tot, heads = 0.0, 0
    for f in glob.glob(os.path.join(out_dir, f'kt{c}', '**', '*kernel_stats.csv'), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if 'ref15_search' in r['Name']:
                    tot += float(r['TotalDurationNs'])
                    heads += int(r['Calls']) if 'search_head' in r['Name'] else 0
    ms = tot * 1e-6 / (heads / classes)
    wave_units = rec['config']['combinations'] / 64
    return dict(kernel='ref15_search_head/cm/pm/end_kernel (one search)', counters_per_launch=vals, kernel_ms=ms,
                launches_profiled=searches, classes=classes, valu_per_wave_step=vals['SQ_INSTS_VALU'] / wave_units,
                valu_issue_frac=vals['SQ_INSTS_VALU'] * CYC / (ms * 1e-3 * CLK * SIMDS),
                wave_cycles_waiting_frac=vals['SQ_WAIT_ANY'] / vals['SQ_WAVE_CYCLES'],
                wave_cycles_issue_stall_frac=vals['SQ_WAIT_INST_ANY'] / vals['SQ_WAVE_CYCLES'],
                unit='one subset (valu_per_wave_step: per 64 subsets)')


def main():
    out_dir, cfgs = sys.argv[1], sys.argv[2:]
    res = {'note': ' '.join(__doc__.split('\n\n')[2].split())}
    for c in cfgs:
        d = os.path.join(out_dir, f'cfg{c}')
        rec = bench_line(os.path.join(out_dir, f'cfg{c}.log'))
        if c in ('bf', 'bf40'):
            res[f'config{c}'] = search_valu(out_dir, rec, c)
            continue
        units = rec['value'] * rec['ms_per_step'] * 1e-3        # filter-steps (events) per launch
        wave_steps = units / 64
        if c == 'sched' and 'apply' in rec['roofline']['kernel']:
            # the two passes, each timed by its own GRBM_GUI_ACTIVE (GPU busy cycles in the dispatch)
            kerns = {'apply': 'ref15_apply_kernel', 'pick': 'ref15_pick_kernel'}
        else:
            kerns = {'': {'ref15': 'ref_events', 'sched': 'ref15_sched', '1': 'ref_chain_kernel',
                          '3gen': 'cv_run_kernel'}.get(c, 'cv_block_kernel')}
        for tag, kern in kerns.items():
            vals = {}
            for ctr in COUNTERS:
                v = pick(per_kernel(d, ctr), kern)
                vals[ctr] = sum(v) / len(v)
            ms = rec['roofline']['kernel_ms'] if len(kerns) == 1 else kernel_trace_ms(out_dir, c, kern)
            res[f'config{c}' + (f'_{tag}' if tag else '')] = dict(
                kernel=kern, counters_per_launch=vals, kernel_ms=ms, launches_profiled=len(v),
                valu_per_wave_step=vals['SQ_INSTS_VALU'] / wave_steps,
                valu_issue_frac=vals['SQ_INSTS_VALU'] * CYC / (ms * 1e-3 * CLK * SIMDS),
                wave_cycles_waiting_frac=vals['SQ_WAIT_ANY'] / vals['SQ_WAVE_CYCLES'],
                wave_cycles_issue_stall_frac=vals['SQ_WAIT_INST_ANY'] / vals['SQ_WAVE_CYCLES'])
    with open(os.path.join(out_dir, 'pmc_valu.json'), 'w') as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
