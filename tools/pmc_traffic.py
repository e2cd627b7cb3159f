"""Reduce rocprofv3 PMC CSVs (tools/pmc_traffic.sh) to HBM bytes per launch of each config's
dominant kernel (cv_block_kernel for the BASELINE configs, ref_events_kernel for ref15).

usage: python tools/pmc_traffic.py OUTDIR CFG [CFG ...]   -> writes OUTDIR/pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE is only
calibrated for 16 B/lane streams (reads half the bytes there); other widths must be calibrated
on a known byte count in the same access pattern.  The probe's soa_read (T*6*B*8 bytes read,
8 B per lane) and soa_write (T*7*B*8 bytes written) provide that calibration here.  Where the
RDSIZED pass ran (TCC_EA0_RDREQ_{32B,64B,128B}_sum: the L2's memory-side read requests by size),
the fetched bytes are counted exactly as 32 n32 + 64 n64 + 128 n128 instead, whatever the access
pattern (the calibration holds for streams of whole lines, not for per-lane gathers), and the
FETCH_SIZE figure is kept beside it.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sensorfusion-kalmanfilter_amd"))


def per_kernel(d, counter):
    """kernel name substring -> list of per-dispatch counter values (KiB)."""
    rows = {}
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get('Counter_Name') != counter:
                    continue
                key = (r['Kernel_Name'], r.get('Dispatch_Id') or r.get('Correlation_Id'))
                rows[key] = rows.get(key, 0.0) + float(r['Counter_Value'])
    out = {}
    for (name, _), v in rows.items():
        out.setdefault(name, []).append(v)
    return out


SIZED = ('TCC_EA0_RDREQ_32B_sum', 'TCC_EA0_RDREQ_64B_sum', 'TCC_EA0_RDREQ_128B_sum', 'TCC_EA0_RDREQ_sum')


def sized_fetch(out_dir, tag, match):
    """(bytes per dispatch, requests of no size bucket per dispatch) of the kernels whose name
    satisfies match, from the RDSIZED pass (None if it did not run); a list per dispatch."""
    d = os.path.join(out_dir, f'{tag}_RDSIZED')
    if not os.path.isdir(d):
        return None
    cols = {c: [v for k, vs in per_kernel(d, c).items() if match(k) for v in vs] for c in SIZED}
    n = len(cols[SIZED[0]])
    if not n or any(len(v) != n for v in cols.values()):
        raise SystemExit(f'RDSIZED pass of {tag}: uneven dispatch counts {[len(v) for v in cols.values()]}')
    by = [32 * a + 64 * b + 128 * c for a, b, c in zip(*(cols[x] for x in SIZED[:3]))]
    other = [t - a - b - c for a, b, c, t in zip(*(cols[x] for x in SIZED))]
    return by, other


def fetch(out_dir, tag, match, fetch_kib, read_scale):
    """Fetched bytes per dispatch (mean) and how they were counted: the sized requests where that
    pass ran, else FETCH_SIZE (KiB) times the probe's calibration."""
    sz = sized_fetch(out_dir, tag, match)
    cal = 1024 * sum(fetch_kib) / len(fetch_kib) * read_scale
    if sz is None:
        return cal, {'fetch_source': 'FETCH_SIZE x calibration'}
    by, other = sz
    return sum(by) / len(by), {'fetch_source': 'TCC_EA0_RDREQ by size (32/64/128 B)',
                               'fetch_bytes_calibrated': cal,
                               'requests_of_no_size_bucket': sum(other) / len(other)}


def pick(d, sub):
    vals = [v for k, v in d.items() if sub in k]
    if not vals:
        raise SystemExit(f'no kernel matching {sub!r} in {list(d)[:5]}')
    return vals[0]


def main():
    out_dir, cfgs = sys.argv[1], sys.argv[2:]
    from bench import CONFIGS, algorithmic_bytes, ref15_algorithmic_bytes
    B, T = 1048576, 64
    known_read, known_write = T * 6 * B * 8, T * 7 * B * 8
    pf = per_kernel(os.path.join(out_dir, 'probe_FETCH_SIZE'), 'FETCH_SIZE')
    pw = per_kernel(os.path.join(out_dir, 'probe_WRITE_SIZE'), 'WRITE_SIZE')
    rd = pick(pf, 'soa_read')
    wr = pick(pw, 'soa_write')
    read_scale = known_read / (1024 * sum(rd) / len(rd))
    write_scale = known_write / (1024 * sum(wr) / len(wr))
    res = {'calibration': {'fetch_size_scale': read_scale, 'write_size_scale': write_scale,
                           'probe': 'tools/probes/bw_probe soa_read/soa_write, 8 B per lane, B=2^20, T=64'}}
    sz = sized_fetch(out_dir, 'probe', lambda k: 'soa_read' in k)
    if sz is not None:  # the sized count against the probe's known bytes
        res['calibration']['sized_over_known_read'] = sum(sz[0]) / len(sz[0]) / known_read
    for c in cfgs:
        if c in ('bf', 'bf40'):
            # one search = its launches (ref15_search_*_kernel), summed: one kf_search_combos call
            # (bf), or one per class (bf40: 256 class searches, each with its head launch)
            with open(os.path.join(out_dir, f'cfg{c}_FETCH_SIZE.log')) as fh:  # the bench line's own count
                for line in fh:
                    if line.startswith('{"metric"'):
                        rec = json.loads(line)
            alg = rec['roofline']['hbm']['algorithmic_bytes_per_launch']
            classes = rec['config'].get('classes', 1)
            is_search = lambda k: 'ref15_search' in k  # noqa: E731
            fk = per_kernel(os.path.join(out_dir, f'cfg{c}_FETCH_SIZE'), 'FETCH_SIZE')
            wk = per_kernel(os.path.join(out_dir, f'cfg{c}_WRITE_SIZE'), 'WRITE_SIZE')
            f = [v for k, vs in fk.items() if is_search(k) for v in vs]
            w = [v for k, vs in wk.items() if is_search(k) for v in vs]
            searches = len(pick(fk, 'ref15_search_head')) / classes
            fb, info = fetch(out_dir, f'cfg{c}', is_search, f, read_scale)
            fb *= len(f) / searches
            if 'fetch_bytes_calibrated' in info:
                info['fetch_bytes_calibrated'] *= len(f) / searches
            write = 1024 * sum(w) / searches
            res[f'config{c}'] = {
                'fetch_bytes_raw': 1024 * sum(f) / searches, 'write_bytes_raw': write,
                'bytes_per_launch': fb + write * write_scale,
                'algorithmic_bytes_per_launch': alg,
                'traffic_over_algorithmic': (fb + write * write_scale) / alg,
                'launches_profiled': len(f), 'searches_profiled': searches, 'classes': classes,
                'note': f'per search: the sum over its {len(f) / searches:.0f} launches', **info}
            continue
        if c == 'sched':
            # the two passes per launch, each against its own bytes; the algorithmic total is the
            # bench line's (it depends on the picks: n_selected)
            rec = None
            with open(os.path.join(out_dir, 'cfgsched_FETCH_SIZE.log')) as fh:
                for line in fh:
                    if line.startswith('{"metric"'):
                        rec = json.loads(line)
            tot = 0.0
            for tag, kern in (('apply', 'ref15_apply_kernel'), ('pick', 'ref15_pick_kernel')):
                f = pick(per_kernel(os.path.join(out_dir, 'cfgsched_FETCH_SIZE'), 'FETCH_SIZE'), kern)
                w = pick(per_kernel(os.path.join(out_dir, 'cfgsched_WRITE_SIZE'), 'WRITE_SIZE'), kern)
                fb, info = fetch(out_dir, 'cfgsched', lambda k, kern=kern: kern in k, f, read_scale)
                write = 1024 * sum(w) / len(w)
                res[f'configsched_{tag}'] = {'kernel': kern, 'fetch_bytes_raw': 1024 * sum(f) / len(f),
                                             'write_bytes_raw': write, 'bytes_per_launch': fb + write * write_scale,
                                             'launches_profiled': len(f), **info}
                tot += fb + write * write_scale
            alg = rec['roofline']['algorithmic_bytes_per_launch']
            res['configsched'] = {'bytes_per_launch': tot, 'algorithmic_bytes_per_launch': alg,
                                  'traffic_over_algorithmic': tot / alg, 'note': 'pick + apply passes'}
            continue
        kern = {'ref15': 'ref_events', 'ref15f32': 'ref_events', '3gen': 'cv_run_kernel'}.get(c, 'cv_block_kernel')
        f = pick(per_kernel(os.path.join(out_dir, f'cfg{c}_FETCH_SIZE'), 'FETCH_SIZE'), kern)
        w = pick(per_kernel(os.path.join(out_dir, f'cfg{c}_WRITE_SIZE'), 'WRITE_SIZE'), kern)
        fb, info = fetch(out_dir, f'cfg{c}', lambda k: kern in k, f, read_scale)
        write = 1024 * sum(w) / len(w)
        alg, _ = (ref15_algorithmic_bytes if c in ('ref15', 'ref15f32') else algorithmic_bytes)(CONFIGS[str(c)])
        res[f'config{c}'] = {
            'fetch_bytes_raw': 1024 * sum(f) / len(f), 'write_bytes_raw': write,
            'bytes_per_launch': fb + write * write_scale,
            'algorithmic_bytes_per_launch': alg,
            'traffic_over_algorithmic': (fb + write * write_scale) / alg,
            'launches_profiled': len(f), **info}
    with open(os.path.join(out_dir, 'pmc_traffic.json'), 'w') as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
