"""Summarise a scripts/profile_bench.sh run (gpurun_out/prof/) into the files
bench.py and DESIGN.md cite:
  profiles/<round>/bench_kernel_stats.csv   rocprofv3 --stats kernel summary
  profiles/<round>/bench_pmc_summary.json   mean counter value per dispatch, per kernel
  profiles/<round>/raw/*.csv                the raw rocprofv3 CSVs
  profiles/traffic.json                      HBM bytes per sep_kernel launch:
      FETCH_SIZE x 2 (gfx950: FETCH_SIZE reports half the bytes of a wide
      streaming read, MI355X_MICROARCH.md) + WRITE_SIZE, KiB -> bytes
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(rnd='r01', src=os.path.join(ROOT, 'gpurun_out', 'prof')):
    dst = os.path.join(ROOT, 'profiles', rnd)
    raw = os.path.join(dst, 'raw')
    os.makedirs(raw, exist_ok=True)
    for f in glob.glob(os.path.join(src, '*', '*', '*.csv')) + glob.glob(os.path.join(src, '*', '*.csv')):
        shutil.copy(f, os.path.join(raw, os.path.basename(os.path.dirname(f)) + '_' + os.path.basename(f)
                                    if not os.path.basename(f).startswith(('trace', 'fetch', 'write', 'sq'))
                                    else os.path.basename(f)))
    stats = glob.glob(os.path.join(src, 'trace', '**', '*kernel_stats.csv'), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, 'bench_kernel_stats.csv'))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, '**', '*counter_collection.csv'), recursive=True):
        per = collections.defaultdict(float)
        for row in csv.DictReader(open(f)):
            per[(row['Kernel_Name'], row['Dispatch_Id'], row['Counter_Name'])] += float(row['Counter_Value'])
        for (k, _, c), v in per.items():
            acc[k][c].append(v)
    summary = {k: {c: {'dispatches': len(v), 'mean_per_dispatch': sum(v) / len(v)}
                   for c, v in d.items()} for k, d in acc.items()}
    json.dump(summary, open(os.path.join(dst, 'bench_pmc_summary.json'), 'w'), indent=1)
    sep = [k for k in summary if 'sep_kernel' in k]
    if sep:
        k = max(sep, key=lambda n: summary[n].get('FETCH_SIZE', {}).get('dispatches', 0))
        fetch = summary[k]['FETCH_SIZE']['mean_per_dispatch']
        write = summary[k]['WRITE_SIZE']['mean_per_dispatch']
        out = {'source': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (profiles/%s/bench_pmc_summary.json); '
                         'FETCH_SIZE doubled per MI355X_MICROARCH.md gfx950 correction (upper bound for '
                         '8-B accesses); per sep_kernel launch of 256 steps; kernel %s' % (rnd, k),
               'fetch_kb_raw': fetch, 'write_kb': write,
               'bytes_per_launch': int(round((2 * fetch + write) * 1024))}
        if 'SQ_INSTS_VALU' in summary[k]:
            out['valu_instr_per_launch'] = summary[k]['SQ_INSTS_VALU']['mean_per_dispatch']
        json.dump(out, open(os.path.join(ROOT, 'profiles', 'traffic.json'), 'w'), indent=1)
        print(json.dumps(out))
    if stats:
        for row in list(csv.DictReader(open(stats[0])))[:6]:
            print(row['Name'][:80], row['Calls'], row['AverageNs'])


if __name__ == '__main__':
    main(*sys.argv[1:])
