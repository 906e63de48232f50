"""Summarise a scripts/profile_r02.sh run (gpurun_out/prof2/) into the files
bench.py and DESIGN.md cite:
  profiles/<round>/driver_cmd_kernel_stats.csv   rocprofv3 --stats of the driver command
  profiles/<round>/driver_cmd_dispatches.csv     every sep_kernel / sep_values dispatch
                                                 (start-ordered, duration in us)
  profiles/<round>/pmc_per_dispatch.json         summed counters per sep_kernel dispatch
  profiles/<round>/raw_counters/n<N>_<pass>_counters.csv
                                                 the raw rocprofv3 counter CSV of every PMC
                                                 pass (renamed: *counter_collection.csv is
                                                 git-ignored as scratch)
  profiles/traffic.json                          per-launch models a + b * steps, per N:
      traffic_bytes = FETCH_SIZE x 2 (gfx950: FETCH_SIZE reports half the bytes of
      a wide streaming read, MI355X_MICROARCH.md) + WRITE_SIZE, KiB -> bytes;
      valu_instr = SQ_INSTS_VALU
The PMC runs launch sep_kernel for 5 (warm-up), 256 and 20 steps, in that order,
over a 281-step run whose history rows (vb.py:375-376) start at step 210, so the
three launches write 0, 51 and 20 history rows: the byte model is
a + b * steps + c * history_rows (solved exactly from the three launches).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PMC_STEPS = [5, 256, 20]
PMC_HIST = [0, 51, 20]


def per_dispatch(pass_dir):
    files = glob.glob(os.path.join(pass_dir, '**', '*counter_collection.csv'), recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if 'sep_kernel' not in row['Kernel_Name']:
                continue
            did = int(row['Dispatch_Id'])
            per[did][row['Counter_Name']] += float(row['Counter_Value'])
            names[did] = row['Kernel_Name']
    return [(d, names[d], dict(per[d])) for d in sorted(per)]


def fit(steps, ys):
    A = np.stack([np.ones(len(steps)), np.asarray(steps, float)], 1)
    coef, *_ = np.linalg.lstsq(A, np.asarray(ys, float), rcond=None)
    pred = A @ coef
    return [float(coef[0]), float(coef[1])], float(np.max(np.abs(pred - ys) / np.abs(ys)))


def main(rnd='r02', src=os.path.join(ROOT, 'gpurun_out', 'prof2')):
    dst = os.path.join(ROOT, 'profiles', rnd)
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, 'trace', '**', '*kernel_stats.csv'), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, 'driver_cmd_kernel_stats.csv'))
        for row in list(csv.DictReader(open(stats[0])))[:8]:
            print(row['Name'][:90], row['Calls'], row['AverageNs'])
    traces = glob.glob(os.path.join(src, 'trace', '**', '*kernel_trace.csv'), recursive=True)
    if traces:
        rows = [r for r in csv.DictReader(open(traces[0]))
                if 'sep_kernel' in r['Kernel_Name'] or 'sep_values' in r['Kernel_Name']]
        rows.sort(key=lambda r: int(r['Start_Timestamp']))
        with open(os.path.join(dst, 'driver_cmd_dispatches.csv'), 'w') as fo:
            fo.write('dispatch,kernel,duration_us\n')
            for r in rows:
                dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
                fo.write('%s,%s,%.2f\n' % (r['Dispatch_Id'], r['Kernel_Name'].split('(')[0], dur))
        print(open(os.path.join(dst, 'driver_cmd_dispatches.csv')).read())
    raw = os.path.join(dst, 'raw_counters')
    os.makedirs(raw, exist_ok=True)
    for ns in ('128', '256'):
        for kind in ('fetch', 'write', 'sq'):
            for f in glob.glob(os.path.join(src, 'n%s_%s' % (ns, kind), '**',
                                            '*counter_collection.csv'), recursive=True):
                shutil.copy(f, os.path.join(raw, 'n%s_%s_counters.csv' % (ns, kind)))
    models, pmc = {}, {}
    for ns in ('128', '256'):
        disp = {}
        for kind in ('fetch', 'write', 'sq'):
            d = per_dispatch(os.path.join(src, 'n%s_%s' % (ns, kind)))
            if len(d) != len(PMC_STEPS):
                print('n%s_%s: %d sep_kernel dispatches, expected %d' % (ns, kind, len(d),
                                                                        len(PMC_STEPS)))
                continue
            for k, (_, name, cnt) in zip(PMC_STEPS, d):
                disp.setdefault(k, {'kernel': name})
                disp[k].update(cnt)
        if not disp:
            continue
        pmc[ns] = disp
        ks = PMC_STEPS
        tb = [(2 * disp[k]['FETCH_SIZE'] + disp[k]['WRITE_SIZE']) * 1024 for k in ks]
        vi = [disp[k]['SQ_INSTS_VALU'] for k in ks]
        A = np.array([[1.0, k, h] for k, h in zip(ks, PMC_HIST)])
        tcoef = [float(v) for v in np.linalg.solve(A, np.array(tb))]
        vcoef, verr = fit(ks, vi)
        models[ns] = {'traffic_bytes': tcoef, 'traffic_terms': ['per launch', 'per step',
                                                                'per history row'],
                      'valu_instr': vcoef, 'valu_fit_max_rel_err': verr,
                      'launch_steps': ks, 'launch_history_rows': PMC_HIST}
    json.dump(pmc, open(os.path.join(dst, 'pmc_per_dispatch.json'), 'w'), indent=1)
    if models:
        out = {'source': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU passes '
                         '(profiles/%s/pmc_per_dispatch.json, raw counters in raw_counters/ beside '
                         'it, scripts/profile_r02.sh); per '
                         'sep_kernel launch of k steps writing h history rows: bytes = a + b k + c h, '
                         'VALU instructions = a + b k, over k in %s; '
                         'FETCH_SIZE doubled per the MI355X_MICROARCH.md gfx950 correction '
                         '(upper bound for 8-B accesses)' % (rnd, PMC_STEPS),
               'models': models}
        json.dump(out, open(os.path.join(ROOT, 'profiles', 'traffic.json'), 'w'), indent=1)
        print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:])
