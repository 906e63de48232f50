"""Per-kernel summary of the config-5 bounds-stage counter passes
(scripts/gpu_cfg5_pmc.sh): duration (kernel trace), SQ_INSTS_VALU and its rate
against the fp64 VALU issue peak, HBM bytes (FETCH_SIZE doubled per the gfx950
correction, WRITE_SIZE), for the dispatches of the M = 1e6 stage."""
import collections
import csv
import json
import sys

base = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/cfg5_pmc'
VALU_PEAK = 256 * 4 * 2.4e9 / 4      # wave64 fp64 instructions / s


def short(n):
    n = n.split('(')[0].replace('vbk::', '').replace('(anonymous namespace)::', '')
    return n.replace('void ', '')[:70]


def per_dispatch(path):
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d[int(r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value'])
        d[int(r['Dispatch_Id'])]['name'] = r['Kernel_Name']
        d[int(r['Dispatch_Id'])]['grid'] = int(r['Grid_Size'])
    return d


trace = sorted(csv.DictReader(open(base + '/trace/run_kernel_trace.csv')),
               key=lambda r: int(r['Start_Timestamp']))
sq = per_dispatch(base + '/sq/run_counter_collection.csv')
fe = per_dispatch(base + '/fetch/run_counter_collection.csv')
wr = per_dispatch(base + '/write/run_counter_collection.csv')
# the M = 1e6 stage: dispatches after the 64-restart fit's last block kernel
last_fit = max(i for i, r in enumerate(trace) if 'block_kernel' in r['Kernel_Name'])
stage = trace[last_fit + 1:]
t_stage = (int(stage[-1]['End_Timestamp']) - int(stage[0]['Start_Timestamp'])) * 1e-9
first_id = int(stage[0]['Dispatch_Id'])
agg = collections.OrderedDict()
for r in stage:
    k = short(r['Kernel_Name'])
    a = agg.setdefault(k, {'calls': 0, 'ms': 0.0, 'valu': 0.0, 'fetch': 0.0, 'write': 0.0})
    a['calls'] += 1
    a['ms'] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-6
    did = int(r['Dispatch_Id'])
    a['valu'] += sq.get(did, {}).get('SQ_INSTS_VALU', 0.0)
    a['fetch'] += 2 * fe.get(did, {}).get('FETCH_SIZE', 0.0) * 1024   # KB -> B, gfx950 x2
    a['write'] += wr.get(did, {}).get('WRITE_SIZE', 0.0) * 1024
tot = {'stage_span_ms': t_stage * 1e3, 'kernels_ms': sum(a['ms'] for a in agg.values()),
       'valu_instr': sum(a['valu'] for a in agg.values())}
tot['valu_frac_of_span'] = tot['valu_instr'] / (t_stage * VALU_PEAK)
out = {'stage': tot, 'kernels': {}}
for k, a in sorted(agg.items(), key=lambda x: -x[1]['ms']):
    s = a['ms'] * 1e-3
    out['kernels'][k] = {'calls': a['calls'], 'ms': round(a['ms'], 4),
                         'valu_instr': a['valu'], 'valu_frac': a['valu'] / (s * VALU_PEAK) if s else None,
                         'fetch_bytes': a['fetch'], 'write_bytes': a['write'],
                         'hbm_GBs': (a['fetch'] + a['write']) / s / 1e9 if s else None}
print(json.dumps(out, indent=1))
