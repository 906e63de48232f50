"""Per-kernel timeline of one config-4 step from a rocprofv3 kernel trace
(scripts/gpu_fr_prof.sh): python scripts/fr_step_trace.py [trace.csv] [step]."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof_fr/fr_kernel_trace.csv'
k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
# a step starts with Sigma = L L^T, the step's only NT GEMM (fused steps have
# no unpack launch)
starts = [i for i, r in enumerate(rows) if 'gemm_f64_kernel<false, true' in r['Kernel_Name']]
i0, i1 = starts[k], starts[k + 1]
t0 = int(rows[i0]['Start_Timestamp'])
prev = t0
groups = {}
for r in rows[i0:i1]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    name = r['Kernel_Name'].split('(')[0].replace('vbk::', '').replace('(anonymous namespace)::', '')
    name = name.replace('gemm_detail::', '')
    print('%8.2f %7.2f gap %5.2f %s' % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, name[-60:]))
    g = groups.setdefault(name[-60:], [0, 0.0])
    g[0] += 1
    g[1] += (e - s) / 1e3
    prev = e
print('step span %.2f us, %d kernels' % ((int(rows[i1]['Start_Timestamp']) - t0) / 1e3, i1 - i0))
for n, (c, t) in sorted(groups.items(), key=lambda x: -x[1][1]):
    print('%4d %8.2f %s' % (c, t, n))
