#!/bin/bash
# Round 5, GPU session ai: rocprofv3 kernel trace + stats of the driver's command on the final
# tree (scripts/profile_r02.sh trace pass), summarised into gpurun_out/rec3/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/rec3
export TMPDIR=/tmp
rm -rf gpurun_out/prof2
PASSES="trace" bash scripts/profile_r02.sh > gpurun_out/rec3/prof2.log 2>&1
grep -q '^{' gpurun_out/prof2/trace.log && find gpurun_out/prof2/trace -name "*kernel_stats.csv" | grep -q . || { tail -5 gpurun_out/rec3/prof2.log; exit 1; }
f=$(find gpurun_out/prof2/trace -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/rec3/driver_cmd_kernel_stats.csv
t=$(find gpurun_out/prof2/trace -name "*kernel_trace.csv" | head -1)
python3 - "$t" > gpurun_out/rec3/driver_cmd_dispatches.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'sep_kernel' in r['Kernel_Name'] or 'sep_values_kernel' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
print('dispatch,kernel,duration_us')
for r in rows:
    print('%s,%s,%.2f' % (r['Dispatch_Id'], r['Kernel_Name'], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
PY
head -8 gpurun_out/rec3/driver_cmd_dispatches.csv
