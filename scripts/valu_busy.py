"""Summarise a rocprofv3 --pmc counter_collection.csv of the headline command:
per sep_kernel dispatch, VALUBusy = SQ_ACTIVE_INST_VALU x 4 / SIMDs / (GRBM_GUI_ACTIVE
/ XCDs) (the rocprofiler-sdk derived metric, derived_counters.xml: SQ_ACTIVE_INST_VALU
counts quad-cycles summed over waves; GRBM_GUI_ACTIVE is reported summed over the 8
XCDs, MI355X_MICROARCH.md), and the effective clock GRBM_GUI_ACTIVE / 8 / duration."""
import collections
import csv
import json
import sys

SIMDS, XCDS = 1024, 8


def main(path):
    rows = list(csv.DictReader(open(path)))
    disp = collections.defaultdict(dict)
    for r in rows:
        key = (r.get('Dispatch_Id') or r.get('Correlation_Id'), r['Kernel_Name'])
        disp[key][r['Counter_Name']] = disp[key].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
        if 'Start_Timestamp' in r and r.get('End_Timestamp'):
            disp[key]['_ns'] = float(r['End_Timestamp']) - float(r['Start_Timestamp'])
    out = []
    for (d, name), c in disp.items():
        if 'sep_kernel' not in name or 'GRBM_GUI_ACTIVE' not in c:
            continue
        g = c['GRBM_GUI_ACTIVE'] / XCDS
        busy = c['SQ_ACTIVE_INST_VALU'] * 4 / SIMDS / g if g else None
        rec = {'dispatch': d, 'valu_busy': busy, 'valu_instr': c.get('SQ_INSTS_VALU'),
               'wave_cycles': c.get('SQ_WAVE_CYCLES'), 'busy_cycles': c.get('SQ_BUSY_CYCLES'),
               'gui_active_per_xcd': g}
        if c.get('_ns'):
            rec['clock_ghz'] = g / c['_ns']
        out.append(rec)
    last = out[-1] if out else None
    print(json.dumps({'source': path, 'kernel': 'sep_kernel (headline)', 'dispatches': out,
                      'timed_dispatch_valu_busy': last['valu_busy'] if last else None,
                      'formula': 'SQ_ACTIVE_INST_VALU*4/1024/(GRBM_GUI_ACTIVE/8)'}, indent=1))


if __name__ == '__main__':
    main(sys.argv[1])
