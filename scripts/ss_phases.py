"""Phase split of the symmetric-sum PCG launches from a VB_SS_PROF build
(scripts/build_variant.sh ssprof -DVB_SS_PROF=8): every block prints its
s_memrealtime stamps (100 MHz); per launch, the median / max over blocks of each
phase boundary relative to the launch's first block entry, in us.
    VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_ssprof.so python scripts/bench_fr.py --steps 12 \\
        > ss.log; python scripts/ss_phases.py ss.log"""
import collections
import statistics
import sys

NAMES = ['entry', 'issued', 'stage0', 'mainloop', 'product', 'scalars', 'end']


def main(path):
    runs = collections.defaultdict(list)
    for line in open(path):
        if not line.startswith('SSPROF'):
            continue
        f = line.split()
        mode, it, b, hw = int(f[1]), int(f[2]), int(f[3]), int(f[4])
        runs[(it, mode)].append([int(x) for x in f[5:12]])
    order = sorted(runs, key=lambda k: min(r[0] for r in runs[k]))
    print('%-10s %6s  ' % ('launch', 'blocks') + '  '.join('%15s' % n for n in NAMES))
    for k in order:
        rs = runs[k]
        t0 = min(r[0] for r in rs)
        cols = []
        for j in range(7):
            v = [(r[j] - t0) / 100.0 for r in rs]
            cols.append('%6.2f /%6.2f' % (statistics.median(v), max(v)))
        print('it%-2d m%d    %6d  ' % (k[0], k[1], len(rs)) + '  '.join('%15s' % c for c in cols))
    # per-phase durations (median over blocks) across launches
    print('\nmedian phase durations over all launches (us):')
    d = collections.defaultdict(list)
    for k in order:
        for r in runs[k]:
            for j in range(1, 7):
                d[NAMES[j]].append((r[j] - r[j - 1]) / 100.0)
    for j in range(1, 7):
        print('  %-9s %6.2f' % (NAMES[j], statistics.median(d[NAMES[j]])))


if __name__ == '__main__':
    main(sys.argv[1])
