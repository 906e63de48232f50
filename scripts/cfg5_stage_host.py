"""Host-side split of config 5's bounds/PSIS stage (restarts._native_compute after
the fit): wall-clock marks between its statements, no syncs added (the stage's own
syncs are divergence_rows' and psis_khat's result copies).  One warm-up pass at the
same shapes, then 3 measured passes; JSON lines of per-segment milliseconds."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from viabel_amd import vb, targets, restarts, experiments, bounds, psis, _native as nat
    tgt = targets.eight_schools_ncp()
    R, iters, M = 64, 5000, 1_000_000
    fac = lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox')
    inits = restarts.default_inits(R, 20)
    ids = list(range(R))
    for rep in range(4):
        fam = fac()
        obj = vb.black_box_klvi(fam, tgt, 100)
        run = vb.DeviceRun(obj, iters, inits, window=10, learning_rate=.01, learning_rate_end=.001)
        run.advance_philox(iters, 0, 1, 0, stream_stride=1)
        _, _, vals, smooth = run.result(history=False)
        t = [time.perf_counter()]
        lw = torch.empty((R, M), dtype=torch.float64, device=torch.device('cuda', nat.context().device))
        t.append(time.perf_counter())
        bfam = fac()
        t.append(time.perf_counter())
        experiments.log_weights_rows(tgt, bfam, smooth, M, (1 << 20), 1, lw_out=lw)
        t.append(time.perf_counter())
        div = bounds.divergence_rows(lw)
        t.append(time.perf_counter())
        recs = restarts.bounds_records(ids, div, smooth, bfam)
        t.append(time.perf_counter())
        khat = psis.psis_khat(lw.t())
        t.append(time.perf_counter())
        if rep:
            names = ['torch_empty', 'family', 'logw_launch', 'logw+divergence', 'bounds_records',
                     'psis_khat']
            print(json.dumps({n: round((t[i + 1] - t[i]) * 1e3, 3) for i, n in enumerate(names)}
                             | {'total': round((t[-1] - t[0]) * 1e3, 3)}), flush=True)
        del lw, recs, khat


if __name__ == '__main__':
    main()
