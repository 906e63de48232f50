"""Config 5's fitting stage split into its host and device pieces (one MI355X):
objective + DeviceRun creation, the advance (pre-draw + block launches, synced),
and run.result(); each the median of 5 runs after a warm-up.  One JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from viabel_amd import vb, targets, restarts, _native as nat
    sync = lambda: nat.context().synchronize()
    tgt = targets.eight_schools_ncp()
    R, iters = 64, 5000
    inits = restarts.default_inits(R, 20)
    res = {}
    for rep in range(6):
        fam = vb.mean_field_t_variational_family(10, 40.0, rng='philox')
        sync()
        t0 = time.perf_counter()
        obj = vb.black_box_klvi(fam, tgt, 100)
        run = vb.DeviceRun(obj, iters, inits, window=10, learning_rate=.01, learning_rate_end=.001)
        sync()
        t1 = time.perf_counter()
        run.advance_philox(iters, 0, 1, 0, stream_stride=1)
        t2 = time.perf_counter()
        sync()
        t3 = time.perf_counter()
        out = run.result()
        sync()
        t4 = time.perf_counter()
        if rep:
            for k, v in (('create', t1 - t0), ('advance_submit', t2 - t1), ('advance', t3 - t1),
                         ('result', t4 - t3), ('total', t4 - t0)):
                res.setdefault(k, []).append(v * 1e3)
    print(json.dumps({k + '_ms': round(float(np.median(v)), 3) for k, v in res.items()}))


if __name__ == '__main__':
    main()
