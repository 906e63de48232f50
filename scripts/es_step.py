"""Per-step time of the block kernel on the config-5 problem (eight-schools NCP,
mf-t(40) KLVI, N = 100, Philox) for P concurrent restarts (one workgroup each):
python scripts/es_step.py [P ...].  Also the whole 5 000-iteration run with the
config's learning-rate schedule, as restarts.run_restarts launches it."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401  (HIP runtime first)
    from viabel_amd import vb, targets, _native as nat
    D, N = 10, 100
    for P in [int(a) for a in sys.argv[1:]] or [1, 64]:
        fam = vb.mean_field_t_variational_family(D, 40.0, rng='philox')
        obj = vb.black_box_klvi(fam, targets.eight_schools_ncp(), N)
        init = np.random.RandomState(0).randn(P, 2 * D) * 0.5
        run = vb.DeviceRun(obj, 3000, init, learning_rate=.01)
        run.advance_philox(1000, 0, 1, 0)
        nat.context().synchronize()
        t0 = time.perf_counter()
        run.advance_philox(2000, 0, 1, 1000)
        nat.context().synchronize()
        print('P', P, 'us_per_step', (time.perf_counter() - t0) / 2000 * 1e6, flush=True)
        run = vb.DeviceRun(obj, 5000, init, learning_rate=.01, learning_rate_end=.001)
        nat.context().synchronize()
        t0 = time.perf_counter()
        run.advance_philox(5000, 0, 1, 0)
        nat.context().synchronize()
        t1 = time.perf_counter()
        run.result()
        t2 = time.perf_counter()
        print('P', P, 'full 5000-iter run: advance %.2f ms, result %.2f ms' %
              ((t1 - t0) * 1e3, (t2 - t1) * 1e3), flush=True)


if __name__ == '__main__':
    main()
