"""Per-step time of one block-kernel problem against D (t funnel CHIVI, N = 128,
pre-drawn noise + copy wave) with the step floor at each shape: how much of the
step scales with the per-sample row work.  One JSON line per D."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from viabel_amd import vb, targets, _native as nat
    steps = 3000
    for D in (2, 4, 6, 8, 10, 12, 16):
        fam = vb.mean_field_t_variational_family(D, 40.0, rng='philox')
        obj = vb.black_box_chivi(2.0, fam, targets.funnel(D), 128)
        run = vb.DeviceRun(obj, steps + 200, np.zeros((1, 2 * D)), learning_rate=.001)
        run.advance_philox(200, 0, 1, 0)
        nat.context().synchronize()
        t0 = time.perf_counter()
        run.advance_philox(steps, 0, 1, 200)
        nat.context().synchronize()
        us = (time.perf_counter() - t0) / steps * 1e6
        fl = nat.block_floor_us(D, 128, chivi=True, host_layout=True, n_steps=2000, n_problems=1)
        print(json.dumps({'D': D, 'us_per_step': round(us, 3), 'floor_us': round(fl, 3)}), flush=True)


if __name__ == '__main__':
    main()
