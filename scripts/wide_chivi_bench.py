"""Per-step time of the wide mean-field paths (D > 16): KLVI on the fused
column-pair kernel vs CHIVI / KLVI-pd on the materialised path.  One MI355X."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from viabel_amd import vb, targets, _native as nat
    D = int(os.environ.get('D', '10000'))
    N = int(os.environ.get('N', '128'))
    steps = int(os.environ.get('STEPS', '400'))
    out = {'D': D, 'N': N}
    for fam_kind in ('gauss', 't'):
        for obj_kind in ('klvi', 'chivi'):
            fam = (vb.mean_field_gaussian_variational_family(D, rng='philox') if fam_kind == 'gauss'
                   else vb.mean_field_t_variational_family(D, 40.0, rng='philox'))
            tgt = targets.isogauss(D)
            obj = (vb.black_box_klvi(fam, tgt, N) if obj_kind == 'klvi'
                   else vb.black_box_chivi(2.0, fam, tgt, N))
            init = np.concatenate([np.zeros(D), np.zeros(D)])
            run = vb.DeviceRun(obj, steps + 20, init[None], learning_rate=.001)
            run.advance_philox(20, 0, 1, 0)
            nat.context().synchronize()
            t0 = time.perf_counter()
            run.advance_philox(steps, 0, 1, 20)
            nat.context().synchronize()
            out['%s_%s_us_per_step' % (fam_kind, obj_kind)] = (time.perf_counter() - t0) / steps * 1e6
    print(json.dumps(out))


if __name__ == '__main__':
    main()
