"""Per-step latency of the block kernel (one problem, Philox draws) over N and D:
isolates the fixed per-step cost of the single-small-problem configs (1, 2)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))


def main():
    import torch
    from viabel_amd import vb, targets, _native as nat
    out = []
    steps = int(os.environ.get("BL_STEPS", "4000"))
    for (fam_kind, tgt, D, N, obj_kind) in [('gauss', 'isogauss', 2, 1, 'klvi'),
                                            ('gauss', 'isogauss', 2, 100, 'klvi'),
                                            ('gauss', 'mixture', 2, 100, 'klvi'),
                                            ('gauss', 'isogauss', 10, 128, 'klvi'),
                                            ('t', 'isogauss', 10, 128, 'klvi'),
                                            ('t', 'funnel', 10, 128, 'klvi'),
                                            ('t', 'funnel', 10, 128, 'chivi'),
                                            ('gauss', 'funnel', 10, 128, 'chivi')]:
        fam = (vb.mean_field_gaussian_variational_family(D, rng='philox') if fam_kind == 'gauss'
               else vb.mean_field_t_variational_family(D, 40.0, rng='philox'))
        t = {'isogauss': targets.isogauss, 'mixture': targets.mixture, 'funnel': targets.funnel}[tgt](D)
        obj = vb.black_box_klvi(fam, t, N) if obj_kind == 'klvi' else vb.black_box_chivi(2.0, fam, t, N)
        init = np.concatenate([np.zeros(D), np.zeros(D)])
        run = vb.DeviceRun(obj, steps + 100, init[None], learning_rate=.001)
        run.advance_philox(100, 0, 1, 0)
        nat.context().synchronize()
        t0 = time.perf_counter()
        run.advance_philox(steps, 0, 1, 100)
        nat.context().synchronize()
        dt = (time.perf_counter() - t0) / steps
        out.append({'fam': fam_kind, 'target': tgt, 'D': D, 'N': N, 'obj': obj_kind,
                    'us_per_step': dt * 1e6})
        print(json.dumps(out[-1]), flush=True)


if __name__ == '__main__':
    main()
