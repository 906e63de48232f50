"""Config 5 time split: the restart optimisation run vs the per-restart
log-weight / bounds / PSIS summaries (one MI355X).  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from viabel_amd import vb, targets, restarts, experiments, bounds, psis, _native as nat
    fac = lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox')
    tgt = targets.eight_schools_ncp()
    sync = lambda: nat.context().synchronize()
    restarts.run_restarts(fac, tgt, 2, 20, n_bounds=1000)
    sync()
    out = {}
    for nb in (1000, 1_000_000):
        t0 = time.perf_counter()
        restarts.run_restarts(fac, tgt, 64, 5000, n_samples=100, n_bounds=nb,
                              learning_rate=.01, learning_rate_end=.001)
        sync()
        out['total_s_nbounds_%d' % nb] = time.perf_counter() - t0
    M = 1_000_000
    lw = torch.empty(M, dtype=torch.float64, device='cuda')
    fam = fac()
    lam = np.random.RandomState(0).randn(20) * 0.5
    for name, fn in [('log_weights', lambda: experiments.log_weights(tgt, fam, lam, M, return_samples=False, lw_out=lw)),
                     ('all_bounds', lambda: bounds.all_bounds(lw, q_var=fam.mean_and_cov(lam)[1],
                                                              moment_bound_fn=lambda p: fam.pth_moment(p, lam))),
                     ('psislw', lambda: psis.psislw(lw))]:
        fn(); sync()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        sync()
        out[name + '_ms'] = (time.perf_counter() - t0) / 10 * 1e3
    print(json.dumps(out))


if __name__ == '__main__':
    main()
