"""Config 5's bounds / PSIS stage alone, for counter passes: 64 restarts fitted
for a few iterations (the stage's cost does not depend on how well), then one
run of the stage at M = 1e6 (vb_log_weights_rows, divergence / Wasserstein
bounds, psislw per restart)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from viabel_amd import vb, targets, restarts, _native as nat
    fac = lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox')
    tgt = targets.eight_schools_ncp()
    restarts.run_restarts(fac, tgt, 4, 20, n_bounds=1000)          # code objects
    nat.context().synchronize()
    tm = {}
    t0 = time.perf_counter()
    restarts.run_restarts(fac, tgt, 64, 50, n_samples=100, n_bounds=1_000_000,
                          learning_rate=.01, learning_rate_end=.001, timings=tm)
    nat.context().synchronize()
    print('total_s %.4f bounds_psis_s %.4f' % (time.perf_counter() - t0, tm.get('bounds_psis_s', -1)),
          flush=True)


if __name__ == '__main__':
    main()
