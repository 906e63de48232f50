import cProfile, pstats, os, sys, time
sys.path.insert(0, os.getcwd())
import torch
from viabel_amd import vb, targets, restarts, _native as nat
fac = lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox')
tgt = targets.eight_schools_ncp()
restarts.run_restarts(fac, tgt, 2, 20, n_bounds=1000)
nat.context().synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
restarts.run_restarts(fac, tgt, 64, 5000, n_samples=100, n_bounds=1000, learning_rate=.01, learning_rate_end=.001)
nat.context().synchronize()
pr.disable()
print('total', time.perf_counter() - t0)
pstats.Stats(pr).sort_stats('cumulative').print_stats(25)
