"""Config 1's adagrad_optimize call (mixture D = 2, mf-Gauss KLVI, N = 100) at several
iteration counts: per-step time against the call's fixed part (the least-squares line
of call seconds on iterations), after a warm-up at each count."""
import sys
import time
sys.path.insert(0, '.')
import numpy as np
from viabel_amd import vb, targets, _native as nat

fam = vb.mean_field_gaussian_variational_family(2, rng='philox')
obj = vb.black_box_klvi(fam, targets.mixture(2), 100)
lam0 = np.array([0., 0., 1., 1.])
xs, ys = [], []
for iters in (500, 1000, 2000, 5000, 10000, 20000):
    vb.adagrad_optimize(iters, obj, lam0)
    nat.context().synchronize()
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        vb.adagrad_optimize(iters, obj, lam0)
        nat.context().synchronize()
        best = min(best, time.perf_counter() - t0)
    xs.append(iters)
    ys.append(best)
    print('iters %6d  call %.3f ms  %.3f us/step' % (iters, best * 1e3, best / iters * 1e6), flush=True)
b, a = np.polyfit(xs, ys, 1)
print('fit: %.3f us/step + %.3f ms fixed per call' % (b * 1e6, a * 1e3))
