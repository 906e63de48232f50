"""Config 5 end to end, three times: the whole call against the rank-local call
(local_s), the fit and bounds stages and the default inits alone (host split of
the ~1.4 ms outside the two stages)."""
import time, sys
sys.path.insert(0,'.')
import numpy as np, torch
from viabel_amd import vb, targets, restarts, _native as nat
fac = lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox')
tgt = targets.eight_schools_ncp()
restarts.run_restarts(fac, tgt, 64, 20, n_bounds=1_000_000)
nat.context().synchronize()
inits0 = restarts.default_inits(64, 20)
for rep in range(6):
    tm={}
    inits = inits0 if rep % 2 else None
    t0=time.perf_counter()
    tab=restarts.run_restarts(fac, tgt, 64, 5000, n_samples=100, n_bounds=1_000_000, learning_rate=.01, learning_rate_end=.001, inits=inits, timings=tm)
    nat.context().synchronize()
    dt=time.perf_counter()-t0
    t1=time.perf_counter(); x=restarts.default_inits(64,20); ti=time.perf_counter()-t1
    print(('given inits ' if rep % 2 else 'own inits   ') + 'pre %.3f post %.3f ' % (tm['pre_s']*1e3, tm['post_s']*1e3) + 'total %.3f ms local %.3f fit %.3f bounds %.3f inits %.3f' % (dt*1e3, tm['local_s']*1e3, tm['fit_s']*1e3, tm['bounds_psis_s']*1e3, ti*1e3), flush=True)
