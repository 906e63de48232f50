"""Config 4: full-rank t, D = 512, df = 100, CHIVI alpha = 2,
N = 128, corr_gauss target, device adagrad with Philox draws.  Prints the
per-step time and MC-samples/s; --cpu also times the oracle's reference
algorithm (scipy sqrtm + solve_sylvester) for one step."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--D', type=int, default=512)
    ap.add_argument('--N', type=int, default=128)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--objective', default='chivi')
    ap.add_argument('--cpu', action='store_true')
    a = ap.parse_args()
    import torch
    from viabel_amd import vb, targets, _native as nat
    D, N = a.D, a.N
    rs = np.random.RandomState(4)
    tri = np.tril_indices(D)
    free = rs.randn(len(tri[0])) * 0.01
    free[tri[0] == tri[1]] = rs.randn(D) * 0.1
    lam0 = np.concatenate([np.zeros(D), free])
    fam = vb.t_variational_family(D, 100.0, rng='philox')
    tgt = targets.corr_gauss(D)
    obj = (vb.black_box_chivi(2.0, fam, tgt, N) if a.objective == 'chivi'
           else vb.black_box_klvi(fam, tgt, N))
    run = vb.DeviceRun(obj, a.steps + 3, lam0, learning_rate=.01)
    run.advance_philox(3, 0, 1, 0)
    nat.context().synchronize()
    t0 = time.perf_counter()
    run.advance_philox(a.steps, 0, 1, 3)
    nat.context().synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    out = {'config': 'cfg4', 'D': D, 'N': N, 'objective': a.objective, 'ms_per_step': dt * 1e3,
           'mc_samples_per_s': N * D / dt}
    vals = run.result()[2][0]
    out['finite'] = bool(np.all(np.isfinite(vals)))
    if a.cpu:
        from oracle import fullrank_oracle as fo
        ofam = fo.FullRankT(D, 100.0)
        otgt = fo.target_fn('corr_gauss', D)
        t0 = time.perf_counter()
        np.random.seed(0)
        fo.chivi_value_grad(ofam, otgt, lam0, N, 2.0)
        out['cpu_ms_per_step'] = (time.perf_counter() - t0) * 1e3
    print(json.dumps(out))


if __name__ == '__main__':
    main()
