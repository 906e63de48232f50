"""Measure BASELINE.json configs 1, 2, 4 and 5 on one MI355X and
time the oracle's CPU restatement on bounded samples of the same workloads.
config 3 is bench.py's headline line.  Prints one JSON line per config.

  python scripts/bench_configs.py [--configs 1,2,4,5] [--cpu-seconds 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _sync():
    from viabel_amd import _native as nat
    nat.context().synchronize()


def _cpu_steps(fn, lam, seconds, lr=.01, lr_end=None, n_iters=None, window=10, eps=.1):
    """Oracle adagrad steps until `seconds` elapse; returns seconds per step."""
    from oracle import vb_oracle
    grads = []
    sched = list(vb_oracle.learning_rate_schedule(n_iters, lr, lr_end)) if n_iters else None
    t0 = time.perf_counter()
    k = 0
    while True:
        v, g = fn(lam)
        grads.append(g)
        if len(grads) > window:
            grads.pop(0)
        acc = np.sum(np.array(grads) ** 2, axis=0)
        cur = sched[k % len(sched)] if sched else lr
        lam = lam - cur * g / np.sqrt(eps + acc)
        k += 1
        if time.perf_counter() - t0 >= seconds:
            break
    return (time.perf_counter() - t0) / k, k


def config1(cpu_s):
    """2-D normal mixture, mf-Gauss KLVI, N=100, 5000 adagrad iterations + bounds on 5e4 draws."""
    from viabel_amd import vb, targets, bounds, experiments
    D, N, iters = 2, 100, 5000
    lam0 = np.array([0., 0., 1., 1.])
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj = vb.black_box_klvi(fam, targets.mixture(D), N)
    vb.adagrad_optimize(iters, obj, lam0)        # warm-up (module load, kernels, first
                                                 # pageable-copy staging of this size)
    _sync()
    t0 = time.perf_counter()
    sm = vb.adagrad_optimize(iters, obj, lam0)[0]
    _sync()
    t_opt = time.perf_counter() - t0
    t0 = time.perf_counter()
    _, lw = experiments.log_weights(targets.mixture(D), fam, sm, 50000, return_samples=False)
    bounds.all_bounds(lw, q_var=fam.mean_and_cov(sm)[1],
                      moment_bound_fn=lambda p: fam.pth_moment(p, sm))
    t_b = time.perf_counter() - t0
    from oracle import vb_oracle
    ofam = vb_oracle.Family('gauss', D)
    cpu_step, k = _cpu_steps(lambda l: vb_oracle.klvi_value_grad(ofam, 'mixture', l, N), lam0,
                             cpu_s)
    return {'config': 1, 'workload': 'mixture D=2 mf-gauss KLVI N=100, 5000 iters',
            'gpu_ms_per_step': t_opt / iters * 1e3, 'gpu_steps_per_s': iters / t_opt,
            'gpu_bounds_s': t_b, 'cpu_ms_per_step': cpu_step * 1e3, 'cpu_steps_sampled': k,
            'speedup': cpu_step / (t_opt / iters)}


def config2(cpu_s):
    """Funnel D=10, mf-t df=40, CHIVI alpha=2, N=128, lr .01 -> .001, 10 000 iterations."""
    from viabel_amd import vb, targets
    D, N, iters = 10, 128, 10000
    lam0 = np.concatenate([np.zeros(D), np.ones(D)])
    lam0[1] = -1.0
    fam = vb.mean_field_t_variational_family(D, 40.0, rng='philox')
    obj = vb.black_box_chivi(2.0, fam, targets.funnel(D), N)
    vb.adagrad_optimize(50, obj, lam0, learning_rate_end=.001)
    _sync()
    t0 = time.perf_counter()
    vb.adagrad_optimize(iters, obj, lam0, learning_rate=.01, learning_rate_end=.001)
    _sync()
    dt = (time.perf_counter() - t0) / iters
    from oracle import vb_oracle
    ofam = vb_oracle.Family('t', D, 40.0)
    cpu_step, k = _cpu_steps(lambda l: vb_oracle.chivi_value_grad(ofam, 'funnel', l, N, 2.0),
                             lam0, cpu_s, lr_end=.001, n_iters=iters)
    return {'config': 2, 'workload': 'funnel D=10 mf-t(40) CHIVI a=2 N=128, 10000 iters',
            'gpu_ms_per_step': dt * 1e3, 'gpu_mc_samples_per_s': N * D / dt,
            'cpu_ms_per_step': cpu_step * 1e3, 'cpu_steps_sampled': k,
            'cpu_mc_samples_per_s': N * D / cpu_step, 'speedup': cpu_step / dt}


def config4(cpu_s, steps=30):
    """Full-rank t D=512 df=100, CHIVI alpha=2 N=128, corr_gauss target."""
    from viabel_amd import vb, targets
    D, N = 512, 128
    rs = np.random.RandomState(4)
    tri = np.tril_indices(D)
    free = rs.randn(len(tri[0])) * 0.01
    free[tri[0] == tri[1]] = rs.randn(D) * 0.1
    lam0 = np.concatenate([np.zeros(D), free])
    fam = vb.t_variational_family(D, 100.0, rng='philox')
    tgt = targets.corr_gauss(D)
    obj = vb.black_box_chivi(2.0, fam, tgt, N)
    run = vb.DeviceRun(obj, steps + 3, lam0)
    run.advance_philox(3, 0, 1, 0)
    _sync()
    t0 = time.perf_counter()
    run.advance_philox(steps, 0, 1, 3)
    _sync()
    dt = (time.perf_counter() - t0) / steps
    from oracle import fullrank_oracle as fo
    ofam = fo.FullRankT(D, 100.0)
    otgt = fo.target_fn('corr_gauss', D)
    np.random.seed(0)
    cpu_step, k = _cpu_steps(lambda l: fo.chivi_value_grad(ofam, otgt, l, N, 2.0), lam0, cpu_s)
    flops = 8 * N * D * D + 20 * D ** 3          # SURVEY §8d config 4 algorithmic flops / step
    return {'config': 4, 'workload': 'full-rank t D=512 df=100 CHIVI a=2 N=128 corr_gauss',
            'gpu_ms_per_step': dt * 1e3, 'gpu_mc_samples_per_s': N * D / dt,
            'algorithmic_tflops': flops / dt / 1e12, 'fp64_peak_tflops': 78.6,
            'cpu_ms_per_step': cpu_step * 1e3, 'cpu_steps_sampled': k,
            'cpu_kind': 'oracle: scipy sqrtm + solve_sylvester (the reference algorithm)',
            'speedup': cpu_step / dt}


def config5(cpu_s, n_restarts=64, iters=5000, M=1_000_000):
    """8-schools NCP, 64 KLVI restarts (mf-t df=40, N=100, lr .01 -> .001) + bounds/PSIS on
    M = 1e6 log weights per restart, one GPU (the 8-GPU run shards restarts)."""
    from viabel_amd import vb, targets, restarts
    fac = lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox')
    tgt = targets.eight_schools_ncp()
    restarts.run_restarts(fac, tgt, 2, 20, n_bounds=1000)     # warm-up
    _sync()
    t0 = time.perf_counter()
    tab = restarts.run_restarts(fac, tgt, n_restarts, iters, n_samples=100, n_bounds=M,
                                learning_rate=.01, learning_rate_end=.001)
    _sync()
    dt = time.perf_counter() - t0
    # CPU: one restart's optimisation (bounded) + bounds/PSIS on a bounded M
    from oracle import vb_oracle, bounds_oracle, psis_oracle
    ofam = vb_oracle.Family('t', 10, 40.0)
    lam0 = np.random.RandomState(0).randn(20) * 0.5
    cpu_step, k = _cpu_steps(lambda l: vb_oracle.klvi_value_grad(ofam, 'eight_schools_ncp', l, 100),
                             lam0, cpu_s / 2, lr_end=.001, n_iters=iters)
    Mc = 200_000
    t0 = time.perf_counter()
    _, lw = vb_oracle.log_weights(ofam, 'eight_schools_ncp', lam0, Mc)
    bounds_oracle.divergence_bound(lw)
    psis_oracle.psislw(lw.copy())
    t_lw = (time.perf_counter() - t0) * M / Mc
    cpu_total = n_restarts * (cpu_step * iters + t_lw)
    return {'config': 5, 'workload': '8-schools NCP, %d KLVI restarts x %d iters, M=%d bounds+PSIS'
            % (n_restarts, iters, M), 'gpu_s': dt, 'restarts_per_s': n_restarts / dt,
            'finite_khat': bool(np.all(np.isfinite(tab[:, 8]))),
            'cpu_s_estimated': cpu_total, 'cpu_ms_per_step': cpu_step * 1e3,
            'cpu_bounds_psis_s_per_restart': t_lw, 'speedup': cpu_total / dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--configs', default='1,2,4,5')
    ap.add_argument('--cpu-seconds', type=float, default=8.0)
    a = ap.parse_args()
    os.environ.setdefault('OMP_NUM_THREADS', '1')
    fns = {'1': config1, '2': config2, '4': config4, '5': config5}
    for c in a.configs.split(','):
        out = fns[c](a.cpu_seconds)
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
