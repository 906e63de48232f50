"""Parity at the exact benchmark configurations (BASELINE.json configs 3 and 4).

* config 3 (the metric): mean-field Gaussian KLVI on isogauss D = 10 000 at
  N = 128 (metric text) and N = 256 (config text):
  - one estimator call on the reference's numpy stream (RandomState(0),
    vb.py:49, 57) vs the oracle: <= 1e-10 relative;
  - bench.py's own run -- DeviceRun, Philox seed 0 stream 1, window 10, lr .01,
    eps .1, lambda0 = [0, 1], a 5-step warm-up launch then launches of up to
    256 steps (sep_kernel's chunk) -- vs the oracle's adagrad loop
    (vb.py:345-389 restated) fed with the C-oracle Philox draws: <= 1e-7
    relative on values, history rows and the final lambda, over >= 130 steps,
    crossing a 256-step chunk boundary at N = 128.
* config 4: full-rank t D = 512, df = 100, CHIVI alpha = 2, N = 128 on
  corr_gauss, 20 adagrad steps (Philox draws) vs fullrank_oracle (scipy sqrtm +
  solve_sylvester, the reference's linear algebra): <= 1e-7 of the largest entry.
"""
import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]

D = 10_000


def _close(a, b, rtol):
    a, b = np.asarray(a), np.asarray(b)
    scale = max(1.0, float(np.max(np.abs(b))))
    err = float(np.max(np.abs(a - b))) / scale
    assert err <= rtol, 'max scaled error %.3e > %.1e' % (err, rtol)


@pytest.mark.parametrize('N', [128, 256])
def test_config3_klvi_call_numpy_stream(N):
    from viabel_amd import vb, targets
    from oracle import vb_oracle as vo
    fam = vb.mean_field_gaussian_variational_family(D, rng='numpy')
    ofam = vo.Family('gauss', D)
    obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
    rs = np.random.RandomState(11)
    for call in range(2):
        lam = np.concatenate([rs.randn(D) * 0.1, 1.0 + rs.randn(D) * 0.05])
        v, g = obj(lam)
        ov, og = vo.klvi_value_grad(ofam, 'isogauss', lam, N)
        assert abs(v - ov) <= 1e-10 * max(1.0, abs(ov)), (v, ov)
        _close(g, og, 1e-10)


def test_config3_short_launches():
    """The driver's shape (a 5-step warm-up launch, then 20-step launches; every
    launch of sep_kernel is followed by sep_values_kernel, which reduces the
    launch's per-step value partials).  Launches of 5, 20 x 5, 1, 24 and 25 steps
    against the oracle on the C-oracle Philox draws: values, history rows and
    lambda to 1e-7."""
    from viabel_amd import vb, targets
    from oracle import vb_oracle as vo, rng_oracle as ro
    N, W, LR, EPS = 128, 10, 0.01, 0.1
    chunks = [5, 20, 20, 20, 20, 20, 1, 24, 25]
    n_iters = sum(chunks)
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    run = vb.DeviceRun(obj, n_iters, init[None, :], window=W, learning_rate=LR, epsilon=EPS)
    done = 0
    for cs in chunks:
        run.advance_philox(cs, 0, 3, done)
        done += cs
    lam, hist, vals, smooth = run.result()
    ofam = vo.Family('gauss', D)
    step = [0]

    def f(l):
        eps = ro.noise(0, 3, step[0], N, D, 'gauss')
        step[0] += 1
        return vo.klvi_value_grad(ofam, 'isogauss', l, N, eps=eps)
    osm, ohist, ovals, _ = vo.adagrad_optimize(n_iters, f, init, window=W, learning_rate=LR,
                                               epsilon=EPS)
    np.testing.assert_allclose(vals[0], ovals, rtol=1e-7, atol=1e-7)
    _close(hist[0], ohist, 1e-7)
    _close(lam[0], ohist[-1], 1e-7)


@pytest.mark.parametrize('N,n_iters', [(128, 300), (256, 130)])
def test_config3_bench_run_philox_trajectory(N, n_iters):
    from viabel_amd import vb, targets
    from oracle import vb_oracle as vo, rng_oracle as ro
    W, LR, EPS = 10, 0.01, 0.1
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    run = vb.DeviceRun(obj, n_iters, init[None, :], window=W, learning_rate=LR, epsilon=EPS)
    seed, strm = 0, 1
    run.advance_philox(5, seed, strm, 0)             # bench.py's warm-up launch
    done = 5
    while done < n_iters:                            # then launches of <= 256 steps
        cs = min(256, n_iters - done)
        run.advance_philox(cs, seed, strm, done)
        done += cs
    lam, hist, vals, smooth = run.result()

    ofam = vo.Family('gauss', D)
    step = [0]

    def f(l):
        eps = ro.noise(seed, strm, step[0], N, D, 'gauss')
        step[0] += 1
        return vo.klvi_value_grad(ofam, 'isogauss', l, N, eps=eps)
    osm, ohist, ovals, _ = vo.adagrad_optimize(n_iters, f, init, window=W, learning_rate=LR,
                                               epsilon=EPS)
    assert hist.shape[1:] == ohist.shape
    np.testing.assert_allclose(vals[0], ovals, rtol=1e-7, atol=1e-7)
    _close(hist[0], ohist, 1e-7)
    _close(lam[0], ohist[-1], 1e-7)
    _close(smooth[0], osm, 1e-7)


def test_config4_chivi_trajectory():
    from viabel_amd import vb, targets
    from oracle import fullrank_oracle as fo, rng_oracle as ro, vb_oracle as vo
    Dm, N, n_iters = 512, 128, 20
    rs = np.random.RandomState(4)
    tri = np.tril_indices(Dm)
    free = rs.randn(len(tri[0])) * 0.01
    free[tri[0] == tri[1]] = rs.randn(Dm) * 0.1
    lam0 = np.concatenate([np.zeros(Dm), free])
    fam = vb.t_variational_family(Dm, 100.0, rng='philox')
    obj = vb.black_box_chivi(2.0, fam, targets.corr_gauss(Dm), N)
    run = vb.DeviceRun(obj, n_iters, lam0)
    run.advance_philox(n_iters, 0, 1, 0)
    lam, hist, vals, smooth = run.result()

    ofam = fo.FullRankT(Dm, 100.0)
    otgt = fo.target_fn('corr_gauss', Dm)
    step = [0]

    def f(l):
        draws = ro.fr_noise(0, 1, step[0], N, Dm, 100.0)
        step[0] += 1
        return fo.chivi_value_grad(ofam, otgt, l, N, 2.0, draws=draws)
    osm, ohist, ovals, _ = vo.adagrad_optimize(n_iters, f, lam0)
    _close(vals[0], ovals, 1e-7)
    _close(hist[0], ohist, 1e-7)
    _close(lam[0], ohist[-1], 1e-7)
