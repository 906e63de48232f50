"""GPU parity of the convergence diagnostics (functions.py:8-77 -> vb_rhat,
vb_iterate_average) and the IA optimisers (vb.py:392-712 -> vb_run with the
RMSProp-IA / Adam-IA updates) against oracle/functions_oracle.py.
Tolerances: diagnostics 1e-12 relative; optimiser histories / values 1e-7
relative to the largest entry (numpy-stream parity mode)."""
import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]


def _close(a, b, rtol):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    assert a.shape == b.shape, (a.shape, b.shape)
    scale = max(1.0, float(np.max(np.abs(b)))) if b.size else 1.0
    err = float(np.max(np.abs(a - b))) / scale if b.size else 0.0
    assert err <= rtol, 'max scaled error %.3e > %.1e' % (err, rtol)


@pytest.mark.parametrize('nc,n,K,warmup', [(2, 1000, 3, 500), (4, 600, 20, 0), (1, 64, 5, 10),
                                           (3, 2001, 2, 1)])
def test_compute_R_hat(nc, n, K, warmup):
    from viabel_amd import functions
    from oracle import functions_oracle as fo
    rs = np.random.RandomState(nc + n)
    chains = rs.randn(nc, n, K).cumsum(axis=1) * 0.01 + rs.randn(nc, 1, K)
    v, r = functions.compute_R_hat(chains, warmup=warmup)
    ov, orr = fo.compute_R_hat(chains, warmup=warmup)
    np.testing.assert_allclose(v, ov, rtol=1e-12)
    np.testing.assert_allclose(r, orr, rtol=1e-12)


def test_compute_R_hat_odd_raises():
    from viabel_amd import functions
    with pytest.raises(ValueError):
        functions.compute_R_hat(np.zeros((2, 101, 1)), warmup=0)


def test_windows_halfway_and_averaging():
    from viabel_amd import functions
    from oracle import functions_oracle as fo
    rs = np.random.RandomState(3)
    chains = rs.randn(4, 3000, 6).cumsum(axis=1) * 0.02
    _close(functions.compute_R_hat_adaptive_numpy(chains, 500),
           fo.compute_R_hat_adaptive_numpy(chains, 500), 1e-12)
    _close(functions.compute_R_hat_halfway(chains, 100, 200),
           fo.compute_R_hat_halfway(chains, 100, 200), 1e-12)
    it, last = functions.stochastic_iterate_averaging(chains[1, :, 2:5], 700)
    oit, olast = fo.stochastic_iterate_averaging(chains[1, :, 2:5], 700)
    _close(it, oit, 1e-13)
    _close(last, olast, 1e-13)
    with pytest.raises(TypeError, match='Start of stationary'):
        functions.stochastic_iterate_averaging(chains[0], 3000)


def _check_ia(res, ores, rtol=1e-7):
    lam, chains, means, sigmas, vals, lns, log = res
    olam, ochains, omeans, osigmas, ovals, olns, olog = ores
    _close(chains, ochains, rtol)
    _close(vals, ovals, rtol)
    _close(lam, olam, rtol)
    for k in ('start_avg_mean_iters', 'start_avg_sigma_iters'):
        assert log[k] == olog[k]
    for k in ('r_hat_mean', 'r_hat_sigma', 'r_hat_mean_halfway', 'r_hat_sigma_halfway'):
        _close(log[k], olog[k], 1e-6)
    for a, b in zip(means, omeans):
        _close(a, b, rtol)
    for a, b in zip(sigmas, osigmas):
        _close(a, b, rtol)


@pytest.mark.parametrize('which', ['rmsprop', 'adam'])
@pytest.mark.parametrize('objective', ['klvi', 'chivi'])
def test_ia_optimizer_numpy_stream(which, objective):
    """3 chains x 600 iterations, R-hat windows of 100: KLVI on 8-schools NCP with
    mean-field t(40); CHIVI on the mixture with mean-field Gaussian."""
    from viabel_amd import vb, targets
    from oracle import vb_oracle as vo, functions_oracle as fo
    N, n_iters = 20, 600
    if objective == 'klvi':
        D = 10
        fam = vb.mean_field_t_variational_family(D, 40.0, rng='numpy')
        ofam = vo.Family('t', D, 40.0)
        obj = vb.black_box_klvi(fam, targets.eight_schools_ncp(), N)
        ofn = lambda lam: vo.klvi_value_grad(ofam, 'eight_schools_ncp', lam, N)
    else:
        # CHIVI on 8-schools with t draws diverges (tau overflows) in the oracle too
        D = 3
        fam = vb.mean_field_gaussian_variational_family(D, rng='numpy')
        ofam = vo.Family('gauss', D)
        obj = vb.black_box_chivi(2.0, fam, targets.mixture(D), N)
        ofn = lambda lam: vo.chivi_value_grad(ofam, 'mixture', lam, N, 2.0)
    init = np.zeros(2 * D)
    kw = dict(window=3, learning_rate=.01, rhat_window=100, n_optimisers=3, tail_avg_iters=400,
              learning_rate_end=.001)
    dev = getattr(vb, which + '_IA_optimize_with_rhat')
    ora = getattr(fo, which + '_IA_optimize_with_rhat')
    res = dev(n_iters, obj, init, D, **kw)
    ores = ora(n_iters, ofn, init, D, **kw)
    assert res[1].shape == (3, 300, 2 * D)        # history capped at 100 * window
    _check_ia(res, ores)


def test_ia_optimizer_fullrank():
    from viabel_amd import vb, targets
    from oracle import fullrank_oracle as fr, functions_oracle as fo
    D, N, n_iters = 4, 30, 400
    fam = vb.t_variational_family(D, 100.0, rng='numpy')
    ofam = fr.FullRankT(D, 100.0)
    otgt = fr.target_fn('corr_gauss', D)
    obj = vb.black_box_klvi(fam, targets.corr_gauss(D), N)
    ofn = lambda lam: fr.klvi_value_grad(ofam, otgt, lam, N)
    init = np.zeros(fam.var_param_dim)
    kw = dict(window=500, learning_rate=.01, rhat_window=100, n_optimisers=2, tail_avg_iters=100)
    _check_ia(vb.rmsprop_IA_optimize_with_rhat(n_iters, obj, init, D, **kw),
              fo.rmsprop_IA_optimize_with_rhat(n_iters, ofn, init, D, **kw))


def test_ia_optimizer_philox_chains():
    from viabel_amd import vb, targets
    D = 10
    fam = vb.mean_field_t_variational_family(D, 40.0, rng='philox')
    obj = vb.black_box_klvi(fam, targets.eight_schools_ncp(), 50)
    res = vb.rmsprop_IA_optimize_with_rhat(2000, obj, np.zeros(2 * D), D, n_optimisers=4,
                                           tail_avg_iters=500)
    lam, chains, means, sigmas, vals, _, log = res
    assert chains.shape == (4, 2000, 2 * D)
    assert np.all(np.isfinite(chains)) and np.all(np.isfinite(vals))
    assert log['r_hat_mean'].shape == (4, D)
    assert len(means) == 4 and means[0].shape[1] == D


def _foreign(kind, D, N, log_norm=False):
    """A caller-supplied (Python) objective over the oracle's own stream; with
    log_norm it returns (value, grad, log_norm) like has_log_norm objectives."""
    from oracle import vb_oracle as vo
    ofam = vo.Family(kind, D, 40.0 if kind == 't' else None)
    tgt = 'eight_schools_ncp' if kind == 't' else 'mixture'

    def f(lam):
        v, g = vo.klvi_value_grad(ofam, tgt, lam, N)
        if log_norm:
            return v, g, 0.05 * float(np.sum(lam ** 2)) - 0.3
        return v, g
    return f


@pytest.mark.parametrize('which', ['rmsprop', 'adam'])
@pytest.mark.parametrize('log_norm', [False, True])
def test_ia_optimizer_foreign_objective(which, log_norm):
    """A Python objective with the device IA update (vb_ia_update): same chains,
    values, log norms and averages as the reference loop (vb.py:392-712)."""
    from viabel_amd import vb
    from oracle import functions_oracle as fo
    D, N, n_iters = 10, 20, 500
    init = np.zeros(2 * D)
    kw = dict(window=3, learning_rate=.01, rhat_window=100, n_optimisers=2, tail_avg_iters=300,
              learning_rate_end=.001, has_log_norm=log_norm)
    res = getattr(vb, which + '_IA_optimize_with_rhat')(n_iters, _foreign('t', D, N, log_norm),
                                                         init, D, **kw)
    ores = getattr(fo, which + '_IA_optimize_with_rhat')(n_iters, _foreign('t', D, N, log_norm),
                                                          init, D, **kw)
    assert res[1].shape == (2, 300, 2 * D)
    _check_ia(res, ores, 1e-10)
    _close(res[5], ores[5], 1e-14)


@pytest.mark.parametrize('native', [False, True])
@pytest.mark.parametrize('log_norm', [False, True])
def test_rmsprop_avg_grad_norm(native, log_norm):
    """avg_grad_norm=True: every coordinate scaled by the scalar sum of squared
    gradients (or exp(log_norm)), vb.py:443-451."""
    from viabel_amd import vb, targets
    from oracle import functions_oracle as fo
    if native and log_norm:
        pytest.skip('native objectives return (value, grad)')
    D, N, n_iters = 3, 30, 400
    if native:
        fam = vb.mean_field_gaussian_variational_family(D, rng='numpy')
        obj = vb.black_box_klvi(fam, targets.mixture(D), N)
    else:
        obj = _foreign('gauss', D, N, log_norm)
    init = np.full(2 * D, 0.1)
    kw = dict(window=5, learning_rate=.02, rhat_window=100, n_optimisers=2, tail_avg_iters=200,
              has_log_norm=log_norm)
    res = vb.rmsprop_IA_optimize_with_rhat(n_iters, obj, init, D, avg_grad_norm=True, **kw)
    ores = fo.rmsprop_IA_optimize_with_rhat(n_iters, _foreign('gauss', D, N, log_norm), init, D,
                                            avg_grad_norm=True, **kw)
    _check_ia(res, ores, 1e-10)


def test_adagrad_foreign_has_log_norm():
    """adagrad_optimize(has_log_norm=True): window gradients scaled by
    exp(min log_norm - log_norm_j) (vb.py:365-373) in vb_adagrad_update_scaled."""
    from viabel_amd import vb
    from oracle import vb_oracle as vo
    D, N = 10, 25
    init = np.zeros(2 * D)
    res = vb.adagrad_optimize(200, _foreign('t', D, N, True), init, has_log_norm=True, window=7,
                              learning_rate=.05, learning_rate_end=.01)
    ores = vo.adagrad_optimize(200, _foreign('t', D, N, True), init, window=7, learning_rate=.05,
                               learning_rate_end=.01, has_log_norm=True)
    for a, b in zip(res, ores):
        _close(a, b, 1e-12)
