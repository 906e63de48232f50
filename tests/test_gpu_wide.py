"""GPU parity of the materialised mean-field path (D > 16 with CHIVI or a
non-separable target, and the IA optimisers at D > 16) against the oracle on
identical numpy-stream draws.  Tolerances as tests/test_gpu_vb.py: single
calls 1e-10 relative, trajectories 1e-7."""
import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]

FAMS = [('gauss', None), ('t', 40.0)]


def _mods():
    from viabel_amd import vb, targets
    from oracle import vb_oracle
    return vb, targets, vb_oracle


def _family(vb, kind, df, D):
    if kind == 'gauss':
        return vb.mean_field_gaussian_variational_family(D, rng='numpy')
    return vb.mean_field_t_variational_family(D, df, rng='numpy')


def _target(targets, name, D):
    return {'isogauss': targets.isogauss, 'mixture': targets.mixture,
            'funnel': targets.funnel}[name](D)


def _lam(D, seed):
    rs = np.random.RandomState(seed)
    return np.concatenate([rs.randn(D) * 0.3, rs.randn(D) * 0.2 - 0.5])


def _close(a, b, rtol):
    a, b = np.asarray(a), np.asarray(b)
    scale = max(1.0, float(np.max(np.abs(b))))
    err = float(np.max(np.abs(a - b))) / scale
    assert err <= rtol, 'max scaled error %.3e > %.1e' % (err, rtol)


@pytest.mark.parametrize('kind,df', FAMS)
@pytest.mark.parametrize('target,D', [('isogauss', 17), ('mixture', 300), ('funnel', 40),
                                      ('funnel', 1000), ('isogauss', 700), ('mixture', 1001)])
@pytest.mark.parametrize('alpha', [2.0, 1.5])
def test_chivi_wide_numpy_stream(kind, df, target, D, alpha):
    vb, targets, vo = _mods()
    fam = _family(vb, kind, df, D)
    ofam = vo.Family(kind, D, df)
    obj = vb.black_box_chivi(alpha, fam, _target(targets, target, D), 64)
    for call in range(2):
        lam = _lam(D, call)
        np.random.seed(10 + call)
        v, g = obj(lam)
        np.random.seed(10 + call)
        ov, og = vo.chivi_value_grad(ofam, target, lam, 64, alpha)
        assert abs(v - ov) <= 1e-10 * max(1.0, abs(ov))
        _close(g, og, 1e-10)


@pytest.mark.parametrize('kind,df', FAMS)
@pytest.mark.parametrize('target,D', [('mixture', 1001), ('isogauss', 3000)])
def test_chivi_wide_philox_fused_rows(kind, df, target, D):
    """Fused per-row draw / target / log q kernel (separable targets, D >= 512):
    its in-register Philox draws equal the C oracle's, so CHIVI matches the
    oracle fed with rng_oracle noise."""
    vb, targets, vo = _mods()
    from oracle import rng_oracle as ro
    N = 96
    fam = (vb.mean_field_gaussian_variational_family(D, rng='philox') if kind == 'gauss'
           else vb.mean_field_t_variational_family(D, df, rng='philox'))
    ofam = vo.Family(kind, D, df)
    obj = vb.black_box_chivi(2.0, fam, _target(targets, target, D), N)
    for call in range(2):
        lam = _lam(D, 40 + call)
        # CHIVI keys each call's Philox draws with a seed from the global numpy
        # RNG (vb.py:258 draws its seed the same way), family stream, step 0
        np.random.seed(70 + call)
        seed = np.random.randint(2 ** 32)
        np.random.seed(70 + call)
        v, g = obj(lam)
        eps = ro.noise(seed, fam.stream, 0, N, D, kind, df or 0.0)
        ov, og = vo.chivi_value_grad(ofam, target, lam, N, 2.0, eps=eps)
        assert abs(v - ov) <= 1e-10 * max(1.0, abs(ov)), (v, ov)
        _close(g, og, 1e-9)


@pytest.mark.parametrize('kind,df', FAMS)
@pytest.mark.parametrize('D', [17, 500])
def test_klvi_funnel_wide(kind, df, D):
    vb, targets, vo = _mods()
    fam = _family(vb, kind, df, D)
    ofam = vo.Family(kind, D, df)
    obj = vb.black_box_klvi(fam, targets.funnel(D), 100)
    lam = _lam(D, 5)
    v, g = obj(lam)
    ov, og = vo.klvi_value_grad(ofam, 'funnel', lam, 100)
    assert abs(v - ov) <= 1e-10 * max(1.0, abs(ov))
    _close(g, og, 1e-10)


@pytest.mark.parametrize('objective,target', [('chivi', 'mixture'), ('klvi', 'funnel')])
def test_adagrad_wide_numpy_stream(objective, target):
    vb, targets, vo = _mods()
    D, N, n_iters = 33, 40, 120
    fam = _family(vb, 'gauss', None, D)
    ofam = vo.Family('gauss', D)
    tgt = _target(targets, target, D)
    lam0 = _lam(D, 1)
    if objective == 'chivi':
        obj = vb.black_box_chivi(2.0, fam, tgt, N)
        ofn = lambda lam: vo.chivi_value_grad(ofam, target, lam, N, 2.0)
    else:
        obj = vb.black_box_klvi(fam, tgt, N)
        ofn = lambda lam: vo.klvi_value_grad(ofam, target, lam, N)
    np.random.seed(4)
    sm, hist, vals, _ = vb.adagrad_optimize(n_iters, obj, lam0, learning_rate=.02)
    np.random.seed(4)
    osm, ohist, ovals = vo.adagrad_optimize(n_iters, ofn, lam0, learning_rate=.02)[:3]
    _close(vals, ovals, 1e-7)
    _close(hist, ohist, 1e-7)


@pytest.mark.parametrize('kind,df', FAMS)
def test_log_weights_funnel_wide(kind, df):
    vb, targets, vo = _mods()
    from viabel_amd import experiments
    D = 30
    fam = _family(vb, kind, df, D)
    ofam = vo.Family(kind, D, df)
    lam = _lam(D, 2)
    xs, lw = experiments.log_weights(targets.funnel(D), fam, lam, 2000)
    ox, olw = vo.log_weights(ofam, 'funnel', lam, 2000)
    _close(xs, ox, 1e-12)
    _close(lw, olw, 1e-10)


def test_rmsprop_ia_wide():
    vb, targets, vo = _mods()
    from oracle import functions_oracle as fo
    D, N = 20, 30
    fam = _family(vb, 'gauss', None, D)
    ofam = vo.Family('gauss', D)
    obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
    ofn = lambda lam: vo.klvi_value_grad(ofam, 'isogauss', lam, N)
    kw = dict(window=500, rhat_window=100, n_optimisers=2, tail_avg_iters=100)
    res = vb.rmsprop_IA_optimize_with_rhat(400, obj, np.zeros(2 * D), D, **kw)
    ores = fo.rmsprop_IA_optimize_with_rhat(400, ofn, np.zeros(2 * D), D, **kw)
    _close(res[1], ores[1], 1e-7)
    _close(res[4], ores[4], 1e-7)


@pytest.mark.parametrize('kind,df', FAMS)
def test_rmsprop_ia_wide_fused_rows(kind, df):
    """KLVI through the fused rows kernel (separable target, D >= 512) with the
    separate weights pass and no fused update (IA optimiser)."""
    vb, targets, vo = _mods()
    from oracle import functions_oracle as fo
    D, N = 601, 24
    fam = _family(vb, kind, df, D)
    ofam = vo.Family(kind, D, df)
    obj = vb.black_box_klvi(fam, targets.mixture(D), N)
    ofn = lambda lam: vo.klvi_value_grad(ofam, 'mixture', lam, N)
    kw = dict(window=100, rhat_window=50, n_optimisers=2, tail_avg_iters=50)
    res = vb.rmsprop_IA_optimize_with_rhat(100, obj, _lam(D, 9), D, **kw)
    ores = fo.rmsprop_IA_optimize_with_rhat(100, ofn, _lam(D, 9), D, **kw)
    _close(res[1], ores[1], 1e-7)
    _close(res[4], ores[4], 1e-7)


@pytest.mark.parametrize('kind,df', [('gauss', None), ('t', 40.0), ('t', 5.0)])
@pytest.mark.parametrize('target,D', [('isogauss', 6), ('mixture', 2000), ('funnel', 10),
                                      ('funnel', 40), ('isogauss', 17)])
def test_klvi_pd_numpy_stream(kind, df, target, D):
    """black_box_klvi_pd / _pd2 (vb.py:268-295) on every mean-field path."""
    vb, targets, vo = _mods()
    fam = _family(vb, kind, df, D)
    ofam = vo.Family(kind, D, df)
    for k, ctor in enumerate((vb.black_box_klvi_pd, vb.black_box_klvi_pd2)):
        obj = ctor(fam, _target(targets, target, D), 50)
        lam = _lam(D, 30 + k)
        v, g = obj(lam)
        ov, og = vo.klvi_pd_value_grad(ofam, target, lam, 50)
        assert abs(v - ov) <= 1e-10 * max(1.0, abs(ov)), (v, ov)
        _close(g, og, 1e-10)


def test_klvi_pd_adagrad_and_fullrank():
    vb, targets, vo = _mods()
    from oracle import fullrank_oracle as fr
    D = 300
    fam = _family(vb, 'gauss', None, D)
    ofam = vo.Family('gauss', D)
    obj = vb.black_box_klvi_pd(fam, targets.isogauss(D), 20)
    lam0 = _lam(D, 7)
    sm, hist, vals, _ = vb.adagrad_optimize(50, obj, lam0)
    osm, ohist, ovals = vo.adagrad_optimize(
        50, lambda lam: vo.klvi_pd_value_grad(ofam, 'isogauss', lam, 20), lam0)[:3]
    _close(vals, ovals, 1e-9)
    _close(hist, ohist, 1e-9)
    Dr = 7
    ffam = vb.t_variational_family(Dr, 100.0, rng='numpy')
    offam = fr.FullRankT(Dr, 100.0)
    rs = np.random.RandomState(2)
    lam = np.concatenate([rs.randn(Dr) * 0.2, rs.randn(Dr * (Dr + 1) // 2) * 0.05])
    v, g = vb.black_box_klvi_pd(ffam, targets.corr_gauss(Dr), 40)(lam)
    ov, og = fr.klvi_pd_value_grad(offam, fr.target_fn('corr_gauss', Dr), lam, 40)
    np.testing.assert_allclose(v, ov, rtol=1e-9)
    _close(g, og, 1e-8)


def test_big_window_and_many_wide_problems():
    """adagrad windows > 64 (materialised path, window in HBM) and several
    problems in one wide run match the oracle."""
    vb, targets, vo = _mods()
    D = 6
    fam = _family(vb, 'gauss', None, D)
    ofam = vo.Family('gauss', D)
    obj = vb.black_box_klvi(fam, targets.mixture(D), 20)
    lam0 = _lam(D, 3)
    res = vb.adagrad_optimize(120, obj, lam0, window=100, learning_rate=.05)
    ores = vo.adagrad_optimize(120, lambda l: vo.klvi_value_grad(ofam, 'mixture', l, 20), lam0,
                               window=100, learning_rate=.05)
    _close(res[1], ores[1], 1e-7)
    _close(res[2], ores[2], 1e-7)
    # three restarts of a wide CHIVI problem in one run (Philox streams 5, 6, 7)
    Dw = 30
    famw = vb.mean_field_gaussian_variational_family(Dw, rng='philox')
    objw = vb.black_box_chivi(2.0, famw, targets.funnel(Dw), 16)
    inits = np.stack([_lam(Dw, s) for s in range(3)])
    run = vb.DeviceRun(objw, 30, inits, learning_rate=.01)
    run.advance_philox(30, 9, 5, 0)
    lam, hist, vals, _ = run.result()
    assert np.all(np.isfinite(vals)) and vals.shape == (3, 30)
    for q in range(3):   # each problem equals a single-problem run on its own stream
        single = vb.DeviceRun(objw, 30, inits[q][None], learning_rate=.01)
        single.advance_philox(30, 9, 5 + q, 0)
        _close(single.result()[2][0], vals[q], 1e-12)
