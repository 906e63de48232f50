"""GPU parity of the full-rank Student-t family (t_variational_family,
viabel/vb.py:192-233) against oracle/fullrank_oracle.py on identical draws.

The oracle follows the reference's own linear algebra (scipy sqrtm, autograd's
solve_sylvester VJP, eigh-based multivariate_t_logpdf); the device uses one
eigendecomposition of Sigma per step.  Tolerances (per test): family helpers
1e-10 relative; estimator values and gradients 1e-8 relative to the largest
gradient entry (the north_star bar is 1e-5; eigensolver vs Schur sqrtm
differ at ~1e-12 x cond); adagrad trajectories 1e-7."""
import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]


def _mods():
    from viabel_amd import vb, targets
    from oracle import fullrank_oracle as fo, rng_oracle, vb_oracle
    return vb, targets, fo, rng_oracle, vb_oracle


def _lam(D, seed, scale=0.05):
    """Non-degenerate Sigma: distinct log-diagonal entries (the reference's CHIVI
    gradient through eigh is NaN at repeated eigenvalues)."""
    rs = np.random.RandomState(seed)
    tri = np.tril_indices(D)
    free = rs.randn(len(tri[0])) * scale
    free[tri[0] == tri[1]] = rs.randn(D) * 0.2
    return np.concatenate([rs.randn(D) * 0.3, free])


def _target(targets, name, D):
    return {'isogauss': lambda: targets.isogauss(D), 'mixture': lambda: targets.mixture(D),
            'funnel': lambda: targets.funnel(D), 'eight_schools_ncp': targets.eight_schools_ncp,
            'corr_gauss': lambda: targets.corr_gauss(D)}[name]()


def _close(a, b, rtol):
    a, b = np.asarray(a), np.asarray(b)
    scale = max(1.0, float(np.max(np.abs(b))))
    err = float(np.max(np.abs(a - b))) / scale
    assert err <= rtol, 'max scaled error %.3e > %.1e' % (err, rtol)


# ---------------------------------------------------------------------------
@pytest.mark.parametrize('D', [1, 5, 31, 32, 33, 100])
def test_moments_and_helpers(D):
    vb, targets, fo, _, _ = _mods()
    fam = vb.t_variational_family(D, 7.0)
    ofam = fo.FullRankT(D, 7.0)
    lam = _lam(D, D)
    mu, L, Sig = fo.unpack(lam, D)
    m, cov = fam.mean_and_cov(lam)
    _close(m, mu, 0)
    _close(cov, 7.0 / 5.0 * Sig, 1e-13)
    np.testing.assert_allclose(fam.entropy(lam), ofam.entropy(lam), rtol=1e-10, atol=1e-12)
    for p in (2, 4):
        np.testing.assert_allclose(fam.pth_moment(p, lam), ofam.pth_moment(p, lam), rtol=1e-10)
    x = np.random.RandomState(1).randn(50, D) + mu
    _close(fam.logdensity(x, lam), ofam.logdensity(x, lam), 1e-10)
    assert np.isscalar(fam.logdensity(x[0], lam)) or np.ndim(fam.logdensity(x[0], lam)) == 0
    assert fam.var_param_dim == ofam.var_param_dim


@pytest.mark.parametrize('D', [2, 17, 64])
def test_sample_numpy_stream(D):
    """sample() draws chisquare then randn from the family's RandomState(0) (vb.py:204-208)."""
    vb, _, fo, _, _ = _mods()
    fam = vb.t_variational_family(D, 100.0, rng='numpy')
    ofam = fo.FullRankT(D, 100.0)
    lam = _lam(D, 3)
    for n in (1, 40, 257):
        _close(fam.sample(lam, n), ofam.sample(lam, n), 1e-11)
    _close(fam.sample(lam, 33, seed=9), ofam.sample(lam, 33, seed=9), 1e-11)


@pytest.mark.parametrize('target,D', [('corr_gauss', 6), ('corr_gauss', 47), ('isogauss', 20),
                                      ('mixture', 9), ('funnel', 7), ('eight_schools_ncp', 10)])
@pytest.mark.parametrize('N', [1, 64, 200])
def test_klvi_call_numpy_stream(target, D, N):
    vb, targets, fo, _, _ = _mods()
    fam = vb.t_variational_family(D, 100.0, rng='numpy')
    ofam = fo.FullRankT(D, 100.0)
    otgt = fo.target_fn(target, D)
    obj = vb.black_box_klvi(fam, _target(targets, target, D), N)
    for call in range(2):
        lam = _lam(D, 10 + call)
        v, g = obj(lam)
        ov, og = fo.klvi_value_grad(ofam, otgt, lam, N)
        np.testing.assert_allclose(v, ov, rtol=1e-10, atol=1e-10)
        _close(g, og, 1e-8)


@pytest.mark.parametrize('target,D', [('corr_gauss', 8), ('corr_gauss', 40), ('isogauss', 5),
                                      ('funnel', 4)])
@pytest.mark.parametrize('alpha', [2.0, 1.5])
def test_chivi_call_numpy_stream(target, D, alpha):
    vb, targets, fo, _, _ = _mods()
    fam = vb.t_variational_family(D, 100.0, rng='numpy')
    ofam = fo.FullRankT(D, 100.0)
    otgt = fo.target_fn(target, D)
    obj = vb.black_box_chivi(alpha, fam, _target(targets, target, D), 128)
    for call in range(2):
        lam = _lam(D, 20 + call)
        np.random.seed(100 + call)
        v, g = obj(lam)
        np.random.seed(100 + call)
        ov, og = fo.chivi_value_grad(ofam, otgt, lam, 128, alpha)
        np.testing.assert_allclose(v, ov, rtol=1e-9)
        _close(g, og, 1e-8)


def test_config4_chivi_call():
    """D = 512, df = 100, CHIVI N = 128 on corr_gauss,
    lambda0 = [0, log-diag 0.1 randn, off-diag 0.01 randn] (RandomState(4))."""
    vb, targets, fo, _, _ = _mods()
    D = 512
    rs = np.random.RandomState(4)
    tri = np.tril_indices(D)
    free = rs.randn(len(tri[0])) * 0.01
    free[tri[0] == tri[1]] = rs.randn(D) * 0.1
    lam = np.concatenate([np.zeros(D), free])
    fam = vb.t_variational_family(D, 100.0, rng='numpy')
    ofam = fo.FullRankT(D, 100.0)
    obj = vb.black_box_chivi(2.0, fam, targets.corr_gauss(D), 128)
    np.random.seed(7)
    v, g = obj(lam)
    np.random.seed(7)
    ov, og = fo.chivi_value_grad(ofam, fo.target_fn('corr_gauss', D), lam, 128, 2.0)
    np.testing.assert_allclose(v, ov, rtol=1e-9)
    _close(g, og, 1e-7)


@pytest.mark.parametrize('D', [3, 16, 65])
def test_philox_noise_equals_c_oracle(D):
    """In-kernel draws: z = normal pairs (purpose 0), s from the reserved pair."""
    vb, targets, fo, ro, _ = _mods()
    fam = vb.t_variational_family(D, 100.0, rng='philox')
    ofam = fo.FullRankT(D, 100.0)
    lam = _lam(D, 5)
    stream, step = fam.stream, fam.step
    x = fam.sample(lam, 300)
    s, z = ro.fr_noise(0, stream, step, 300, D, 100.0)
    _close(x, ofam.transform(lam, s, z), 1e-11)
    # the estimator consumes the same counters
    obj = vb.black_box_klvi(fam, targets.corr_gauss(D), 64)
    stream, step = fam.stream, fam.step
    v, g = obj(lam)
    s, z = ro.fr_noise(0, stream, step, 64, D, 100.0)
    ov, og = fo.klvi_value_grad(ofam, fo.target_fn('corr_gauss', D), lam, 64, draws=(s, z))
    np.testing.assert_allclose(v, ov, rtol=1e-10)
    _close(g, og, 1e-8)


@pytest.mark.parametrize('objective', ['klvi', 'chivi'])
@pytest.mark.parametrize('lr_end', [None, 0.002])
def test_adagrad_trajectory_numpy_stream(objective, lr_end):
    vb, targets, fo, _, vo = _mods()
    D, N, n_iters = 9, 50, 60
    fam = vb.t_variational_family(D, 100.0, rng='numpy')
    ofam = fo.FullRankT(D, 100.0)
    otgt = fo.target_fn('corr_gauss', D)
    tgt = targets.corr_gauss(D)
    lam0 = _lam(D, 2)
    if objective == 'klvi':
        obj = vb.black_box_klvi(fam, tgt, N)
        ofn = lambda lam: fo.klvi_value_grad(ofam, otgt, lam, N)
    else:
        obj = vb.black_box_chivi(2.0, fam, tgt, N)
        ofn = lambda lam: fo.chivi_value_grad(ofam, otgt, lam, N, 2.0)
    np.random.seed(3)
    sm, hist, vals, _ = vb.adagrad_optimize(n_iters, obj, lam0, learning_rate=.05,
                                            learning_rate_end=lr_end)
    np.random.seed(3)
    osm, ohist, ovals = vo.adagrad_optimize(n_iters, ofn, lam0, learning_rate=.05,
                                            learning_rate_end=lr_end)[:3]
    _close(vals, ovals, 1e-7)
    _close(hist, ohist, 1e-7)
    _close(sm, osm, 1e-7)


@pytest.mark.parametrize('target,D', [('corr_gauss', 12), ('mixture', 3)])
def test_log_weights(target, D):
    vb, targets, fo, _, _ = _mods()
    from viabel_amd import experiments
    fam = vb.t_variational_family(D, 100.0, rng='numpy')
    ofam = fo.FullRankT(D, 100.0)
    lam = _lam(D, 8)
    xs, lw = experiments.log_weights(_target(targets, target, D), fam, lam, 500)
    ox = ofam.sample(lam, 500)
    olp, _ = fo.target_fn(target, D)(ox)
    _close(xs, ox, 1e-11)
    _close(lw, olp - ofam.logdensity(ox, lam), 1e-9)


def test_target_corr_gauss_device():
    _, targets, fo, _, _ = _mods()
    D = 70
    t = targets.corr_gauss(D)
    x = np.random.RandomState(0).randn(33, D)
    lp, g = t.logdensity_and_grad(x)
    olp, og = fo.target_fn('corr_gauss', D)(x)
    _close(lp, olp, 1e-12)
    _close(g, og, 1e-12)


def test_errors():
    vb, targets, _, _, _ = _mods()
    with pytest.raises(ValueError, match='df must be greater than 2'):
        vb.t_variational_family(3, 2.0)
    fam = vb.mean_field_gaussian_variational_family(4)
    with pytest.raises(NotImplementedError):
        vb.black_box_klvi(fam, targets.corr_gauss(4), 10)(np.zeros(8))
    ft = vb.t_variational_family(4, 3.5)
    with pytest.raises(ValueError, match='df must be greater than p'):
        ft.pth_moment(4, np.zeros(ft.var_param_dim))


# ---------------------------------------------------------------------------
@pytest.mark.parametrize('objective', ['klvi', 'chivi', 'klvi_pd'])
@pytest.mark.parametrize('target,D', [('corr_gauss', 40), ('corr_gauss', 64), ('funnel', 33)])
def test_fused_philox_steps_across_advances(objective, target, D):
    """The fused full-rank step (Philox draws, adagrad in the last kernel, which
    prepares the next step's L, draws and Z power step; vb_fr.hip fr_value_grad):
    advances of 7, 1 and 5 steps -- ready steps, the first (unprepared) step of
    each advance, a one-step advance, a foreign root in between (log weights at
    another lambda clears the prepared state) -- against the oracle's adagrad on
    the C oracle's draws, step by step."""
    vb, targets, fo, ro, vo = _mods()
    N, n_iters = 24, 13
    lam0 = _lam(D, 7)
    fam = vb.t_variational_family(D, 30.0, rng='philox')
    tgt = _target(targets, target, D)
    if objective == 'klvi':
        obj = vb.black_box_klvi(fam, tgt, N)
    elif objective == 'chivi':
        obj = vb.black_box_chivi(2.0, fam, tgt, N)
    else:
        obj = vb.black_box_klvi_pd(fam, tgt, N)
    run = vb.DeviceRun(obj, n_iters, lam0, learning_rate=0.02)
    run.advance_philox(7, 3, 5, 0)
    run.advance_philox(1, 3, 5, 7)
    from viabel_amd import experiments
    experiments.log_weights(tgt, fam, _lam(D, 8), 64)          # another root on the workspace
    run.advance_philox(5, 3, 5, 8)
    lam, hist, vals, _ = run.result()

    ofam = fo.FullRankT(D, 30.0)
    otgt = fo.target_fn(target, D)
    step = [0]

    def f(l):
        draws = ro.fr_noise(3, 5, step[0], N, D, 30.0)
        step[0] += 1
        if objective == 'klvi':
            return fo.klvi_value_grad(ofam, otgt, l, N, draws=draws)
        if objective == 'chivi':
            return fo.chivi_value_grad(ofam, otgt, l, N, 2.0, draws=draws)
        return fo.klvi_pd_value_grad(ofam, otgt, l, N, draws=draws)
    osm, ohist, ovals, _ = vo.adagrad_optimize(n_iters, f, lam0, learning_rate=0.02)
    _close(vals[0], ovals, 1e-7)
    _close(hist[0], ohist, 1e-7)
    _close(lam[0], ohist[-1], 1e-7)


def test_newton_schulz_retry_when_the_learnt_count_is_short(monkeypatch):
    """Warm Newton-Schulz roots launch exactly the learnt iteration count; a step
    that needs more makes the advance restore its snapshot (lambda, adagrad
    window) and run again with a larger count (vb_capi.hip vb_run_advance,
    vb_fr.hip fr_info).  Forced here by starting warm roots at 3 iterations: the
    retry counter shows the rerun happened, the trajectory equals the unforced
    run's bit for bit and the oracle's to 1e-7."""
    vb, targets, fo, ro, vo = _mods()
    D, N, n_iters = 64, 16, 9
    lam0 = _lam(D, 11)

    def device_run():
        fam = vb.t_variational_family(D, 30.0, rng='philox')
        obj = vb.black_box_chivi(2.0, fam, targets.corr_gauss(D), N)
        run = vb.DeviceRun(obj, n_iters, lam0, learning_rate=0.02)
        run.advance_philox(6, 2, 4, 0)
        run.advance_philox(3, 2, 4, 6)
        return run.fr_retries(), run.result()

    # the unforced run: warm roots start from the default count
    n_plain, (lam_p, hist_p, vals_p, _) = device_run()
    monkeypatch.setenv('VIABEL_AMD_FR_NS_START', '3')
    retries, (lam, hist, vals, _) = device_run()
    assert retries > 0, 'the forced short count did not make an advance run again'
    # the rerun restores lambda, the window AND the warm state (previous root,
    # power vectors, schedule block): it is the run that would have happened
    # with the larger count, bit for bit (iterations past convergence are
    # skipped on the device, so the launched count does not change the bits)
    assert np.array_equal(vals[0], vals_p[0]), np.max(np.abs(vals[0] - vals_p[0]))
    assert np.array_equal(hist[0], hist_p[0]), np.max(np.abs(hist[0] - hist_p[0]))
    assert np.array_equal(lam[0], lam_p[0])
    ofam = fo.FullRankT(D, 30.0)
    otgt = fo.target_fn('corr_gauss', D)
    step = [0]

    def f(l):
        draws = ro.fr_noise(2, 4, step[0], N, D, 30.0)
        step[0] += 1
        return fo.chivi_value_grad(ofam, otgt, l, N, 2.0, draws=draws)
    osm, ohist, ovals, _ = vo.adagrad_optimize(n_iters, f, lam0, learning_rate=0.02)
    _close(vals[0], ovals, 1e-7)
    _close(hist[0], ohist, 1e-7)
    _close(lam[0], ohist[-1], 1e-7)


def test_retries_over_many_short_advances(monkeypatch):
    """Reruns are counted per advance (vb_capi.hip vb_run_advance): a run
    advanced one step at a time under a forced short Newton-Schulz count never
    fails for the reruns of earlier advances, and every advance that reran leaves
    the trajectory of the unforced run, bit for bit."""
    vb, targets, fo, ro, vo = _mods()
    D, N, n_iters = 64, 16, 24
    lam0 = _lam(D, 12)

    def device_run():
        fam = vb.t_variational_family(D, 30.0, rng='philox')
        obj = vb.black_box_chivi(2.0, fam, targets.corr_gauss(D), N)
        run = vb.DeviceRun(obj, n_iters, lam0, learning_rate=0.02)
        for k in range(n_iters):
            run.advance_philox(1, 2, 5, k)
        return run.fr_retries(), run.result()

    _, (lam_p, hist_p, vals_p, _) = device_run()
    monkeypatch.setenv('VIABEL_AMD_FR_NS_START', '3')
    retries, (lam, hist, vals, _) = device_run()
    assert retries > 0
    assert np.array_equal(vals[0], vals_p[0]), np.max(np.abs(vals[0] - vals_p[0]))
    assert np.array_equal(hist[0], hist_p[0])
    assert np.array_equal(lam[0], lam_p[0])


def test_ill_conditioned_sigma_trajectory():
    """Warm PCG steps stop at a relative residual of 1e-8, tightened by kappa / 2
    once the preconditioned condition number kappa = (2 + k + 1/k) / 4 (k =
    cond(S)) passes 2 (vb_fr.hip fr_sched_kernel, FrSched::ee_scale).  Sigma with
    cond ~1e4 (log-diagonal of L spread over [-2.3, 2.3]: k ~ 100, kappa ~ 25):
    the adagrad trajectory still equals the oracle's (scipy sqrtm +
    solve_sylvester) to 1e-7."""
    vb, targets, fo, ro, vo = _mods()
    D, N, n_iters = 64, 32, 12
    rs = np.random.RandomState(21)
    tri = np.tril_indices(D)
    free = rs.randn(len(tri[0])) * 0.01
    free[tri[0] == tri[1]] = np.linspace(-2.3, 2.3, D)[rs.permutation(D)]
    lam0 = np.concatenate([rs.randn(D) * 0.3, free])
    _, _, Sig = fo.unpack(lam0, D)
    ev = np.linalg.eigvalsh(Sig)
    assert ev[-1] / ev[0] > 5e3
    fam = vb.t_variational_family(D, 30.0, rng='philox')
    obj = vb.black_box_chivi(2.0, fam, targets.corr_gauss(D), N)
    run = vb.DeviceRun(obj, n_iters, lam0, learning_rate=0.01)
    run.advance_philox(8, 6, 2, 0)
    run.advance_philox(4, 6, 2, 8)
    lam, hist, vals, _ = run.result()
    ofam = fo.FullRankT(D, 30.0)
    otgt = fo.target_fn('corr_gauss', D)
    step = [0]

    def f(l):
        draws = ro.fr_noise(6, 2, step[0], N, D, 30.0)
        step[0] += 1
        return fo.chivi_value_grad(ofam, otgt, l, N, 2.0, draws=draws)
    osm, ohist, ovals, _ = vo.adagrad_optimize(n_iters, f, lam0, learning_rate=0.01)
    _close(vals[0], ovals, 1e-7)
    _close(hist[0], ohist, 1e-7)
    _close(lam[0], ohist[-1], 1e-7)


@pytest.mark.parametrize('objective', ['klvi', 'chivi'])
def test_ill_conditioned_single_call(objective):
    """A single value-and-gradient call at cond(Sigma) ~1e4 (a cold root, no run):
    the call runs again with larger Newton-Schulz / PCG counts until the device
    status is clean (vb_capi.hip, vb_fr.hip fr_info), and matches the oracle on
    the reference's numpy stream."""
    vb, targets, fo, _, _ = _mods()
    D, N = 48, 64
    rs = np.random.RandomState(5)
    tri = np.tril_indices(D)
    free = rs.randn(len(tri[0])) * 0.01
    free[tri[0] == tri[1]] = np.linspace(-2.3, 2.3, D)[rs.permutation(D)]
    lam = np.concatenate([rs.randn(D) * 0.3, free])
    fam = vb.t_variational_family(D, 30.0, rng='numpy')
    ofam = fo.FullRankT(D, 30.0)
    otgt = fo.target_fn('corr_gauss', D)
    if objective == 'klvi':
        v, g = vb.black_box_klvi(fam, targets.corr_gauss(D), N)(lam)
        ov, og = fo.klvi_value_grad(ofam, otgt, lam, N)
    else:
        np.random.seed(3)
        v, g = vb.black_box_chivi(2.0, fam, targets.corr_gauss(D), N)(lam)
        np.random.seed(3)
        ov, og = fo.chivi_value_grad(ofam, otgt, lam, N, 2.0)
    np.testing.assert_allclose(v, ov, rtol=1e-9)
    _close(g, og, 1e-7)


_EPI = '''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from viabel_amd import vb, targets
Dm = 512
rs = np.random.RandomState(4)
tri = np.tril_indices(Dm)
free = rs.randn(len(tri[0])) * 0.01
free[tri[0] == tri[1]] = rs.randn(Dm) * 0.1
lam0 = np.concatenate([np.zeros(Dm), free])
fam = vb.t_variational_family(Dm, 100.0, rng='philox')
obj = vb.black_box_chivi(2.0, fam, targets.corr_gauss(Dm), 128)
run = vb.DeviceRun(obj, 30, lam0, window=10, learning_rate=0.01, epsilon=0.1)
run.advance_philox(30, 0, 1, 0)
lam, hist, vals, _ = run.result()
np.savez(sys.argv[2], lam=lam, vals=vals)
'''


def test_exact_epilogue_kernels_equal_the_generic_kernel(tmp_path):
    """The GEMM kernels compiled for exact epilogue feature sets
    against the generic kernel (VIABEL_AMD_GEMM_EPI_EXACT=0, read once per process:
    child processes): 30 config-4 steps agree to rounding (the two compilations
    contract a few multiply-adds differently: ~1 ulp per step, 6e-16 absolute
    after 30 steps; bar 1e-12 absolute, 1e-9 relative)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for mode in ('0', '1'):
        f = str(tmp_path / ('e%s.npz' % mode))
        env = dict(os.environ, VIABEL_AMD_GEMM_EPI_EXACT=mode)
        r = subprocess.run([sys.executable, '-c', _EPI, root, f], env=env, capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        res[mode] = np.load(f)
    for key in ('lam', 'vals'):
        np.testing.assert_allclose(res['0'][key], res['1'][key], rtol=1e-9, atol=1e-12)


def test_flop_tally_counts_the_launched_products():
    """vb_flop_tally (the executed-flop figure of bench.py's config-4 leg): a
    reset zeroes it, a full-rank advance at D = 64 adds the matrix-core work of its
    products (per step at least three of the PCG's symmetric sums, 2 D^3 each -- D^2 / 2
    complete entries of depth 2D -- and the Sigma = L L^T product, 3 of its 4 tiles at
    D = 64), and a read without reset leaves it unchanged."""
    vb, targets, _, _, _ = _mods()
    from viabel_amd import _native as nat
    D, N = 64, 16
    fam = vb.t_variational_family(D, 30.0, rng='philox')
    run = vb.DeviceRun(vb.black_box_chivi(2.0, fam, targets.corr_gauss(D), N), 4, _lam(D, 3))
    run.advance_philox(1, 0, 1, 0)
    nat.context().synchronize()
    nat.lib().vb_flop_tally(1)
    assert nat.lib().vb_flop_tally(0) == 0.0
    run.advance_philox(3, 0, 1, 1)
    nat.context().synchronize()
    f = nat.lib().vb_flop_tally(0)
    assert f >= 3 * (3 * 2 * D ** 3 + 0.75 * 2 * D ** 3), f
    assert f < 3 * 200 * 2 * D ** 3, f
    assert nat.lib().vb_flop_tally(1) == f
    assert nat.lib().vb_flop_tally(0) == 0.0
