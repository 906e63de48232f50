"""GPU parity: the HIP estimators / optimiser against the oracle on identical
noise.  Tolerances (written per test): single estimator calls 1e-10 relative
(SURVEY §8c asks <= 1e-12 for identical noise; reduction-order and FMA
differences stay around 1e-14..1e-12); adagrad trajectories <= 1e-7 relative
over >= 100 steps (the bar is 1e-5)."""
import os

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]

FAMS = [('gauss', None), ('t', 40.0), ('t', 8.0)]
SMALL_TARGETS = [('isogauss', 6), ('mixture', 5), ('funnel', 10), ('eight_schools_ncp', 10),
                 ('funnel', 2), ('isogauss', 1)]


def test_gpu_library_was_built_from_these_sources():
    """Build provenance on the GPU box: the library this process loads carries
    the hash of the sources in the tree it runs from (vb_build_id,
    tests/test_abi.py::source_hash), so the parity results below are those of
    the committed sources."""
    from tests.test_abi import source_hash
    from viabel_amd import _native
    assert _native.lib().vb_build_id().decode() == source_hash()


def _mods():
    from viabel_amd import vb, targets
    from oracle import vb_oracle, rng_oracle
    return vb, targets, vb_oracle, rng_oracle


def _family(vb, kind, df, D, rng):
    if kind == 'gauss':
        return vb.mean_field_gaussian_variational_family(D, rng=rng)
    return vb.mean_field_t_variational_family(D, df, rng=rng)


def _target(targets, name, D):
    return {'isogauss': lambda: targets.isogauss(D), 'mixture': lambda: targets.mixture(D),
            'funnel': lambda: targets.funnel(D),
            'eight_schools_ncp': targets.eight_schools_ncp}[name]()


def _lam(D, seed):
    rs = np.random.RandomState(seed)
    return np.concatenate([rs.randn(D) * 0.7, rs.randn(D) * 0.3 - 0.2])


def _scale(g):
    return max(1.0, float(np.max(np.abs(g))))


# ---------------------------------------------------------------------------
@pytest.mark.parametrize('kind,df', FAMS)
@pytest.mark.parametrize('target,D', SMALL_TARGETS)
@pytest.mark.parametrize('N', [1, 100, 128, 700])
def test_klvi_call_numpy_stream(kind, df, target, D, N):
    """black_box_klvi(fam, p, N)(lam) consumes fam's RandomState(0) like vb.py:239."""
    vb, targets, vo, _ = _mods()
    fam = _family(vb, kind, df, D, 'numpy')
    ofam = vo.Family(kind, D, df)
    obj = vb.black_box_klvi(fam, _target(targets, target, D), N)
    for call in range(3):  # the stream continues across calls
        lam = _lam(D, call)
        v, g = obj(lam)
        ov, og = vo.klvi_value_grad(ofam, target, lam, N)
        assert abs(v - ov) <= 1e-10 * max(1.0, abs(ov))
        np.testing.assert_allclose(g, og, rtol=1e-10, atol=1e-10 * _scale(og))


@pytest.mark.parametrize('kind,df', FAMS)
@pytest.mark.parametrize('target,D', SMALL_TARGETS)
@pytest.mark.parametrize('alpha', [2.0, 1.5])
def test_chivi_call_numpy_stream(kind, df, target, D, alpha):
    """black_box_chivi draws seed = npr.randint(2**32) from the GLOBAL RNG (vb.py:258)."""
    vb, targets, vo, _ = _mods()
    fam = _family(vb, kind, df, D, 'numpy')
    ofam = vo.Family(kind, D, df)
    obj = vb.black_box_chivi(alpha, fam, _target(targets, target, D), 128)
    for call in range(2):
        lam = _lam(D, 10 + call)
        np.random.seed(77 + call)
        v, g = obj(lam)
        np.random.seed(77 + call)
        ov, og = vo.chivi_value_grad(ofam, target, lam, 128, alpha)
        assert abs(v - ov) <= 1e-10 * max(1.0, abs(ov))
        np.testing.assert_allclose(g, og, rtol=1e-9, atol=1e-9 * _scale(og))


@pytest.mark.parametrize('kind,df', FAMS)
@pytest.mark.parametrize('target', ['isogauss', 'mixture'])
@pytest.mark.parametrize('D', [17, 1000, 10001])
def test_klvi_call_wide_separable(kind, df, target, D):
    """D > 16 with a separable target goes through the column-pair kernel."""
    vb, targets, vo, _ = _mods()
    N = 96
    fam = _family(vb, kind, df, D, 'numpy')
    ofam = vo.Family(kind, D, df)
    obj = vb.black_box_klvi(fam, _target(targets, target, D), N)
    lam = _lam(D, 5)
    v, g = obj(lam)
    ov, og = vo.klvi_value_grad(ofam, target, lam, N)
    assert abs(v - ov) <= 1e-10 * max(1.0, abs(ov))
    np.testing.assert_allclose(g, og, rtol=1e-10, atol=1e-10 * _scale(og))


@pytest.mark.parametrize('kind,df', FAMS)
@pytest.mark.parametrize('target,D', [('isogauss', 7), ('funnel', 10), ('mixture', 4000)])
def test_klvi_call_philox_matches_oracle_noise(kind, df, target, D):
    """Philox mode: the kernel's in-register draws equal the C oracle's draws, so
    the estimator matches the oracle fed with rng_oracle noise."""
    vb, targets, vo, ro = _mods()
    N = 128
    fam = _family(vb, kind, df, D, 'philox')
    obj = vb.black_box_klvi(fam, _target(targets, target, D), N)
    ofam = vo.Family(kind, D, df)
    for call in range(2):
        lam = _lam(D, 20 + call)
        v, g = obj(lam)
        eps = ro.noise(fam.seed, fam.stream, call, N, D, kind, df or 0.0)
        ov, og = vo.klvi_value_grad(ofam, target, lam, N, eps=eps)
        assert abs(v - ov) <= 1e-10 * max(1.0, abs(ov))
        np.testing.assert_allclose(g, og, rtol=1e-9, atol=1e-9 * _scale(og))


# ---------------------------------------------------------------------------
def _oracle_run(vo, ofam, objective, target, n_iters, init, N, alpha=2.0, eps_fn=None, **kw):
    step = [0]

    def f(lam):
        eps = eps_fn(step[0]) if eps_fn else None
        step[0] += 1
        if objective == 'klvi':
            return vo.klvi_value_grad(ofam, target, lam, N, eps=eps)
        return vo.chivi_value_grad(ofam, target, lam, N, alpha, eps=eps)
    return vo.adagrad_optimize(n_iters, f, init, **kw)


@pytest.mark.parametrize('kind,df', FAMS)
@pytest.mark.parametrize('objective', ['klvi', 'chivi'])
@pytest.mark.parametrize('target,D', [('funnel', 10), ('eight_schools_ncp', 10), ('mixture', 3)])
def test_adagrad_trajectory_numpy_stream(kind, df, objective, target, D):
    """Device-resident adagrad == reference loop on the same numpy streams,
    with the funnel notebook's decaying schedule (lr .01 -> .001)."""
    vb, targets, vo, _ = _mods()
    N, n_iters = 100, 120
    fam = _family(vb, kind, df, D, 'numpy')
    ofam = vo.Family(kind, D, df)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    init[1] = -1.0
    tgt = _target(targets, target, D)
    obj = (vb.black_box_klvi(fam, tgt, N) if objective == 'klvi'
           else vb.black_box_chivi(2.0, fam, tgt, N))
    np.random.seed(4)
    res = vb.adagrad_optimize(n_iters, obj, init, learning_rate=.01, learning_rate_end=.001)
    np.random.seed(4)
    ores = _oracle_run(vo, ofam, objective, target, n_iters, init, N,
                       learning_rate=.01, learning_rate_end=.001)
    assert res[1].shape == ores[1].shape == (n_iters - 3 * n_iters // 4, 2 * D)
    np.testing.assert_allclose(res[1], ores[1], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(res[0], ores[0], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(res[2], ores[2], rtol=1e-7, atol=1e-7)
    assert np.all(res[3] == 0)


@pytest.mark.parametrize('kind,df', [('gauss', None), ('t', 40.0)])
@pytest.mark.parametrize('D', [33, 2000])
def test_adagrad_trajectory_wide(kind, df, D):
    """Column-pair persistent kernel: 130 steps (crosses the chunk and window
    boundaries), constant lr like config 3."""
    vb, targets, vo, _ = _mods()
    N, n_iters = 64, 130
    fam = _family(vb, kind, df, D, 'numpy')
    ofam = vo.Family(kind, D, df)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
    res = vb.adagrad_optimize(n_iters, obj, init, learning_rate=0.05)
    ores = _oracle_run(vo, ofam, 'klvi', 'isogauss', n_iters, init, N, learning_rate=0.05)
    np.testing.assert_allclose(res[1], ores[1], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(res[2], ores[2], rtol=1e-7, atol=1e-7)


@pytest.mark.parametrize('kind,df', [('gauss', None), ('t', 40.0)])
@pytest.mark.parametrize('target,D', [('isogauss', 3000), ('funnel', 10)])
def test_adagrad_trajectory_philox(kind, df, target, D):
    """Philox mode trajectories equal the oracle loop fed with the C-oracle draws."""
    vb, targets, vo, ro = _mods()
    N, n_iters = 64, 110
    fam = _family(vb, kind, df, D, 'philox')
    ofam = vo.Family(kind, D, df)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    obj = vb.black_box_klvi(fam, _target(targets, target, D), N)
    seed, stream, step0 = fam.seed, fam.stream, fam.step
    res = vb.adagrad_optimize(n_iters, obj, init, learning_rate=0.02, learning_rate_end=0.005)
    eps_fn = lambda i: ro.noise(seed, stream, step0 + i, N, D, kind, df or 0.0)
    ores = _oracle_run(vo, ofam, 'klvi', target, n_iters, init, N, eps_fn=eps_fn,
                       learning_rate=0.02, learning_rate_end=0.005)
    np.testing.assert_allclose(res[1], ores[1], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(res[2], ores[2], rtol=1e-7, atol=1e-7)


def test_many_problems_one_launch():
    """n_problems restarts in one vb_run (one workgroup each) == independent runs."""
    vb, targets, vo, ro = _mods()
    from viabel_amd.vb import DeviceRun
    D, N, n_iters, R = 10, 100, 60, 5
    fam = vb.mean_field_t_variational_family(D, 40, rng='philox')
    obj = vb.black_box_klvi(fam, targets.eight_schools_ncp(), N)
    inits = np.random.RandomState(0).randn(R, 2 * D) * 0.5
    run = DeviceRun(obj, n_iters, inits, learning_rate=0.01, learning_rate_end=0.001)
    run.advance_philox(n_iters, seed=9, stream=100, step=0)
    lam, hist, vals, smooth = run.result()
    ofam = vo.Family('t', D, 40.0)
    for r in range(R):
        eps_fn = lambda i, r=r: ro.noise(9, 100 + r, i, N, D, 't', 40.0)
        ores = _oracle_run(vo, ofam, 'klvi', 'eight_schools_ncp', n_iters, inits[r], N,
                           eps_fn=eps_fn, learning_rate=0.01, learning_rate_end=0.001)
        np.testing.assert_allclose(hist[r], ores[1], rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(vals[r], ores[2], rtol=1e-7, atol=1e-7)
        np.testing.assert_allclose(smooth[r], ores[0], rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize('kind,df,objective,N', [('gauss', None, 'klvi', 100), ('t', 40.0, 'klvi', 100),
                                                 ('t', 40.0, 'chivi', 128), ('gauss', None, 'klvi', 600)])
def test_many_problems_first_steps(kind, df, objective, N):
    """96 problems x 3 steps in one launch: every workgroup's first draws (the
    pipelined prologue reads the LDS Box-Muller tables) and the draw/row
    overlap of the next steps match the oracle.  N = 600 takes the chunked
    (non-overlapped) layout."""
    vb, targets, vo, ro = _mods()
    D, n_iters, R = 10, 3, 96
    fam = _family(vb, kind, df, D, 'philox')
    tgt = targets.funnel(D)
    obj = (vb.black_box_klvi(fam, tgt, N) if objective == 'klvi'
           else vb.black_box_chivi(2.0, fam, tgt, N))
    inits = np.random.RandomState(5).randn(R, 2 * D) * 0.3
    run = vb.DeviceRun(obj, n_iters, inits, learning_rate=0.05)
    run.advance_philox(n_iters, seed=3, stream=7, step=0)
    lam, hist, vals, smooth = run.result()
    ofam = vo.Family(kind, D, df)
    for r in range(R):
        eps_fn = lambda i, r=r: ro.noise(3, 7 + r, i, N, D, kind, df or 0.0)
        ores = _oracle_run(vo, ofam, objective, 'funnel', n_iters, inits[r], N,
                           eps_fn=eps_fn, learning_rate=0.05)
        np.testing.assert_allclose(vals[r], ores[2], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(lam[r], ores[1][-1], rtol=1e-9, atol=1e-11)


def test_foreign_objective_device_update():
    """A plain Python objective runs with the device adagrad update kernel."""
    vb, targets, vo, _ = _mods()
    D = 4
    ofam_a = vo.Family('gauss', D)
    ofam_b = vo.Family('gauss', D)
    f_a = lambda l: vo.klvi_value_grad(ofam_a, 'isogauss', l, 50)
    f_b = lambda l: vo.klvi_value_grad(ofam_b, 'isogauss', l, 50)
    init = np.ones(2 * D)
    res = vb.adagrad_optimize(40, f_a, init, learning_rate=0.1, learning_rate_end=0.01)
    ores = vo.adagrad_optimize(40, f_b, init, learning_rate=0.1, learning_rate_end=0.01)
    np.testing.assert_allclose(res[1], ores[1], rtol=1e-12, atol=1e-14)


# ---------------------------------------------------------------------------
@pytest.mark.parametrize('kind,df', FAMS)
@pytest.mark.parametrize('D', [3, 10, 100])
def test_family_sample_and_logdensity(kind, df, D):
    vb, targets, vo, _ = _mods()
    fam = _family(vb, kind, df, D, 'numpy')
    ofam = vo.Family(kind, D, df)
    lam = _lam(D, 2)
    x = fam.sample(lam, 500)
    ox = ofam.sample(lam, 500)
    np.testing.assert_allclose(x, ox, rtol=1e-14, atol=1e-14)
    np.testing.assert_allclose(fam.logdensity(x, lam), ofam.logdensity(x, lam), rtol=1e-12)
    xs = fam.sample(lam, 7, seed=99)
    np.testing.assert_allclose(xs, ofam.sample(lam, 7, seed=99), rtol=1e-14, atol=1e-14)


@pytest.mark.parametrize('target,D', SMALL_TARGETS + [('mixture', 300), ('isogauss', 5000)])
def test_target_logdensity_and_grad(target, D):
    vb, targets, vo, _ = _mods()
    from oracle import targets_oracle
    x = np.random.RandomState(1).randn(333, D)
    lp, g = _target(targets, target, D).logdensity_and_grad(x)
    olp, og = targets_oracle.TARGETS[target](x)
    np.testing.assert_allclose(lp, olp, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(g, og, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize('kind,df', FAMS)
@pytest.mark.parametrize('target,D', [('eight_schools_ncp', 10), ('mixture', 2), ('isogauss', 40)])
def test_log_weights(kind, df, target, D):
    """experiments.py:60-63 on the device, continuing the family stream."""
    from viabel_amd import experiments
    vb, targets, vo, _ = _mods()
    fam = _family(vb, kind, df, D, 'numpy')
    ofam = vo.Family(kind, D, df)
    lam = _lam(D, 6)
    x, lw = experiments.get_samples_and_log_weights(_target(targets, target, D), fam, lam, 5000)
    ox, olw = vo.log_weights(ofam, target, lam, 5000)
    np.testing.assert_allclose(x, ox, rtol=1e-14, atol=1e-14)
    np.testing.assert_allclose(lw, olw, rtol=1e-11, atol=1e-11)


@pytest.mark.parametrize('kind,df', [('gauss', None), ('t', 40.0), ('t', 3.5)])
@pytest.mark.parametrize('D', [1, 2, 9, 64])
def test_device_philox_noise_equals_c_oracle(kind, df, D):
    """The in-kernel draws (lambda = 0: x = eps) equal oracle/vbrng.c's draws to
    ~1 ulp (the device uses short fp64 log/sqrt/sincospi, the oracle libm)."""
    vb, targets, vo, ro = _mods()
    fam = _family(vb, kind, df, D, 'philox')
    lam = np.zeros(2 * D)
    for call in range(2):
        x = fam.sample(lam, 3000)
        eps = ro.noise(fam.seed, fam.stream, call, 3000, D, kind, df or 0.0)
        np.testing.assert_allclose(x, eps, rtol=2e-14, atol=1e-13)
    # a seeded call uses key = seed, stream 0, step 0
    x = fam.sample(lam, 100, seed=1234)
    np.testing.assert_allclose(x, ro.noise(1234, 0, 0, 100, D, kind, df or 0.0),
                               rtol=2e-14, atol=1e-13)


@pytest.mark.parametrize('kind,df,D', [('gauss', None, 17), ('t', 40.0, 8200), ('gauss', None, 9001),
                                       ('gauss', None, 18432), ('t', 40.0, 40000)])
def test_sep_layouts_agree(kind, df, D):
    """Every branch of the column-pair kernel's grid split (vb_mf.hip sep_split)
    gives the oracle's trajectory (Philox noise): 1-pair waves only (D = 17), one
    4-pair wave per SIMD + 1-pair waves (8200, 9001: partial blocks of each kind),
    two layers of 4-pair waves + 1-pair waves (18 432), all 4-pair waves (40 000)."""
    vb, targets, vo, ro = _mods()
    N, n_iters = 100, 24
    fam = _family(vb, kind, df, D, 'philox')
    ofam = vo.Family(kind, D, df)
    init = np.concatenate([np.linspace(-1, 1, D), np.full(D, 0.3)])
    obj = vb.black_box_klvi(fam, targets.mixture(D), N)
    seed, stream, step0 = fam.seed, fam.stream, fam.step
    res = vb.adagrad_optimize(n_iters, obj, init, learning_rate=0.03, window=7)
    eps_fn = lambda i: ro.noise(seed, stream, step0 + i, N, D, kind, df or 0.0)
    ores = _oracle_run(vo, ofam, 'klvi', 'mixture', n_iters, init, N, eps_fn=eps_fn,
                       learning_rate=0.03, window=7)
    np.testing.assert_allclose(res[1], ores[1], rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(res[2], ores[2], rtol=1e-9, atol=1e-9)


def test_adagrad_chunked_progress_and_interrupt(monkeypatch):
    """adagrad_optimize runs the device loop in chunks (>= 1000 steps) with the
    reference's progress bar between them; the result equals one unchunked
    device run, and a KeyboardInterrupt returns the steps done so far
    (vb.py:377-389)."""
    vb, targets, vo, ro = _mods()
    D, N, n_iters = 6, 64, 2400
    monkeypatch.setenv('VIABEL_AMD_PROGRESS', '1')
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    init = np.concatenate([np.zeros(D), np.ones(D)])
    obj = vb.black_box_klvi(fam, targets.funnel(D), N)
    seed, stream, step0 = fam.seed, fam.stream, fam.step
    res = vb.adagrad_optimize(n_iters, obj, init, learning_rate=0.02, learning_rate_end=0.005)
    # the same run as one device launch chain
    run = vb.DeviceRun(obj, n_iters, init[None, :], 10, 0.02, 0.1, 0.005)
    run.advance_philox(n_iters, seed, stream, step0)
    _, hist, vals, smooth = run.result()
    np.testing.assert_array_equal(res[2], vals[0])
    np.testing.assert_array_equal(res[1], hist[0])
    np.testing.assert_array_equal(res[0], smooth[0])
    # interrupt after the first chunk (1000 steps): partial results
    calls = []
    orig = vb.DeviceRun.advance_philox

    def interrupting(self, *a, **k):
        if calls:
            raise KeyboardInterrupt
        calls.append(1)
        return orig(self, *a, **k)
    monkeypatch.setattr(vb.DeviceRun, 'advance_philox', interrupting)
    fam2 = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj2 = vb.black_box_klvi(fam2, targets.funnel(D), N)
    seed2, stream2, step2 = fam2.seed, fam2.stream, fam2.step
    part = vb.adagrad_optimize(n_iters, obj2, init, learning_rate=0.02, learning_rate_end=0.005)
    assert part[2].shape == (1000,) and part[3].shape == (1000,)
    monkeypatch.setattr(vb.DeviceRun, 'advance_philox', orig)
    run2 = vb.DeviceRun(obj2, n_iters, init[None, :], 10, 0.02, 0.1, 0.005)
    run2.advance_philox(1000, seed2, stream2, step2)
    np.testing.assert_array_equal(part[2], run2.values()[:1000])
    assert part[1].shape == (0, 2 * D) and np.all(np.isnan(part[0]))
    # an interrupt landing after an advance returned (before the caller counted
    # it): the result covers every step the device ran
    def late(self, *a, **k):
        orig(self, *a, **k)
        raise KeyboardInterrupt
    monkeypatch.setattr(vb.DeviceRun, 'advance_philox', late)
    fam3 = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj3 = vb.black_box_klvi(fam3, targets.funnel(D), N)
    part3 = vb.adagrad_optimize(n_iters, obj3, init, learning_rate=0.02, learning_rate_end=0.005)
    assert part3[2].shape == (1000,)


# ---------------------------------------------------------------------------
@pytest.mark.parametrize('objective', ['klvi', 'chivi', 'klvi_pd'])
@pytest.mark.parametrize('target,D,N,nprob', [('funnel', 10, 128, 1), ('eight_schools_ncp', 10, 100, 3),
                                              ('mixture', 5, 300, 2), ('isogauss', 1, 64, 1)])
def test_predraw_equals_in_kernel_draws(objective, target, D, N, nprob, monkeypatch):
    """Gaussian-family block-kernel runs whose Philox draws are pre-drawn by the
    throughput kernel (VIABEL_AMD_PREDRAW=all; the t family always pre-draws,
    DESIGN §4) give bit-identical trajectories, values and histories to the
    in-kernel draws, across predraw chunk boundaries."""
    import viabel_amd.vb as vbm
    vb, targets, _, _ = _mods()
    fam = _family(vb, 'gauss', None, D, 'philox')
    tgt = _target(targets, target, D)
    obj = {'klvi': lambda: vb.black_box_klvi(fam, tgt, N),
           'chivi': lambda: vb.black_box_chivi(2.0, fam, tgt, N),
           'klvi_pd': lambda: vb.black_box_klvi_pd(fam, tgt, N)}[objective]()
    init = np.stack([_lam(D, 40 + q) for q in range(nprob)])
    out = {}
    for mode in ('0', 'all'):
        monkeypatch.setenv('VIABEL_AMD_PREDRAW', mode)
        run = vbm.DeviceRun(obj, 700, init, learning_rate=0.01)
        run.advance_philox(3, 7, 5, 0)
        run.advance_philox(697, 7, 5, 3)        # > one 512-step predraw chunk
        out[mode] = run.result()
    if _split_rows(D, N):
        # the pre-drawn rows run as split rows (two lanes per sample):
        # the same draws and arithmetic summed in another order -- equal to
        # rounding; the bitwise identity of the unsplit layout is
        # test_predraw_equals_in_kernel_draws_unsplit
        for a, b in zip(out['0'], out['all']):
            np.testing.assert_allclose(a, b, rtol=1e-10, atol=1e-12)
    else:
        for a, b in zip(out['0'], out['all']):
            np.testing.assert_array_equal(a, b)


def _split_rows(D, N):
    """block_layout's split-row condition (copy-wave layout, VIABEL_AMD_BLOCK_SPLIT
    not 0)."""
    return os.environ.get('VIABEL_AMD_BLOCK_SPLIT', '1') != '0' and 2 <= D <= 10 and N <= 128


_UNSPLIT = '''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import viabel_amd.vb as vb
from viabel_amd import targets
D, N, nprob = 10, int(sys.argv[3]), int(sys.argv[4])
fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
tgt = targets.eight_schools_ncp() if sys.argv[2] == 'eight_schools_ncp' else getattr(targets, sys.argv[2])(D)
obj = vb.black_box_chivi(2.0, fam, tgt, N) if sys.argv[5] == 'chivi' else vb.black_box_klvi(fam, tgt, N)
rs = np.random.RandomState(40)
init = np.stack([np.concatenate([rs.randn(D) * 0.3, rs.randn(D) * 0.2 - 0.5]) for _ in range(nprob)])
out = {}
import os
for mode in ('0', 'all'):
    os.environ['VIABEL_AMD_PREDRAW'] = mode
    run = vb.DeviceRun(obj, 700, init, learning_rate=0.01)
    run.advance_philox(3, 7, 5, 0)
    run.advance_philox(697, 7, 5, 3)
    out[mode] = run.result()
for a, b in zip(out['0'], out['all']):
    np.testing.assert_array_equal(a, b)
print('bitwise-equal')
'''


_OVERLAP = '''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import viabel_amd.vb as vb
from viabel_amd import targets
D, R, iters = 10, 10, 1300
fam = vb.mean_field_t_variational_family(D, 40.0, rng='philox')
obj = vb.black_box_klvi(fam, targets.eight_schools_ncp(), 100)
rs = np.random.RandomState(3)
init = rs.randn(R, 2 * D) * 0.5
run = vb.DeviceRun(obj, iters, init, window=10, learning_rate=.01, learning_rate_end=.001)
run.advance_philox(700, 0, 1, 0, stream_stride=1)
run.advance_philox(600, 0, 1, 700, stream_stride=1)
lam, hist, vals, smooth = run.result()
np.savez(sys.argv[2], lam=lam, hist=hist, vals=vals)
'''


def test_predraw_overlap_is_bitwise_serial(tmp_path):
    """The overlapped pre-draw (chunk k + 1 drawn on the odd CUs beside chunk k's
    block kernel, two buffers) against the serial order
    (VIABEL_AMD_PREDRAW_OVERLAP=0, read once per process: child processes): the same
    trajectories, values and histories bit for bit, over 1 300 steps = 3 chunks of
    10 problems (the overlap needs >= 8)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for mode in ('0', '1'):
        f = str(tmp_path / ('ov%s.npz' % mode))
        env = dict(os.environ, VIABEL_AMD_PREDRAW_OVERLAP=mode)
        r = subprocess.run([sys.executable, '-c', _OVERLAP, root, f], env=env, capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        out[mode] = np.load(f)
    for k in ('lam', 'hist', 'vals'):
        np.testing.assert_array_equal(out['0'][k], out['1'][k])


@pytest.mark.parametrize('target,N,nprob,objective', [('funnel', 128, 1, 'chivi'),
                                                      ('eight_schools_ncp', 100, 3, 'klvi')])
def test_predraw_equals_in_kernel_draws_unsplit(target, N, nprob, objective):
    """With split rows off (VIABEL_AMD_BLOCK_SPLIT=0, read once per process, so in
    a child process) the copy-wave layout gives the in-kernel draws' bits."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, VIABEL_AMD_BLOCK_SPLIT='0')
    r = subprocess.run([sys.executable, '-c', _UNSPLIT, root, target, str(N), str(nprob), objective],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and 'bitwise-equal' in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize('objective', ['klvi', 'chivi'])
def test_t_family_predraw_large_n_matches_oracle(objective):
    """The t family's pre-drawn block-kernel path at N > 256 (rows looped per
    thread, several problems, per-problem Philox streams) against the oracle loop
    fed with the C-oracle draws (trajectory bar 1e-7)."""
    vb, targets, vo, ro = _mods()
    D, N, n_iters, R = 5, 300, 40, 2
    fam = _family(vb, 't', 40.0, D, 'philox')
    tgt = targets.mixture(D)
    obj = (vb.black_box_klvi(fam, tgt, N) if objective == 'klvi'
           else vb.black_box_chivi(2.0, fam, tgt, N))
    inits = np.stack([_lam(D, 40 + q) for q in range(R)])
    run = vb.DeviceRun(obj, n_iters, inits, learning_rate=0.01)
    run.advance_philox(n_iters, seed=7, stream=5, step=0)
    lam, hist, vals, smooth = run.result()
    ofam = vo.Family('t', D, 40.0)
    for r in range(R):
        eps_fn = lambda i, r=r: ro.noise(7, 5 + r, i, N, D, 't', 40.0)
        ores = _oracle_run(vo, ofam, objective, 'mixture', n_iters, inits[r], N,
                           eps_fn=eps_fn, learning_rate=0.01)
        np.testing.assert_allclose(vals[r], ores[2], rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(lam[r], ores[1][-1], rtol=1e-7, atol=1e-9)


# ---------------------------------------------------------------------------
@pytest.mark.parametrize('kind,df', [('gauss', None), ('t', 40.0)])
@pytest.mark.parametrize('objective', ['klvi', 'chivi'])
@pytest.mark.parametrize('D', [1, 2, 10, 16])
def test_in_kernel_draws_at_layout_boundaries(kind, df, objective, D, monkeypatch):
    """In-kernel Philox draws of the block kernel (VIABEL_AMD_PREDRAW=0, the t
    family included: its instance faulted at N > 256 when its draw routine was
    compiled out of line) across the draw-buffer layouts: N from the
    overlapped draw/row layout through the chunked layout and several chunks,
    for every DMAX instance; each N equals the pre-drawn path to rounding and the
    oracle fed with the C-oracle draws (1e-9)."""
    import viabel_amd.vb as vbm
    vb, targets, vo, ro = _mods()
    tgt = targets.funnel(D) if D >= 2 else targets.isogauss(D)
    tname = 'funnel' if D >= 2 else 'isogauss'
    ofam = vo.Family(kind, D, df)
    for N in (255, 256, 257, 300, 600):
        fam = _family(vb, kind, df, D, 'philox')
        obj = (vb.black_box_klvi(fam, tgt, N) if objective == 'klvi'
               else vb.black_box_chivi(2.0, fam, tgt, N))
        init = np.stack([_lam(D, 60 + q) for q in range(2)])
        out = {}
        for mode in ('0', 'all'):
            monkeypatch.setenv('VIABEL_AMD_PREDRAW', mode)
            run = vbm.DeviceRun(obj, 4, init, learning_rate=0.02)
            run.advance_philox(4, 11, 9, 0)
            out[mode] = run.result()
        # the two paths share every draw; past the overlapped layout (N > 256)
        # the row threads accumulate their samples in a different association,
        # so equality is to rounding (observed <= 2 ulp)
        for a, b in zip(out['0'], out['all']):
            np.testing.assert_allclose(a, b, rtol=1e-13, atol=1e-15, err_msg='N=%d' % N)
        lam, _, vals, _ = out['0']
        for r in range(2):
            eps_fn = lambda i, r=r: ro.noise(11, 9 + r, i, N, D, kind, df or 0.0)
            ores = _oracle_run(vo, ofam, objective, tname, 4, init[r], N, eps_fn=eps_fn,
                               learning_rate=0.02)
            np.testing.assert_allclose(vals[r], ores[2], rtol=1e-9, atol=1e-9, err_msg='N=%d' % N)
            np.testing.assert_allclose(lam[r], ores[1][-1], rtol=1e-9, atol=1e-11,
                                       err_msg='N=%d' % N)
