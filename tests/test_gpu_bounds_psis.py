"""GPU parity for viabel_amd.bounds and viabel_amd.psis against the reference's
golden vectors (tests/golden) and the oracle.  Tolerances: bounds 1e-10
relative (bar: 1e-5); PSIS k 1e-10 (bar: 1e-5), smoothed log weights 1e-11,
tail order (tailinds[x2si]) bit-exact."""
import warnings

import numpy as np
import pytest
from scipy.special import factorial2

from tests.conftest import gpu_available
from tests.golden.make_golden import mixture_inputs

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]


def _close(a, b, rtol=1e-10, atol=1e-12):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


class TestBounds:
    def test_normal_mixture_notebook(self, golden):
        import viabel_amd as va
        g = golden['bounds']
        samples, lw, q_var = mixture_inputs()
        mb = lambda order: factorial2(order - 1) ** (1 / order) * np.sqrt(q_var)
        cases = {
            'mix_a': va.all_bounds(lw, samples),
            'mix_b': va.all_bounds(lw, samples, q_var=q_var, log_norm_bound=0),
            'mix_c': va.all_bounds(lw, moment_bound_fn=mb, q_var=q_var),
        }
        for cname, res in cases.items():
            assert set(res) == {'W1', 'W2', 'mean_error', 'std_error', 'cov_error', 'd2',
                                'log_norm_bound'}
            for k, v in res.items():
                _close(v, g['%s_%s' % (cname, k)])

    @pytest.mark.parametrize('alpha', [1.5, 2.0, 3.0])
    @pytest.mark.parametrize('elbo', [None, 0.0])
    def test_divergence(self, golden, alpha, elbo):
        import viabel_amd as va
        g = golden['bounds']
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            d, lnb = va.divergence_bound(g['div_lw'], alpha, elbo, return_log_norm_bound=True)
        tag = 'div_a%g_%s' % (alpha, 'none' if elbo is None else 'zero')
        _close([d, lnb], g[tag])

    def test_wasserstein_and_cov(self, golden):
        import viabel_amd as va
        g = golden['bounds']
        for tag, s in (('w1d', g['w_s1']), ('w3d', g['w_s3'])):
            r = va.wasserstein_bounds(5.0, s)
            _close([r['W1'], r['W2']], g[tag])
        r = va.all_bounds(g['ab3_lw'], g['w_s3'])
        for k, v in r.items():
            _close(v, g['ab3_' + k])

    def test_warnings_and_errors(self, golden):
        import viabel_amd as va
        g = golden['bounds']
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter('always')
            va.divergence_bound(g['warn_lw'])
        assert [str(x.message) for x in w] == list(g['warn_msgs'])
        with pytest.raises(ValueError, match='alpha must be greater than 1'):
            va.divergence_bound(g['warn_lw'], alpha=1.0)
        with pytest.raises(ValueError, match='must provides samples'):
            va.wasserstein_bounds(1.0)

    def test_large_sizes_properties(self):
        """1e7 draws (reference test_bounds.py MC_SAMPLES): closed-form Renyi
        divergence of two Gaussians within the reference's MC_TOL, and the
        oracle within 1e-9."""
        import viabel_amd as va
        from oracle import bounds_oracle
        rs = np.random.RandomState(846)
        var1, var2 = 4.0, 16.0
        s = rs.randn(10_000_000) * np.sqrt(var2)
        lw = (-0.5 * s ** 2 / var1 - 0.5 * np.log(var1)) - (-0.5 * s ** 2 / var2 - 0.5 * np.log(var2))
        d = va.divergence_bound(lw, 2.0, 0.0)
        od = bounds_oracle.divergence_bound(lw, 2.0, 0.0)
        _close(d, od, rtol=1e-9)
        tmp = 2 * var2 - var1
        expected = -0.5 * np.log(tmp) + np.log(var2) - 0.5 * np.log(var1)
        assert abs(d - expected) < 5 / np.sqrt(1e7) * (1 + abs(expected))


class TestPsis:
    @pytest.mark.parametrize('case', ['normal1000', 't3_1000', 'n5', 'n128', 'heavy2e4', 'cols'])
    def test_psislw_golden(self, golden, case):
        from viabel_amd import psis
        from oracle import psis_oracle
        g = golden['psis']
        lw = g[case + '_in'].copy()
        out, k = psis.psislw(lw)
        _close(out, g[case + '_out'], rtol=1e-11, atol=1e-11)
        _close(np.atleast_1d(k), g[case + '_k'])
        if lw.ndim == 1:
            assert np.isscalar(k) or np.ndim(k) == 0
        # tail order bit-exact vs the oracle's argsort
        _, _, tails = psis.psislw_with_tail(lw)
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            _, _, otails = psis_oracle.psislw(lw.copy(), return_tail=True)
        for t, ot in zip(tails, otails):
            if len(ot) > 4:
                np.testing.assert_array_equal(t, ot)

    def test_psislw_output_layout(self, golden):
        from viabel_amd import psis
        g = golden['psis']
        lw = g['cols_in'].copy()
        out, k = psis.psislw(lw)
        assert out.flags.f_contiguous and out.shape == lw.shape and k.shape == (3,)
        lwf = np.asfortranarray(g['cols_in'])
        res, _ = psis.psislw(lwf, overwrite_lw=True)
        assert res is lwf
        _close(lwf, g['cols_out'], rtol=1e-11, atol=1e-11)

    def test_gpdfit_gpinv_sumlogs(self, golden):
        from viabel_amd import psis
        g = golden['psis']
        k, sigma, ks, w = psis.gpdfitnew(g['gpd_x'].copy(), return_quadrature=True)
        _close([k, sigma], g['gpd_k'])
        _close(ks, g['gpd_ks'])
        _close(w, g['gpd_w'])
        p = g['gpinv_p']
        for tag, (kk, ss) in {'gpinv_pos': (0.4, 1.3), 'gpinv_neg': (-0.3, 2.0),
                              'gpinv_zero': (1e-18, 0.7), 'gpinv_badsig': (0.2, -1.0)}.items():
            _close(psis.gpinv(p, kk, ss), g[tag], rtol=1e-13)
        _close(psis.sumlogs(g['sumlogs_x']), g['sumlogs'][0], rtol=1e-13)

    def test_errors(self):
        from viabel_amd import psis
        with pytest.raises(ValueError, match='More than one log-weight'):
            psis.psislw(np.zeros(1))
        with pytest.raises(ValueError, match='Invalid input array'):
            psis.gpdfitnew(np.zeros(1))

    @pytest.mark.parametrize('n', [1_000_000, 2_500_000])
    def test_full_size(self, n):
        """The notebooks' sizes (funnel 1e6, eight schools 2.5e6): k within 1e-9,
        tail order bit-exact, smoothed weights within 1e-11 of the oracle."""
        from viabel_amd import psis
        from oracle import psis_oracle
        rs = np.random.RandomState(n % 997)
        lw = rs.standard_t(3, n) * 1.3 - 2.0
        out, k, tails = psis.psislw_with_tail(lw)
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            oout, ok, otails = psis_oracle.psislw(lw.copy(), return_tail=True)
        _close(k, ok, rtol=1e-9)
        np.testing.assert_array_equal(tails[0], otails[0])
        _close(out[:, 0], oout, rtol=1e-11, atol=1e-11)
        # size-independent property: smoothed weights are normalised
        assert abs(np.log(np.sum(np.exp(out))) ) < 1e-10


@pytest.mark.parametrize('n,reff', [(200_000, 0.01), (10_000_000, 1.0)])
def test_psislw_large_tail(n, reff):
    """Tails beyond one workgroup's LDS sort (M_t > 8192) take the device radix
    sort: same k, tail order and smoothed weights as the oracle."""
    from viabel_amd import psis
    from oracle import psis_oracle
    rs = np.random.RandomState(7)
    lw = rs.standard_t(4, n) * 1.1
    out, k, tails = psis.psislw_with_tail(lw, Reff=reff)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        oout, ok, otails = psis_oracle.psislw(lw.copy(), Reff=reff, return_tail=True)
    assert len(otails[0]) > 8192
    _close(k, ok, rtol=1e-9)
    np.testing.assert_array_equal(tails[0], otails[0])
    _close(out[:, 0], oout, rtol=1e-11, atol=1e-11)


def test_psislw_tied_values_take_the_radix_path():
    """Log weights on a grid of step 2 (value 8, where the order statistic falls,
    is shared by ~8 500 of the 1e6 draws): the fast select's candidates -- every
    draw at or above the order statistic's 22-bit key prefix -- exceed one
    workgroup's sort, so the call takes the 8-pass radix select.  k equals the
    oracle's; the smoothed weights are compared as a sorted multiset (np.argsort
    orders ties arbitrarily, the device stably)."""
    from viabel_amd import psis
    from oracle import psis_oracle
    rs = np.random.RandomState(11)
    lw = 2.0 * np.round(rs.randn(1_000_000) * 1.5)
    assert np.sum(lw == 8.0) > 8192
    out, k = psis.psislw(lw)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        oout, ok = psis_oracle.psislw(lw.copy())
    _close(k, ok, rtol=1e-9)
    _close(np.sort(out), np.sort(oout), rtol=1e-11, atol=1e-11)


_FAST = '''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from viabel_amd import psis
rs = np.random.RandomState(5)
lw = rs.standard_t(3, (300_000, 6)) * 1.4 - 3.0
out, k, tails = psis.psislw_with_tail(lw)
np.savez(sys.argv[2], out=out, k=k, t0=tails[0], t5=tails[5])
'''


def test_psis_fast_select_equals_radix_select(tmp_path):
    """The two-digit select + candidate sort against the 8-pass radix select
    (VIABEL_AMD_PSIS_FAST_SELECT=0, read once per process: child processes) on 6
    columns: k, smoothed weights and tail orders bit for bit."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for mode in ('0', '1'):
        f = str(tmp_path / ('f%s.npz' % mode))
        env = dict(os.environ, VIABEL_AMD_PSIS_FAST_SELECT=mode)
        r = subprocess.run([sys.executable, '-c', _FAST, root, f], env=env, capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        res[mode] = np.load(f)
    for key in ('out', 'k', 't0', 't5'):
        np.testing.assert_array_equal(res['0'][key], res['1'][key])


def test_gpdfit_large():
    from viabel_amd import psis
    from oracle import psis_oracle
    x = np.random.RandomState(3).pareto(3.0, 20000)
    k, sigma = psis.gpdfitnew(x)
    ok, osigma = psis_oracle.gpdfit(x)[:2]
    _close(k, ok, rtol=1e-10)
    _close(sigma, osigma, rtol=1e-10)


# ---- covariance at any d, PSIS-weighted moments (experiments.py:73-89) -------
@pytest.mark.parametrize('n,d', [(500, 3), (2000, 100), (700, 300)])
@pytest.mark.parametrize('weighted', [False, True])
def test_weighted_covariance_vs_numpy(n, d, weighted):
    """np.cov(x.T, aweights=w, ddof) / np.average: numpy is the reference's own call."""
    from viabel_amd import experiments
    rs = np.random.RandomState(n + d)
    x = rs.randn(n, d) @ (np.eye(d) + 0.1 * rs.randn(d, d)) + rs.randn(d)
    w = rs.rand(n) if weighted else None
    for ddof in (0, 1):
        m, c = experiments.weighted_mean_and_cov(x, w, ddof=ddof)
        np.testing.assert_allclose(m, np.average(x, axis=0, weights=w), rtol=1e-11, atol=1e-12)
        np.testing.assert_allclose(c, np.cov(x.T, aweights=w, ddof=ddof), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize('n,d', [(500, 3), (1_000_000, 2), (700, 300)])
def test_weighted_covariance_log_weights(n, d):
    """Weights from log weights on the device (improve_with_psis,
    experiments.py:80-85): exp(lw - max) normalised, against numpy."""
    from viabel_amd import experiments
    rs = np.random.RandomState(n + d + 1)
    x = rs.randn(n, d) + rs.randn(d)
    lw = rs.randn(n) * 3.0 - 700.0         # exp(lw) alone would underflow
    w = np.exp(lw - lw.max())
    w /= w.sum()
    m, c = experiments.weighted_mean_and_cov(x, log_weights=lw, ddof=0)
    np.testing.assert_allclose(m, np.average(x, axis=0, weights=w), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(c, np.cov(x.T, aweights=w, ddof=0), rtol=1e-9, atol=1e-12)
    with pytest.raises(ValueError, match='weights sum to zero'):
        experiments.weighted_mean_and_cov(x[:10], np.zeros(10))


def test_sumlogs_axis_batched():
    """sumlogs with an axis: all rows in one device call (psis.py:379-395)."""
    from viabel_amd import psis
    from oracle import psis_oracle
    rs = np.random.RandomState(5)
    x = rs.randn(7, 3000, 4) * 20
    for axis in (0, 1, 2):
        _close(psis.sumlogs(x, axis=axis), psis_oracle.sumlogs(x, axis=axis), rtol=1e-13)


def test_all_bounds_samples_wide():
    """all_bounds with raw samples at d > 64 (np.cov on the MFMA GEMM path)."""
    import viabel_amd as va
    from oracle import bounds_oracle
    rs = np.random.RandomState(2)
    lw = rs.randn(4000) * 0.3
    x = rs.randn(4000, 90)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        res = va.all_bounds(lw, samples=x)
        ores = bounds_oracle.all_bounds(lw, samples=x)
    for k in ('W1', 'W2', 'mean_error', 'std_error', 'cov_error', 'd2'):
        np.testing.assert_allclose(res[k], ores[k], rtol=1e-9)


def test_improve_with_psis_vs_oracle():
    from viabel_amd import vb, targets, experiments
    from oracle import vb_oracle, psis_oracle
    D = 4
    fam = vb.mean_field_gaussian_variational_family(D, rng='numpy')
    ofam = vb_oracle.Family('gauss', D)
    lam = np.concatenate([np.zeros(D) + 0.2, np.zeros(D) - 0.1])
    true_mean, true_cov = np.zeros(D), np.eye(D)
    res, m, c = experiments.improve_with_psis(targets.isogauss(D), fam, lam, 20000, true_mean,
                                              true_cov)
    x, lw = vb_oracle.log_weights(ofam, 'isogauss', lam, 20000)
    slw, khat = psis_oracle.psislw(lw.copy())
    slw = slw - np.max(slw)
    wts = np.exp(slw)
    wts /= np.sum(wts)
    om = np.sum(wts[:, None] * x, axis=0)
    oc = np.cov(x.T, aweights=wts, ddof=0)
    np.testing.assert_allclose(m, om, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(c, oc, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(res['khat'], khat, rtol=1e-9)
    np.testing.assert_allclose(res['mean_error'], np.linalg.norm(true_mean - om), rtol=1e-8)


def test_device_resident_chain_matches_host():
    """log weights -> all_bounds -> psislw with the log weights kept in HBM (a
    float64 device tensor) give bitwise the host-array results."""
    import torch
    from viabel_amd import vb, targets, experiments, bounds, psis
    tgt = targets.eight_schools_ncp()
    lam = np.random.RandomState(1).randn(20) * 0.3
    M = 200_000
    fams = [vb.mean_field_t_variational_family(10, 40.0, rng='philox') for _ in range(2)]
    for f in fams:
        f.stream = 4242                      # identical draws for both paths
    _, lw_h = experiments.log_weights(tgt, fams[0], lam, M, return_samples=False)
    lw_d = torch.empty(M, dtype=torch.float64, device='cuda')
    xs, out = experiments.log_weights(tgt, fams[1], lam, M, return_samples=False, lw_out=lw_d)
    assert xs is None and out is lw_d
    np.testing.assert_array_equal(lw_d.cpu().numpy(), lw_h)
    kw = dict(q_var=fams[0].mean_and_cov(lam)[1], moment_bound_fn=lambda p: fams[0].pth_moment(p, lam))
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        bh = bounds.all_bounds(lw_h, **kw)
        bd = bounds.all_bounds(lw_d, **kw)
    assert bh == bd
    oh, kh = psis.psislw(lw_h)
    od, kd = psis.psislw(lw_d)
    assert kd == kh and isinstance(od, torch.Tensor)
    np.testing.assert_array_equal(od.cpu().numpy(), oh)
    with pytest.raises(ValueError):
        experiments.log_weights(tgt, fams[1], lam, M + 1, return_samples=False, lw_out=lw_d)


def test_run_restarts_records_match_host_recomputation():
    """restarts.run_restarts (device-resident bounds stage) == each restart's
    record recomputed with host arrays from the same fitted parameters."""
    from viabel_amd import vb, targets, restarts, experiments, bounds, psis
    fac = lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox')
    tgt = targets.eight_schools_ncp()
    R, iters, M = 3, 40, 30_000
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        tab = restarts.run_restarts(fac, tgt, R, iters, n_samples=50, n_bounds=M)
        assert tab.shape == (R, len(restarts.RECORD_HEAD) + 20)
        for j in range(R):
            r = int(tab[j, 0])
            opt = tab[j, len(restarts.RECORD_HEAD):]
            bfam = fac()
            bfam.stream = (1 << 20) + r
            _, lw = experiments.log_weights(tgt, bfam, opt, M, return_samples=False)
            res = bounds.all_bounds(lw, q_var=bfam.mean_and_cov(opt)[1],
                                    moment_bound_fn=lambda p: bfam.pth_moment(p, opt))
            _, khat = psis.psislw(lw)
            expect = [r, np.mean(lw), res['d2'], res['W1'], res['W2'], res['mean_error'],
                      res['std_error'], res['cov_error'], khat]
            np.testing.assert_allclose(tab[j, :9], expect, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize('scale', [0.001, 1.0])
def test_mean_and_check_mc_error(scale):
    """bounds.py:183-192 on the device: the mean, and the warning exactly when
    the oracle warns."""
    from viabel_amd import bounds
    from oracle import bounds_oracle
    a = np.random.RandomState(4).randn(5000) * scale + 2.0
    with warnings.catch_warnings(record=True) as w1:
        warnings.simplefilter('always')
        m = bounds.mean_and_check_mc_error(a, quantity_name='X')
    with warnings.catch_warnings(record=True) as w2:
        warnings.simplefilter('always')
        om = bounds_oracle.mc_mean(a, 'X')
    _close(m, om, rtol=1e-13)
    assert len(w1) == len(w2) == (1 if scale == 1.0 else 0)


@pytest.mark.parametrize('layout', ['C', 'F', 'device_T'])
def test_psislw_many_columns(layout):
    """All columns of a psislw call run through one column-batched pipeline:
    every column equals the oracle's (k, smoothed weights, tail order), for
    C-ordered, Fortran-ordered and transposed-device-tensor inputs."""
    import torch
    from viabel_amd import psis
    from oracle import psis_oracle
    rs = np.random.RandomState(11)
    n, m = 6000, 37
    cols = []
    for c in range(m):   # light and heavy tails, shifted / scaled columns
        df = [2.5, 4.0, 30.0][c % 3]
        cols.append(rs.standard_t(df, n) * (0.5 + 0.1 * c) + 0.3 * c)
    lw = np.stack(cols, axis=1)          # (n, m)
    if layout == 'C':
        src = lw.copy()
    elif layout == 'F':
        src = np.asfortranarray(lw)
    else:
        src = torch.tensor(lw.T.copy(), dtype=torch.float64, device='cuda').t()
    out, k, tails = psis.psislw_with_tail(src)
    if layout == 'device_T':
        out = out.cpu().numpy()
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        oout, ok, otails = psis_oracle.psislw(lw.copy(), return_tail=True)
    _close(k, ok, rtol=1e-9)
    _close(np.asarray(out), oout, rtol=1e-11, atol=1e-11)
    for t, ot in zip(tails, otails):
        np.testing.assert_array_equal(t, ot)


def test_psislw_many_columns_large_tail():
    """Batched columns whose tails exceed one workgroup's LDS sort (per-column
    device radix sort inside the batched pipeline)."""
    from viabel_amd import psis
    from oracle import psis_oracle
    rs = np.random.RandomState(5)
    n, m = 120_000, 3
    lw = np.asfortranarray(rs.standard_t(4, (n, m)) * 1.1)
    out, k, tails = psis.psislw_with_tail(lw, Reff=0.01)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        oout, ok, otails = psis_oracle.psislw(np.array(lw), Reff=0.01, return_tail=True)
    assert min(len(t) for t in otails) > 8192
    _close(k, ok, rtol=1e-9)
    _close(np.asarray(out), oout, rtol=1e-11, atol=1e-11)
    for t, ot in zip(tails, otails):
        np.testing.assert_array_equal(t, ot)


@pytest.mark.parametrize('device', [False, True])
def test_divergence_rows_matches_per_row(device):
    """bounds.divergence_rows (one batched reduction chain over [rows, M]) equals
    the single-row device divergence bit for bit, and the oracle to 1e-10."""
    import torch
    from viabel_amd import bounds
    from oracle import bounds_oracle as bo
    rs = np.random.RandomState(5)
    rows, M = 7, 30_001
    lw = rs.standard_t(5, size=(rows, M)) * 0.7 - 3.0
    src = torch.from_numpy(lw).cuda() if device else lw
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        div = bounds.divergence_rows(src, alpha=2.0)
        assert div.shape == (rows, 7)
        for r in range(rows):
            one = bounds._device_divergence(lw[r], 2.0, None)
            np.testing.assert_array_equal(div[r], one)
            d2, lnb = bo.divergence_bound(lw[r], return_log_norm_bound=True)
            _close(div[r, 0], d2)
            _close(div[r, 1], lnb)
            res = bounds.all_bounds_from_divergence(div[r], moment_bound_fn=lambda p: 1.0 + p,
                                                    q_var=2.0)
            ref = bounds.all_bounds(lw[r], moment_bound_fn=lambda p: 1.0 + p, q_var=2.0)
            assert res.keys() == ref.keys()
            for k in ref:
                assert res[k] == ref[k], k


@pytest.mark.parametrize('layout', ['1d', 'c', 'f', 'device_t'])
def test_psis_khat_equals_psislw_k(layout):
    """psis_khat (vb_psislw with a null lw_out: the pipeline stops after the GPD
    fit, the shift applied on the fly) gives psislw's k bit for bit."""
    import torch
    from viabel_amd import psis
    rs = np.random.RandomState(5)
    lw = rs.standard_t(3, size=(20000, 4))
    if layout == '1d':
        x = lw[:, 0].copy()
    elif layout == 'c':
        x = np.ascontiguousarray(lw)
    elif layout == 'f':
        x = np.asfortranarray(lw)
    else:
        x = torch.tensor(lw.T.copy(), dtype=torch.float64, device='cuda').t()
    k_full = psis.psislw(x)[1]
    k_only = psis.psis_khat(x)
    np.testing.assert_array_equal(np.atleast_1d(k_only), np.atleast_1d(k_full))
