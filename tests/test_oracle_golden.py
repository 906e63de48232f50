"""Pin the oracle to the reference: bounds_oracle / psis_oracle against golden
vectors produced by the reference's own bounds.py / psis.py
(tests/golden/make_golden.py), and numpy legacy RNG streams against golden
draws.  CPU only."""
import warnings

import numpy as np
import pytest
from scipy.special import factorial2
from scipy.stats import norm

from oracle import bounds_oracle, psis_oracle

from tests.golden.make_golden import mixture_inputs, gauss_ratio_inputs


def _close(a, b, rtol=1e-12, atol=1e-14):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


class TestBoundsGolden:
    def test_normal_mixture_notebook(self, golden):
        g = golden['bounds']
        samples, lw, q_var = mixture_inputs()
        mb = lambda order: factorial2(order - 1) ** (1 / order) * np.sqrt(q_var)
        cases = {
            'mix_a': bounds_oracle.all_bounds(lw, samples),
            'mix_b': bounds_oracle.all_bounds(lw, samples, q_var=q_var, log_norm_bound=0),
            'mix_c': bounds_oracle.all_bounds(lw, moment_bound_fn=mb, q_var=q_var),
        }
        for cname, res in cases.items():
            for k, v in res.items():
                _close(v, g['%s_%s' % (cname, k)])
        # normal-mixture.ipynb recorded outputs (3 s.f.): W2 6.08, d2 0.768, cov 101
        a = cases['mix_a']
        assert '%.3g' % a['W2'] == '6.08' and '%.3g' % a['d2'] == '0.768'
        assert '%.3g' % a['cov_error'] == '101'

    @pytest.mark.parametrize('alpha', [1.5, 2.0, 3.0])
    @pytest.mark.parametrize('elbo', [None, 0.0])
    def test_divergence(self, golden, alpha, elbo):
        g = golden['bounds']
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            d, lnb = bounds_oracle.divergence_bound(g['div_lw'], alpha, elbo,
                                                    return_log_norm_bound=True)
        tag = 'div_a%g_%s' % (alpha, 'none' if elbo is None else 'zero')
        _close([d, lnb], g[tag])

    def test_wasserstein(self, golden):
        g = golden['bounds']
        for tag, s in (('w1d', g['w_s1']), ('w3d', g['w_s3'])):
            r = bounds_oracle.wasserstein_bounds(5.0, s)
            _close([r['W1'], r['W2']], g[tag])

    def test_all_bounds_cov(self, golden):
        g = golden['bounds']
        r = bounds_oracle.all_bounds(g['ab3_lw'], g['w_s3'])
        for k, v in r.items():
            _close(v, g['ab3_' + k])

    def test_warning_text(self, golden):
        g = golden['bounds']
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter('always')
            bounds_oracle.divergence_bound(g['warn_lw'])
        assert [str(x.message) for x in w] == list(g['warn_msgs'])

    def test_errors(self):
        with pytest.raises(ValueError, match='alpha must be greater than 1'):
            bounds_oracle.divergence_bound(np.zeros(3), alpha=1.0)
        with pytest.raises(ValueError, match='must provides samples'):
            bounds_oracle.wasserstein_bounds(1.0)


class TestPsisGolden:
    @pytest.mark.parametrize('case', ['normal1000', 't3_1000', 'n5', 'n128', 'heavy2e4', 'cols'])
    def test_psislw(self, golden, case):
        g = golden['psis']
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            out, k = psis_oracle.psislw(g[case + '_in'].copy())
        _close(out, g[case + '_out'], rtol=1e-12, atol=1e-12)
        _close(np.atleast_1d(k), g[case + '_k'])

    def test_gpdfit_quadrature(self, golden):
        g = golden['psis']
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            k, sigma, ks, w = psis_oracle.gpdfit(g['gpd_x'].copy(), return_quadrature=True)
        _close([k, sigma], g['gpd_k'])
        _close(ks, g['gpd_ks'])
        _close(w, g['gpd_w'])

    def test_gpinv(self, golden):
        g = golden['psis']
        p = g['gpinv_p']
        for tag, (kk, ss) in {'gpinv_pos': (0.4, 1.3), 'gpinv_neg': (-0.3, 2.0),
                              'gpinv_zero': (1e-18, 0.7), 'gpinv_badsig': (0.2, -1.0)}.items():
            np.testing.assert_allclose(psis_oracle.gpinv(p, kk, ss), g[tag], rtol=1e-14)
        np.testing.assert_allclose(psis_oracle.gpinv(np.array([0.1, 0.5, 0.9]), 0.4, 1.3),
                                   g['gpinv_open'], rtol=1e-14)

    def test_sumlogs(self, golden):
        g = golden['psis']
        _close(psis_oracle.sumlogs(g['sumlogs_x']), g['sumlogs'][0])

    def test_errors(self):
        with pytest.raises(ValueError, match='More than one log-weight'):
            psis_oracle.psislw(np.zeros(1))
        with pytest.raises(ValueError, match='Invalid input array'):
            psis_oracle.gpdfit(np.zeros(1))


class TestNumpyStreams:
    """The reference's draws: numpy legacy RandomState calls (vb.py:49, 57, 151,
    204-206, 258) are frozen by numpy's stream-compatibility policy."""

    def test_family_draws(self, golden):
        g = golden['rng']
        np.testing.assert_array_equal(np.random.RandomState(0).randn(4, 5), g['randn_4x5'])
        np.testing.assert_array_equal(np.random.RandomState(0).standard_t(40, size=(4, 5)),
                                      g['t40_4x5'])
        rs = np.random.RandomState(0)
        np.testing.assert_array_equal(rs.chisquare(100, 4), g['chisq100_4'])
        np.testing.assert_array_equal(rs.randn(4, 3), g['randn_after_chisq_4x3'])

    def test_global_seed_draws(self, golden):
        np.random.seed(0)
        got = [np.random.randint(2 ** 32) for _ in range(3)]
        np.testing.assert_array_equal(got, golden['rng']['global_randint'])

    def test_chunked_draws_equal_per_step_draws(self):
        """adagrad streams C steps of noise with one call; the reference makes
        one randn(N, D) call per step.  The legacy stream (incl. the cached
        second Box-Muller value) makes these identical."""
        a = np.random.RandomState(0)
        b = np.random.RandomState(0)
        per_step = np.concatenate([a.randn(7, 3) for _ in range(5)])
        np.testing.assert_array_equal(per_step, b.randn(35, 3))
        a = np.random.RandomState(1)
        b = np.random.RandomState(1)
        per_step = np.concatenate([a.standard_t(40, size=(7, 3)) for _ in range(5)])
        np.testing.assert_array_equal(per_step, b.standard_t(40, size=(35, 3)))
