"""The reference's own known-answer tests (tests/test_bounds.py:1-70), restated
at its sample size MC_SAMPLES = 1e7 and imported the way its users import:
``from viabel import all_bounds, error_bounds, wasserstein_bounds,
divergence_bound`` -- the drop-in namespace over the device implementation.

Closed forms (Gaussian Renyi / KL divergences, Wasserstein bounds of a
Gaussian) and tolerances (MC_TOL = 5 / sqrt(MC_SAMPLES)) are the reference's;
the draws come from the same numpy seeds (846, 341, 1639) and scipy calls.
This file restates the tests; it does not ship the reference's file.
"""
import numpy as np
import pytest
from scipy.stats import norm

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]

MC_SAMPLES = 10_000_000
MC_TOL = 5 / np.sqrt(MC_SAMPLES)


def gaussian_alpha_divergence(alpha, var1, var2):
    """D_alpha(N(0, var1) | N(0, var2)) in closed form (inf when undefined)."""
    t = alpha * var2 - (alpha - 1) * var1
    if t < 0:
        return np.inf
    return (-0.5 / (alpha - 1) * np.log(t) + .5 * alpha / (alpha - 1) * np.log(var2)
            - .5 * np.log(var1))


def gaussian_kl_divergence(var1, var2):
    return .5 * (var1 / var2 + np.log(var2 / var1) - 1)


def _gaussian_log_weights(seed, var1, var2):
    np.random.seed(seed)
    p1 = norm(scale=np.sqrt(var1))
    p2 = norm(scale=np.sqrt(var2))
    samples = p2.rvs(MC_SAMPLES)
    return samples, p1.logpdf(samples) - p2.logpdf(samples)


@pytest.mark.parametrize('alpha', [1.5, 2, 3])
@pytest.mark.parametrize('elbo', [None, 0])
def test_divergence_bound(alpha, elbo):
    from viabel import divergence_bound
    var1, var2 = 4, 16
    _, log_weights = _gaussian_log_weights(846, var1, var2)
    expected = gaussian_alpha_divergence(alpha, var1, var2)
    if elbo is None:
        expected += alpha / (alpha - 1) * gaussian_kl_divergence(var2, var1)
    np.testing.assert_allclose(divergence_bound(log_weights, alpha, elbo), expected,
                               atol=MC_TOL, rtol=MC_TOL, err_msg='incorrect d2 value')


def test_wasserstein_bounds():
    from viabel import wasserstein_bounds
    np.random.seed(341)
    d2, stdev = 5.0, 3.5
    samples = norm.rvs(scale=stdev, size=MC_SAMPLES)
    res = wasserstein_bounds(d2, samples)
    np.testing.assert_allclose(res['W1'], 2 * stdev * np.sqrt(np.expm1(d2)),
                               rtol=MC_TOL, err_msg='incorrect W1 value')
    np.testing.assert_allclose(res['W2'], 2 * stdev * (3 * np.expm1(d2)) ** 0.25,
                               rtol=MC_TOL, err_msg='incorrect W2 value')


def test_all_bounds():
    from viabel import all_bounds
    var1, var2 = 2.5, 9.3
    samples, log_weights = _gaussian_log_weights(1639, var1, var2)
    res = all_bounds(log_weights, samples, q_var=var2, log_norm_bound=None)
    expected_d2 = (gaussian_alpha_divergence(2, var1, var2)
                   + 2 * gaussian_kl_divergence(var2, var1))
    np.testing.assert_allclose(res['d2'], expected_d2, rtol=MC_TOL, err_msg='incorrect d2 value')
    stdev2 = np.sqrt(var2)
    np.testing.assert_allclose(res['W1'], 2 * stdev2 * np.sqrt(np.expm1(res['d2'])),
                               rtol=MC_TOL, err_msg='incorrect W1 value')
    np.testing.assert_allclose(res['W2'], 2 * stdev2 * (3 * np.expm1(res['d2'])) ** 0.25,
                               rtol=MC_TOL, err_msg='incorrect W2 value')
    assert set(res) == {'W1', 'W2', 'mean_error', 'std_error', 'cov_error', 'd2',
                        'log_norm_bound'}


def test_error_bounds_through_namespace():
    """error_bounds (bounds.py:70-100) from the same namespace: pure algebra."""
    from viabel import error_bounds
    r = error_bounds(W1=1.0, W2=2.0, q_var=4.0)
    assert r['mean_error'] == 1.0 and r['std_error'] == 2.0
    assert r['cov_error'] == pytest.approx(2 * (2.0 * 2.0 + 4.0))
