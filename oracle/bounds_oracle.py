"""ORACLE -- TEST INFRASTRUCTURE ONLY.

numpy restatement of viabel/bounds.py (divergence, Wasserstein and moment
error bounds).  Pinned against golden outputs of the reference module
(tests/golden/bounds_golden.npz, tests/test_oracle_golden.py).
"""
from warnings import warn

import numpy as np


def mc_mean(a, quantity, atol=0.01, rtol=0.0):
    """bounds.py:183-192: mean with a Monte Carlo standard-error warning."""
    m = np.mean(a)
    se = np.std(a) / np.sqrt(a.size)
    if se > rtol * np.abs(m) + atol:
        warn('significant Monte Carlo error when computing {} (mean = {}, '
             'standard deviation = {})'.format(quantity, m, se))
    return m


def divergence_bound(lw, alpha=2., log_norm_bound=None, return_log_norm_bound=False):
    """bounds.py:142-180."""
    if alpha <= 1:
        raise ValueError('alpha must be greater than 1')
    lw = np.asarray(lw)
    top = np.max(lw)
    cubo = np.log(mc_mean(np.exp(lw - top) ** alpha, 'CUBO')) / alpha + top
    if log_norm_bound is None:
        log_norm_bound = mc_mean(lw, 'ELBO')
    d = alpha / (alpha - 1) * (cubo - log_norm_bound)
    return (d, log_norm_bound) if return_log_norm_bound else d


def wasserstein_bounds(d2, samples=None, moment_bound_fn=None):
    """bounds.py:103-139."""
    if moment_bound_fn is None:
        if samples is None:
            raise ValueError('must provides samples if moment_bound_fn not given')
        xs = np.asarray(samples)
        if xs.ndim == 1:
            xs = xs[:, None]
        xc = xs - xs.mean(axis=0, keepdims=True)

        def moment_bound_fn(p):
            return np.mean(np.sum(xc ** p, axis=1))
    out = {}
    for p in (1, 2):
        out['W%d' % p] = 2 * moment_bound_fn(2 * p) ** (.5 / p) * np.expm1(d2) ** (.5 / p)
    return out


def spectral_norm(v):
    """bounds.py:64-67."""
    return np.linalg.norm(v, ord=2) if np.asarray(v).ndim == 2 else v


def error_bounds(W1=np.inf, W2=np.inf, q_var=np.inf, p_var=np.inf):
    """bounds.py:70-100 with mean/std/var_bound (195-213) inlined."""
    qv, pv = spectral_norm(q_var), spectral_norm(p_var)
    min_var = np.min([qv, pv], axis=0) if pv is not None else qv
    return {'mean_error': min(W1, W2),
            'std_error': W2,
            'cov_error': 2 * (np.sqrt(min_var) * W2 + W2 ** 2)}


def all_bounds(lw, samples=None, moment_bound_fn=None, q_var=None, p_var=None,
               log_norm_bound=None):
    """bounds.py:13-61."""
    d2, lnb = divergence_bound(lw, log_norm_bound=log_norm_bound, return_log_norm_bound=True)
    res = wasserstein_bounds(d2, samples, moment_bound_fn)
    if q_var is None and samples is not None:
        q_var = np.cov(samples.T)
    res.update(error_bounds(q_var=q_var, p_var=p_var, **res))
    res['d2'] = d2
    res['log_norm_bound'] = lnb
    return res
