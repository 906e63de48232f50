"""Divergence, Wasserstein and moment-error bounds (viabel.bounds API).

Mirrors viabel/bounds.py (names, signatures, dict keys, ValueError and
Monte-Carlo-error warning texts).  The O(n) and O(n d) passes over log
weights and samples run in libviabel_amd.so (vb_divergence_bound,
vb_centered_moments, vb_covariance); what remains here is O(1) scalar
algebra on their results, plus the spectral norm of a (d x d) covariance
(d <= 64), which is O(d^3) on a matrix the device already reduced.
"""
from warnings import warn

import numpy as np

from . import _native as nat

__all__ = [
    'all_bounds',
    'error_bounds',
    'wasserstein_bounds',
    'divergence_bound'
]   # bounds.py:5-10 (mean_and_check_mc_error and the *_bound helpers are module-level, as there)


def _mc_warning(m, s, quantity_name, atol=0.01, rtol=0.0):
    """bounds.py:183-192 (the check; the mean and s.e. come from the device)."""
    if s > rtol * np.abs(m) + atol:
        msg = 'significant Monte Carlo error'
        if quantity_name is not None:
            msg += ' when computing ' + quantity_name
        msg += ' (mean = {}, standard deviation = {})'.format(m, s)
        warn(msg)


def mean_and_check_mc_error(a, atol=0.01, rtol=0.0, quantity_name=None):
    """bounds.py:183-192: mean of `a` with a warning when its Monte Carlo
    standard error std(a) / sqrt(n) exceeds rtol |mean| + atol (the mean and
    standard error come from the device reduction of vb_divergence_bound)."""
    out = _device_divergence(a, 2.0, None)
    m, s = out[4], out[5]
    _mc_warning(m, s, quantity_name, atol=atol, rtol=rtol)
    return m


def _device_divergence(log_weights, alpha, log_norm_bound):
    lw = nat.device_tensor(log_weights)   # HBM-resident log weights are read in place
    if lw is None:
        lw = nat.as_f64(np.ravel(np.asarray(log_weights)))
    else:
        lw = lw.reshape(-1)
    out = np.empty(7)
    has = log_norm_bound is not None
    nat.check(nat.lib().vb_divergence_bound(nat.context().handle, nat.dptr(lw), int(lw.numel()
                                            if hasattr(lw, 'numel') else lw.size),
                                            float(alpha), int(has),
                                            float(log_norm_bound) if has else 0.0,
                                            nat.dptr(out)))
    return out


def all_bounds(log_weights, samples=None, moment_bound_fn=None,
               q_var=None, p_var=None, log_norm_bound=None):
    """bounds.py:13-61: dict with W1, W2, mean_error, std_error, cov_error, d2,
    log_norm_bound."""
    d2, log_norm_bound = divergence_bound(log_weights,
                                          log_norm_bound=log_norm_bound,
                                          return_log_norm_bound=True)
    results = wasserstein_bounds(d2, samples, moment_bound_fn)
    if q_var is None and samples is not None:
        q_var = _sample_cov(samples)
    results.update(error_bounds(q_var=q_var, p_var=p_var, **results))
    results['d2'] = d2
    results['log_norm_bound'] = log_norm_bound
    return results


def _sample_cov(samples):
    """np.cov(samples.T) (ddof=1) on the device; scalar for 1-D samples."""
    x = np.asarray(samples, dtype=float)
    one_d = x.ndim == 1
    x = nat.as_f64(x.reshape(x.shape[0], -1))
    n, d = x.shape
    cov = np.empty((d, d))
    nat.check(nat.lib().vb_covariance(nat.context().handle, nat.dptr(x), n, d, None,
                                      nat.dptr(cov)))
    return np.array(cov[0, 0]) if one_d else cov


def _compute_norm_if_needed(var):
    """bounds.py:64-67: spectral norm of a covariance matrix."""
    if np.asarray(var).ndim == 2:
        v = np.asarray(var, dtype=float)
        if np.count_nonzero(v - np.diag(np.diagonal(v))) == 0:
            return np.max(np.abs(np.diagonal(v)))     # diagonal: largest |entry|
        return np.linalg.norm(v, ord=2)
    return var


def error_bounds(W1=np.inf, W2=np.inf, q_var=np.inf, p_var=np.inf):
    """bounds.py:70-100."""
    results = dict()
    results['mean_error'] = mean_bound(min(W1, W2))
    results['std_error'] = std_bound(W2)
    results['cov_error'] = var_bound(W2, _compute_norm_if_needed(q_var),
                                     _compute_norm_if_needed(p_var))
    return results


def wasserstein_bounds(d2, samples=None, moment_bound_fn=None):
    """bounds.py:103-139: W1, W2 from d2 and 2p-th central moments."""
    results = dict()
    if moment_bound_fn is None:
        if samples is None:
            raise ValueError('must provides samples if moment_bound_fn not given')
        x = np.asarray(samples, dtype=float)
        if x.ndim == 1:
            x = x[:, np.newaxis]
        x = nat.as_f64(x)
        c2, c4 = np.empty(1), np.empty(1)
        nat.check(nat.lib().vb_centered_moments(nat.context().handle, nat.dptr(x), x.shape[0],
                                                x.shape[1], nat.dptr(c2), nat.dptr(c4)))
        moments = {2: c2[0], 4: c4[0]}
        moment_bound_fn = moments.__getitem__
    for p in [1, 2]:
        Cp = moment_bound_fn(2 * p)
        results['W{}'.format(p)] = 2 * Cp ** (.5 / p) * np.expm1(d2) ** (.5 / p)
    return results


def divergence_bound(log_weights, alpha=2., log_norm_bound=None,
                     return_log_norm_bound=False):
    """bounds.py:142-180: bound on the alpha-divergence (CUBO - ELBO)."""
    if alpha <= 1:
        raise ValueError('alpha must be greater than 1')
    out = _device_divergence(log_weights, alpha, log_norm_bound)
    dalpha, lnb, mean_r, se_r, mean_lw, se_lw = out[:6]
    _mc_warning(mean_r, se_r, 'CUBO')
    if log_norm_bound is None:
        _mc_warning(mean_lw, se_lw, 'ELBO')
        log_norm_bound = lnb
    if return_log_norm_bound:
        return dalpha, log_norm_bound
    return dalpha


def divergence_rows(log_weights, alpha=2.):
    """Device divergence statistics of every row of a [rows, M] log-weight matrix
    (HBM tensor or array) in one launch chain: ndarray [rows, 7] of (d_alpha,
    elbo, mean_r, se_r, mean_lw, se_lw, log max) per row, the values
    `divergence_bound` derives its result and warnings from."""
    if alpha <= 1:
        raise ValueError('alpha must be greater than 1')
    lw = nat.device_tensor(log_weights)
    if lw is None:
        lw = nat.as_f64(np.atleast_2d(np.asarray(log_weights, dtype=float)))
        rows, n = lw.shape
        ld = n
    else:
        if lw.dim() == 1:
            lw = lw.reshape(1, -1)
        rows, n = lw.shape
        if lw.stride(1) != 1:
            lw = lw.contiguous()
        ld = lw.stride(0)
    out = np.empty((rows, 7))
    nat.check(nat.lib().vb_divergence_bound_rows(nat.context().handle, nat.dptr(lw), int(rows),
                                                 int(n), int(ld), float(alpha), 0, 0.0,
                                                 nat.dptr(out)))
    return out


def all_bounds_from_divergence(div7, moment_bound_fn, q_var=None, p_var=None):
    """`all_bounds(log_weights, moment_bound_fn=..., q_var=...)` (bounds.py:13-61)
    from one row of `divergence_rows` (same warnings, same dict)."""
    d2, lnb, mean_r, se_r, mean_lw, se_lw = div7[:6]
    _mc_warning(mean_r, se_r, 'CUBO')
    _mc_warning(mean_lw, se_lw, 'ELBO')
    results = wasserstein_bounds(d2, None, moment_bound_fn)
    results.update(error_bounds(q_var=q_var, p_var=p_var, **results))
    results['d2'] = d2
    results['log_norm_bound'] = lnb
    return results


_var_bound_const_1 = 2 * np.sqrt(2)
_var_bound_const_2 = 1 + 3 * np.sqrt(2)


def mean_bound(Wp):
    return Wp


def std_bound(W2):
    return W2


def var_bound(W2, var1, var2=None):
    if var2 is not None:
        min_var = np.min([var1, var2], axis=0)
    else:
        min_var = var1
    min_std = np.sqrt(min_var)
    return 2 * (min_std * W2 + W2 ** 2)
