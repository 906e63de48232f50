"""Log-weight producer of the reference's experiment harness, on the device.

  check_accuracy                notebooks/experiments.py:26-48 (host algebra on d x d)
  check_approx_accuracy         notebooks/experiments.py:51-55
  get_samples_and_log_weights   notebooks/experiments.py:60-63
  psis_correction               notebooks/experiments.py:66-70
  improve_with_psis             notebooks/experiments.py:73-89

Draws continue the family's stream (numpy mode: fam.rs, as the reference's
``var_family.sample(var_param, n_samples)``; philox mode: the family's
counter), then one kernel computes samples and lw = log p(x) - log q(x).
"""
import numpy as np

from . import _native as nat
from .psis import psislw
from .targets import Target

__all__ = ['print_bounds', 'plot_history', 'plot_approx_and_exact_contours',
           'plot_dist_to_opt_param', 'run_experiment', 'get_samples_and_log_weights', 'psis_correction', 'log_weights', 'log_weights_rows', 'check_accuracy',
           'check_approx_accuracy', 'improve_with_psis', 'weighted_mean_and_cov']


def log_weights(logdensity, var_family, var_param, n_samples, return_samples=True,
                lw_out=None):
    """(samples [m, D] or None, lw [m]).  `lw_out`: a float64 device tensor of m
    entries to write the log weights into (they stay in HBM for the bounds /
    PSIS calls that follow)."""
    if not isinstance(logdensity, Target):
        raise TypeError('log weights on the device need a viabel_amd.targets target')
    logdensity = logdensity.bind(var_family.dim)
    lam = nat.as_f64(var_param)
    m = int(n_samples)
    if lw_out is not None:
        lw = nat.device_tensor(lw_out)
        if lw is None or lw.numel() != m:
            raise ValueError('lw_out must be a float64 device tensor of n_samples entries')
    else:
        lw = np.empty(m)
    xs = np.empty((m, var_family.dim)) if return_samples else None
    if var_family.rng == 'numpy':
        eps = nat.as_f64(var_family._draw(m))
        nz = nat.Noise(nat.NOISE_HOST, 0, 0, 0, nat.dptr(eps))
    else:
        nz = var_family._philox_noise()
    nat.check(nat.lib().vb_log_weights(nat.context().handle, var_family._struct(),
                                       logdensity._struct(), nat.dptr(lam), m, nz,
                                       nat.dptr(lw), nat.dptr(xs)))
    return xs, lw


def log_weights_rows(logdensity, var_family, var_params, n_samples, stream, stream_stride=1,
                     seed=None, lw_out=None):
    """log_weights for many parameter vectors of one mean-field family at once
    (the restart loop of vb.py:417-421 followed by experiments.py:60-63 per
    restart): var_params [R, 2D]; row r draws n_samples Philox draws from stream
    `stream + r * stream_stride` (key `seed`, default the family's), one device
    launch.  Returns lw [R, n_samples] (lw_out: a float64 device tensor of that
    shape to write into, kept in HBM for the bounds / PSIS calls)."""
    if not isinstance(logdensity, Target):
        raise TypeError('log weights on the device need a viabel_amd.targets target')
    logdensity = logdensity.bind(var_family.dim)
    lams = nat.as_f64(np.atleast_2d(var_params))
    R, m = lams.shape[0], int(n_samples)
    if lw_out is not None:
        lw = nat.device_tensor(lw_out)
        if lw is None or tuple(lw.shape) != (R, m) or not lw.is_contiguous():
            raise ValueError('lw_out must be a contiguous float64 device tensor of shape (R, n_samples)')
    else:
        lw = np.empty((R, m))
    key = var_family.seed if seed is None else int(seed) & 0xFFFFFFFFFFFFFFFF
    nz = nat.Noise(nat.NOISE_PHILOX, int(stream) & 0xFFFFFF, key, 0, None, int(stream_stride))
    nat.check(nat.lib().vb_log_weights_rows(nat.context().handle, var_family._struct(),
                                            logdensity._struct(), nat.dptr(lams), R, m, nz,
                                            nat.dptr(lw)))
    return lw


def get_samples_and_log_weights(logdensity, var_family, var_param, n_samples):
    return log_weights(logdensity, var_family, var_param, n_samples, True)


def psis_correction(logdensity, var_family, var_param, n_samples):
    samples, lw = get_samples_and_log_weights(logdensity, var_family, var_param, n_samples)
    smoothed_log_weights, khat = psislw(lw)
    return samples.T, smoothed_log_weights, khat


def weighted_mean_and_cov(samples, weights=None, ddof=1, log_weights=None):
    """Device np.average(samples.T, axis=1, weights) and np.cov(samples.T,
    aweights=weights, ddof=ddof) for samples [n, d].  `log_weights` instead of
    `weights`: the weights are exp(log_weights - max), formed on the device."""
    x = nat.as_f64(np.atleast_2d(np.asarray(samples, dtype=float).T).T)
    n, d = x.shape
    mean = np.empty(d)
    cov = np.empty((d, d))
    if log_weights is not None:
        if weights is not None:
            raise ValueError('give weights or log_weights, not both')
        lw = nat.as_f64(np.ravel(log_weights))
        nat.check(nat.lib().vb_weighted_covariance_logw(nat.context().handle, nat.dptr(x), n, d,
                                                        nat.dptr(lw), int(ddof), nat.dptr(mean),
                                                        nat.dptr(cov)))
        return mean, cov
    w = None if weights is None else nat.as_f64(np.ravel(weights))
    nat.check(nat.lib().vb_weighted_covariance(nat.context().handle, nat.dptr(x), n, d,
                                               nat.dptr(w), int(ddof), nat.dptr(mean),
                                               nat.dptr(cov)))
    return mean, cov


def print_bounds(results):
    """experiments.py:14-21: the bounds table of an all_bounds result."""
    print('Bounds on...')
    for label, key in (('2-Wasserstein  ', 'W2'), ('2-divergence   ', 'd2'),
                       ('mean error     ', 'mean_error'), ('stdev error    ', 'std_error')):
        print('  {} {:.3g}'.format(label, results[key]))
    print('  sqrt cov error  {:.3g}'.format(np.sqrt(results['cov_error'])))
    print('  cov error       {:.3g}'.format(results['cov_error']))


def _out_of_scope(name):
    def f(*args, **kwargs):
        raise NotImplementedError('%s (notebooks/experiments.py plotting / reporting harness) is '
                                  'out of scope for viabel_amd' % name)
    f.__name__ = name
    f.__doc__ = 'Importable stand-in for notebooks/experiments.py:%s; raises NotImplementedError.' % name
    return f


plot_history = _out_of_scope('plot_history')                                     # :113-124
plot_approx_and_exact_contours = _out_of_scope('plot_approx_and_exact_contours')  # :94-110
plot_dist_to_opt_param = _out_of_scope('plot_dist_to_opt_param')                 # :127-135
run_experiment = _out_of_scope('run_experiment')                                 # :183-212


def check_accuracy(true_mean, true_cov, approx_mean, approx_cov, verbose=False, method=None):
    """experiments.py:26-48: error summaries of an approximate mean / covariance."""
    true_std = np.sqrt(np.diag(true_cov))
    approx_std = np.sqrt(np.diag(approx_cov))
    results = dict(mean_error=np.linalg.norm(true_mean - approx_mean),
                   cov_error_2=np.linalg.norm(true_cov - approx_cov, ord=2),
                   cov_norm_2=np.linalg.norm(true_cov, ord=2),
                   cov_error_nuc=np.linalg.norm(true_cov - approx_cov, ord='nuc'),
                   cov_norm_nuc=np.linalg.norm(true_cov, ord='nuc'),
                   std_error=np.linalg.norm(true_std - approx_std),
                   rel_std_error=np.linalg.norm(approx_std / true_std - 1))
    if method is not None:
        results['method'] = method
    if verbose:
        print('mean   =', approx_mean)
        print('stdevs =', approx_std)
        print()
        print('mean error             = {:.3g}'.format(results['mean_error']))
        print('stdev error            = {:.3g}'.format(results['std_error']))
        print('||cov error||_2^{{1/2}}  = {:.3g}'.format(np.sqrt(results['cov_error_2'])))
        print('||true cov||_2^{{1/2}}   = {:.3g}'.format(np.sqrt(results['cov_norm_2'])))
    return results


def check_approx_accuracy(var_family, var_param, true_mean, true_cov, verbose=False, name=None):
    """experiments.py:51-55: check_accuracy of the family's (mean, cov) at var_param."""
    return check_accuracy(true_mean, true_cov, *var_family.mean_and_cov(var_param), verbose, name)


def improve_with_psis(logdensity, var_family, var_param, n_samples, true_mean, true_cov,
                      transform=None, verbose=False):
    """experiments.py:73-89: PSIS-reweighted mean and covariance (ddof 0) of
    n_samples draws from q; the draws, log weights, PSIS and the weighted
    moments run on the device (a user `transform` runs on the host)."""
    samples, slw, khat = psis_correction(logdensity, var_family, var_param, n_samples)
    if verbose:
        print('khat = {:.3g}'.format(khat))
        print()
    if transform is not None:
        samples = transform(samples)
    # weights exp(slw - max slw) / sum (experiments.py:80-82) are formed on the device
    approx_mean, approx_cov = weighted_mean_and_cov(np.asarray(samples).T, log_weights=slw,
                                                    ddof=0)
    res = check_accuracy(true_mean, true_cov, approx_mean, approx_cov, verbose)
    res['khat'] = khat
    return res, approx_mean, approx_cov
