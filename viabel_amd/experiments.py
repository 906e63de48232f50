"""Log-weight producer of the reference's experiment harness, on the device.

  get_samples_and_log_weights   notebooks/experiments.py:60-63
  psis_correction               notebooks/experiments.py:66-70

Draws continue the family's stream (numpy mode: fam.rs, as the reference's
``var_family.sample(var_param, n_samples)``; philox mode: the family's
counter), then one kernel computes samples and lw = log p(x) - log q(x).
"""
import numpy as np

from . import _native as nat
from .psis import psislw
from .targets import Target

__all__ = ['get_samples_and_log_weights', 'psis_correction', 'log_weights']


def log_weights(logdensity, var_family, var_param, n_samples, return_samples=True):
    if not isinstance(logdensity, Target):
        raise TypeError('log weights on the device need a viabel_amd.targets target')
    lam = nat.as_f64(var_param)
    m = int(n_samples)
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


def get_samples_and_log_weights(logdensity, var_family, var_param, n_samples):
    return log_weights(logdensity, var_family, var_param, n_samples, True)


def psis_correction(logdensity, var_family, var_param, n_samples):
    samples, lw = get_samples_and_log_weights(logdensity, var_family, var_param, n_samples)
    smoothed_log_weights, khat = psislw(lw)
    return samples.T, smoothed_log_weights, khat
