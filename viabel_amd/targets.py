"""Device target log densities (the model plug-in boundary).

In the reference, ``logdensity`` is an arbitrary autograd-differentiable
callable or ``make_stan_log_density(fit)`` (viabel/vb.py:314-321).  A Python
callable cannot run inside a HIP kernel, so the device path takes targets
from this registry; each carries the kernel-side target id.  Calling a target
evaluates log p(x) for x of shape (N, D) on the GPU, like the reference's
``logdensity(samples)``.

Targets:
  isogauss(D)            N(0, I_D)                                  config 3
  mixture(D)             per-coordinate 0.5 N(-2,1) + 0.5 N(2,1)    normal-mixture.ipynb
  funnel(D)              Neal's funnel, x[1] = log sigma            funnel-distribution.ipynb
  eight_schools_ncp()    eight_schools_ncp.stan log_prob (D = 10)   eight-schools.ipynb
  corr_gauss(D)          N(0, A A^T / D + I), A = RandomState(512).randn(D, D)
                         (full-rank family)
"""
import numpy as np

from . import _native as nat

__all__ = ['Target', 'isogauss', 'mixture', 'funnel', 'eight_schools_ncp', 'corr_gauss']


class Target:
    def __init__(self, kind, dim, name, params=None):
        self.kind, self.dim, self.name = int(kind), int(dim), name
        self.params = None if params is None else nat.as_f64(params)

    @property
    def separable(self):
        return self.kind in (nat.TARGET_ISOGAUSS, nat.TARGET_MIXTURE)

    def _struct(self):
        if self.params is None:
            return nat.Target(self.kind, 0, self.dim, None, 0)
        return nat.Target(self.kind, 0, self.dim, nat.dptr(self.params), self.params.size)

    def logdensity_and_grad(self, x):
        x = nat.as_f64(np.atleast_2d(x))
        if x.shape[1] != self.dim:
            raise ValueError('expected x with %d columns, got %s' % (self.dim, x.shape))
        n = x.shape[0]
        lp = np.empty(n)
        g = np.empty_like(x)
        t = self._struct()
        nat.check(nat.lib().vb_target_logdensity(nat.context().handle, t, nat.dptr(x), n,
                                                 nat.dptr(lp), nat.dptr(g)))
        return lp, g

    def __call__(self, x):
        return self.logdensity_and_grad(x)[0]

    def __repr__(self):
        return 'viabel_amd.targets.%s(D=%d)' % (self.name, self.dim)


def isogauss(dim):
    return Target(nat.TARGET_ISOGAUSS, dim, 'isogauss')


def mixture(dim=1):
    return Target(nat.TARGET_MIXTURE, dim, 'mixture')


def funnel(dim=2):
    if dim < 2:
        raise ValueError('funnel needs dim >= 2')
    return Target(nat.TARGET_FUNNEL, dim, 'funnel')


def eight_schools_ncp():
    return Target(nat.TARGET_EIGHT_SCHOOLS_NCP, 10, 'eight_schools_ncp')


def corr_gauss(dim, seed=512):
    """N(0, Sigma*) with Sigma* = A A^T / dim + I, A = RandomState(seed).randn(dim, dim).
    The precision and log normaliser are formed once here (model set-up); every
    evaluation runs on the device."""
    a = np.random.RandomState(seed).randn(dim, dim)
    sigma = a @ a.T / dim + np.eye(dim)
    prec = np.linalg.inv(sigma)
    prec = 0.5 * (prec + prec.T)
    _, logdet = np.linalg.slogdet(sigma)
    const = -0.5 * logdet - 0.5 * dim * np.log(2 * np.pi)
    t = Target(nat.TARGET_CORR_GAUSS, dim, 'corr_gauss', np.concatenate([prec.ravel(), [const]]))
    t.sigma = sigma
    return t
