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

User models (the reference's make_stan_log_density, vb.py:314-321, and autograd
callables): callback(fn, D), from_stan(fit, D) and torch_target(f, D) evaluate
the model on the HOST once per optimisation step on the whole batch of samples
(VB_TARGET_CALLBACK); sampling, weights, gradient reductions and the optimiser
stay on the device.  This is the model boundary, not a fallback of the VI
computation: the model is the user's code and runs where that code runs.
"""
import numpy as np

from . import _native as nat

__all__ = ['Target', 'isogauss', 'mixture', 'funnel', 'eight_schools_ncp', 'corr_gauss',
           'callback', 'from_stan', 'torch_target', 'as_target']


class Target:
    def __init__(self, kind, dim, name, params=None):
        # dim None: a user model whose dimension is taken from the variational
        # family it is used with (like the reference's make_stan_log_density)
        self.kind, self.dim, self.name = int(kind), None if dim is None else int(dim), name
        self.params = None if params is None else nat.as_f64(params)

    def bind(self, dim):
        """This target for dimension `dim` (a copy when the dimension was left open)."""
        if self.dim is None:
            import copy
            t = copy.copy(self)
            t.dim = int(dim)
            return t
        return self

    _cfunc = None   # ctypes callback of a host target (kept alive with the target)

    @property
    def separable(self):
        return self.kind in (nat.TARGET_ISOGAUSS, nat.TARGET_MIXTURE)

    def _struct(self):
        cb = self._cfunc if self._cfunc is not None else nat.TARGET_CALLBACK_T()
        if self.params is None:
            return nat.Target(self.kind, 0, self.dim, None, 0, cb, None)
        return nat.Target(self.kind, 0, self.dim, nat.dptr(self.params), self.params.size, cb, None)

    def logdensity_and_grad(self, x):
        x = nat.as_f64(np.atleast_2d(x))
        if self.dim is None:
            return self.bind(x.shape[1]).logdensity_and_grad(x)
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


def callback(logdensity_and_grad, dim=None, name='callback'):
    """A user model: logdensity_and_grad(x) -> (log p (n,), d log p / dx (n, d)) for
    x of shape (n, dim) (numpy, host).  dim None: the dimension of the family
    the target is used with."""

    def _cb(user, xp, n, d, lpp, gp):
        try:
            x = np.ctypeslib.as_array(xp, shape=(n, d)).copy()
            lp, g = logdensity_and_grad(x)
            np.ctypeslib.as_array(lpp, shape=(n,))[:] = np.asarray(lp, dtype=float).reshape(n)
            np.ctypeslib.as_array(gp, shape=(n, d))[:] = np.asarray(g, dtype=float).reshape(n, d)
            return 0
        except BaseException as e:          # re-raised by _native.check after the call
            nat.PENDING_CALLBACK_ERRORS.append(e)
            return 1

    t = Target(nat.TARGET_CALLBACK, dim, name)
    t._cfunc = nat.TARGET_CALLBACK_T(_cb)
    t.fn = logdensity_and_grad
    return t


def from_stan(fitobj, dim=None):
    """make_stan_log_density (vb.py:314-321): log_prob / grad_log_prob of a fitted
    Stan model (pystan 2 fit object), applied row by row on the host."""
    def f(x):
        lp = np.array([fitobj.log_prob(row) for row in x])
        g = np.array([fitobj.grad_log_prob(row) for row in x])
        return lp, g
    return callback(f, dim, 'stan')


def torch_target(logdensity, dim=None, device=None):
    """A model written in torch: logdensity(x: tensor (n, dim)) -> (n,); the
    gradient comes from torch.autograd (on `device`, default the GPU when present)."""
    import torch
    dev = torch.device(device if device is not None else ('cuda' if torch.cuda.is_available() else 'cpu'))

    def f(x):
        xt = torch.tensor(x, dtype=torch.float64, device=dev, requires_grad=True)
        lp = logdensity(xt)
        g, = torch.autograd.grad(lp.sum(), xt)
        return lp.detach().cpu().numpy(), g.cpu().numpy()
    return callback(f, dim, 'torch')


def as_target(logdensity, dim):
    """The reference accepts any differentiable callable as logdensity
    (vb.py:236-241, 249-253).  A device target passes through; a plain callable
    that torch can differentiate (logdensity(x: tensor (n, dim)) -> tensor (n,)
    with a grad_fn) is wrapped with torch_target; anything else -- e.g. an
    autograd.numpy function, whose derivatives only autograd can take -- raises
    TypeError."""
    if isinstance(logdensity, Target):
        return logdensity
    msg = ('logdensity must be a viabel_amd.targets target, a user model wrapped with '
           'targets.callback / targets.from_stan, or a callable that torch can differentiate '
           '(x: tensor (n, dim) -> tensor (n,)); got %r' % (logdensity,))
    if not callable(logdensity) or dim is None:
        raise TypeError(msg)
    try:
        import torch
        dev = torch.device('cuda' if torch.cuda.is_available() else 'cpu')
        x = torch.zeros((2, int(dim)), dtype=torch.float64, device=dev, requires_grad=True)
        out = logdensity(x)
        ok = (isinstance(out, torch.Tensor) and out.requires_grad and tuple(out.shape) == (2,))
    except Exception as e:       # the probe failed: not a torch-differentiable callable
        raise TypeError(msg + ' (probe: %s: %s)' % (type(e).__name__, e)) from None
    if not ok:
        raise TypeError(msg)
    return torch_target(logdensity, int(dim))
