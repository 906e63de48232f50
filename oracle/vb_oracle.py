"""ORACLE -- TEST INFRASTRUCTURE ONLY.

numpy restatement of the reference's Monte Carlo VI path (viabel/vb.py).
Each function cites the reference lines it follows.  Differences from the
reference are confined to HOW derivatives are obtained (closed forms instead
of autograd's tape) and to computing mean-field log densities in closed form
instead of scipy's dense-covariance mvn.logpdf; both are pinned by
tests/test_oracle_vb.py (torch.autograd fp64 + finite differences).

Noise can be drawn exactly like the reference (numpy legacy RandomState,
same calls in the same order) or injected by the caller (``eps=``), which is
how tests feed the same draws to the oracle and to the HIP kernels.
"""
import math

import numpy as np

from . import targets_oracle

LOG2PI = np.log(2 * np.pi)


class Family:
    """Mean-field Gaussian (vb.py:48-82) or Student-t (vb.py:140-182)."""

    def __init__(self, kind, dim, df=None):
        if kind == 't' and df <= 2:
            raise ValueError('df must be greater than 2')
        self.kind, self.dim, self.df = kind, dim, df
        self.rs = np.random.RandomState(0)          # vb.py:49 / vb.py:143
        self.var_param_dim = 2 * dim

    # standardized draws, in the reference's call order
    def draw(self, n, seed=None):
        rs = self.rs if seed is None else np.random.RandomState(seed)
        if self.kind == 'gauss':
            return rs.randn(n, self.dim)                       # vb.py:57
        return rs.standard_t(self.df, size=(n, self.dim))      # vb.py:151

    def split(self, lam):
        return lam[:self.dim], lam[self.dim:]

    def transform(self, lam, eps):
        mu, ls = self.split(lam)
        if self.kind == 'gauss':
            return eps * np.exp(ls) + mu                       # vb.py:57
        return mu + np.exp(ls) * eps                           # vb.py:151

    def sample(self, lam, n, seed=None):
        return self.transform(lam, self.draw(n, seed))

    def entropy(self, lam):
        _, ls = self.split(lam)
        if self.kind == 'gauss':
            return 0.5 * self.dim * (1.0 + LOG2PI) + np.sum(ls)   # vb.py:61
        return np.sum(ls)                                         # vb.py:156

    def logdensity(self, x, lam):
        """log q(x; lam) with all constants (vb.py:63-65, 158-162)."""
        mu, ls = self.split(lam)
        x = np.atleast_2d(x)
        z = (x - mu) / np.exp(ls)
        if self.kind == 'gauss':
            return np.sum(-0.5 * z * z - ls - 0.5 * LOG2PI, axis=1)
        df = self.df
        c = math.lgamma(0.5 * (df + 1)) - math.lgamma(0.5 * df) - 0.5 * np.log(df * np.pi)
        return np.sum(c - 0.5 * (df + 1) * np.log1p(z * z / df) - ls, axis=1)

    def mean_and_cov(self, lam):
        mu, ls = self.split(lam)
        if self.kind == 'gauss':
            return mu, np.diag(np.exp(2 * ls))                  # vb.py:67-69
        return mu, self.df / (self.df - 2) * np.diag(np.exp(2 * ls))   # vb.py:164-166

    def pth_moment(self, p, lam):
        if p not in [2, 4]:
            raise ValueError('only p = 2 or 4 supported')
        _, ls = self.split(lam)
        if self.kind == 'gauss':                                # vb.py:71-79
            v = np.exp(2 * ls)
            return np.sum(v) if p == 2 else 2 * np.sum(v ** 2) + np.sum(v) ** 2
        if self.df <= p:                                        # vb.py:168-179
            raise ValueError('df must be greater than p')
        s = np.exp(ls)
        c = self.df / (self.df - 2)
        if p == 2:
            return c * np.sum(s ** 2)
        return c ** 2 * (2 * (self.df - 1) / (self.df - 4) * np.sum(s ** 4) + np.sum(s ** 2) ** 2)


def _target(target):
    """A target name of targets_oracle.TARGETS, or a callable x -> (log p, grad)."""
    return target if callable(target) else targets_oracle.TARGETS[target]


def klvi_value_grad(fam, target, lam, n_samples, eps=None):
    """black_box_klvi (vb.py:236-245): value = -(H + mean log p), analytic grad.

    d/dmu = -mean_n g_n ; d/dlog sigma = -(1 + sigma * mean_n g_n * eps_n)."""
    if eps is None:
        eps = fam.draw(n_samples)
    x = fam.transform(lam, eps)
    lp, g = _target(target)(x)
    value = -(fam.entropy(lam) + np.mean(lp))
    _, ls = fam.split(lam)
    gmu = -np.mean(g, axis=0)
    gls = -(1.0 + np.exp(ls) * np.mean(g * eps, axis=0))
    return value, np.concatenate([gmu, gls])


def klvi_pd_value_grad(fam, target, lam, n_samples, eps=None):
    """black_box_klvi_pd / _pd2 (vb.py:268-295): value = -(mean log p - mean log q(x)).
    autograd differentiates log q through x and lambda; for these families the
    total derivative of log q(x(lambda); lambda) is (0, -1) per coordinate, so the
    gradient equals klvi_value_grad's (tests pin this with torch.autograd)."""
    if eps is None:
        eps = fam.draw(n_samples)
    x = fam.transform(lam, eps)
    lp, g = _target(target)(x)
    value = -(np.mean(lp) - np.mean(fam.logdensity(x, lam)))
    _, ls = fam.split(lam)
    gmu = -np.mean(g, axis=0)
    gls = -(1.0 + np.exp(ls) * np.mean(g * eps, axis=0))
    return value, np.concatenate([gmu, gls])


def chivi_value_grad(fam, target, lam, n_samples, alpha, eps=None):
    """black_box_chivi (vb.py:248-266).  The reference draws a fresh seed from the
    GLOBAL numpy RNG each call (vb.py:258) and samples from RandomState(seed).

    grad = alpha/N sum_n w_n d lw_n/d lam with w = exp(lw - max)^alpha;
    d lw_n/d mu = g_n, d lw_n/d log sigma = g_n sigma eps_n + 1 (log q's total
    derivative: its explicit and through-x parts cancel except the -log sigma)."""
    if eps is None:
        seed = np.random.randint(2 ** 32)
        eps = fam.draw(n_samples, seed)
    x = fam.transform(lam, eps)
    lp, g = _target(target)(x)
    lw = lp - fam.logdensity(x, lam)
    log_norm = np.max(lw)
    w = np.exp(lw - log_norm) ** alpha
    value = np.log(np.mean(w)) / alpha + log_norm
    _, ls = fam.split(lam)
    gmu = alpha * np.sum(w[:, None] * g, axis=0) / w.size
    gls = alpha * np.sum(w[:, None] * (g * np.exp(ls) * eps + 1.0), axis=0) / w.size
    return value, np.concatenate([gmu, gls])


def learning_rate_schedule(n_iters, learning_rate, learning_rate_end):
    """vb.py:324-342 (restated)."""
    if learning_rate <= 0:
        raise ValueError('learning rate must be positive')
    if learning_rate_end is not None:
        if learning_rate <= learning_rate_end:
            raise ValueError('initial learning rate must be greater than final learning rate')
        b = n_iters * learning_rate_end / (2 * (learning_rate - learning_rate_end))
        a = learning_rate * b
        lo, hi = n_iters // 4, 3 * n_iters // 4
    out = []
    for i in range(n_iters):
        if learning_rate_end is None or i < lo:
            out.append(learning_rate)
        elif i < hi:
            out.append(a / (b + i - lo + 1))
        else:
            out.append(learning_rate_end)
    return out


def adagrad_optimize(n_iters, objective_and_grad, init_param, window=10,
                     learning_rate=.01, epsilon=.1, learning_rate_end=None, has_log_norm=False):
    """vb.py:345-389.  has_log_norm: the objective returns (value, grad, log_norm)
    and the window's gradients are scaled by exp(min log_norm - log_norm_j)
    (vb.py:365-373)."""
    grads = []
    values = []
    log_norms, local_log_norms = [], []
    lam = init_param.copy()
    hist = []
    for i, lr in enumerate(learning_rate_schedule(n_iters, learning_rate, learning_rate_end)):
        if has_log_norm:
            val, g, ln = objective_and_grad(lam)
        else:
            val, g = objective_and_grad(lam)
            ln = 0
        values.append(val)
        log_norms.append(ln)
        grads.append(g)
        local_log_norms.append(ln)
        if len(grads) > window:
            grads.pop(0)
            local_log_norms.pop(0)
        if has_log_norm:
            scale = np.exp(np.min(local_log_norms) - np.array(local_log_norms))
            acc = np.sum((scale[:, np.newaxis] * np.array(grads)) ** 2, axis=0)
        else:
            acc = np.sum(np.array(grads) ** 2, axis=0)
        lam = lam - lr * g / np.sqrt(epsilon + acc)
        if i >= 3 * n_iters // 4:
            hist.append(lam.copy())
    hist = np.array(hist)
    smoothed = np.mean(hist, axis=0) if len(hist) else np.full(lam.shape, np.nan)
    return smoothed, hist, np.array(values), np.array(log_norms, dtype=float)


def log_weights(fam, target, lam, n_samples, eps=None):
    """experiments.py:60-63: samples from q (continuing fam.rs), lw = log p - log q."""
    if eps is None:
        eps = fam.draw(n_samples)
    x = fam.transform(lam, eps)
    lp, _ = _target(target)(x)
    return x, lp - fam.logdensity(x, lam)
