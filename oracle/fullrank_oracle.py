"""ORACLE -- TEST INFRASTRUCTURE ONLY.

numpy/scipy restatement of the full-rank Student-t family
(t_variational_family, viabel/vb.py:185-233, and multivariate_t_logpdf,
viabel/_distributions.py:8-38) with its KLVI / CHIVI value and gradient.

Free parametrisation (paragami PSDSymmetricMatrixPattern, diag_lb = 0, the
helpers copied in viabel/functions.py:88-136): lambda = [mu (D), tril(M)] with
tril in row-major lower-triangle order (index k2 + k1 (k1 + 1) / 2 for
k2 <= k1), L = M with its diagonal exponentiated, Sigma = L L^T.

The gradient restates autograd's chain literally: sqrtm's VJP is
solve_sylvester(S^T, S^T, g) (autograd/scipy/linalg.py), det's VJP is
det * inv(Sigma)^T, matmul's VJP gives (G + G^T) L.  For CHIVI the log q
derivative uses the invariance of the Mahalanobis term under x = mu + S z / s
(so only log det Sigma contributes); tests pin this against torch.autograd
through eigh.
"""
import math

import numpy as np
from scipy import linalg

from . import targets_oracle


def n_free(D):
    return D + D * (D + 1) // 2


def unpack(lam, D):
    mu = lam[:D]
    M = np.zeros((D, D))
    M[np.tril_indices(D)] = lam[D:]
    L = M - np.diag(np.diag(M)) + np.diag(np.exp(np.diag(M)))
    return mu, L, L @ L.T


def pack_grad_L(GL, L):
    """Cotangent of L -> cotangent of the free tril vector (exp on the diagonal)."""
    G = np.tril(GL).copy()
    G[np.diag_indices_from(G)] *= np.diag(L)
    return G[np.tril_indices(L.shape[0])]


def mvt_logpdf(x, m, S, df):
    """_distributions.py:8-38 (eigh, absolute pinv cutoff 1e-10)."""
    d = m.shape[-1]
    s, u = np.linalg.eigh(S)
    s_pinv = np.array([0 if abs(v) <= 1e-10 else 1 / v for v in s], dtype=float)
    U = u * np.sqrt(s_pinv)
    log_pdet = np.sum(np.log(s))
    out = math.lgamma(.5 * (df + d)) - math.lgamma(.5 * df) - .5 * d * np.log(np.pi * df)
    out = out - .5 * log_pdet
    maha = np.sum(np.square((x - m) @ U), axis=-1)
    return out - .5 * (df + d) * np.log(1 + maha / df)


class FullRankT:
    def __init__(self, dim, df):
        if df <= 2:
            raise ValueError('df must be greater than 2')
        self.dim, self.df = dim, float(df)
        self.rs = np.random.RandomState(0)               # vb.py:195
        self.var_param_dim = n_free(dim)

    def draw(self, n, seed=None):
        """(s, z) in the reference's order: chisquare first, then randn (vb.py:204-206)."""
        rs = self.rs if seed is None else np.random.RandomState(seed)
        s = np.sqrt(rs.chisquare(self.df, n) / self.df)
        z = rs.randn(n, self.dim)
        return s, z

    def transform(self, lam, s, z):
        mu, L, Sig = unpack(lam, self.dim)
        S = np.real(linalg.sqrtm(Sig))
        return mu + np.dot(z, S) / s[:, None]

    def sample(self, lam, n, seed=None):
        s, z = self.draw(n, seed)
        return self.transform(lam, s, z)

    def entropy(self, lam):
        return .5 * np.log(np.linalg.det(unpack(lam, self.dim)[2]))

    def logdensity(self, x, lam):
        mu, L, Sig = unpack(lam, self.dim)
        return mvt_logpdf(np.atleast_2d(x), mu, Sig, self.df)

    def mean_and_cov(self, lam):
        mu, L, Sig = unpack(lam, self.dim)
        return mu, self.df / (self.df - 2.) * Sig

    def pth_moment(self, p, lam):
        if p not in [2, 4]:
            raise ValueError('only p = 2 or 4 supported')
        if self.df <= p:
            raise ValueError('df must be greater than p')
        ev = np.linalg.eigvalsh(unpack(lam, self.dim)[2])
        c = self.df / (self.df - 2)
        if p == 2:
            return c * np.sum(ev)
        return c ** 2 * (2 * (self.df - 1) / (self.df - 4) * np.sum(ev ** 2) + np.sum(ev) ** 2)


def _grad_from_GS(fam, lam, GS, coef_inv, gmu):
    """Assemble d/d lambda from the cotangent of S (GS), a multiple of
    inv(Sigma) in d/dSigma (coef_inv) and d/dmu."""
    mu, L, Sig = unpack(lam, fam.dim)
    S = np.real(linalg.sqrtm(Sig))
    X = linalg.solve_sylvester(S.T, S.T, GS)               # autograd sqrtm VJP
    GSig = X + coef_inv * np.linalg.inv(Sig).T
    GL = (GSig + GSig.T) @ L
    return np.concatenate([gmu, pack_grad_L(GL, L)])


def klvi_value_grad(fam, target, lam, n_samples, draws=None):
    """black_box_klvi (vb.py:236-245) for the full-rank t family."""
    s, z = fam.draw(n_samples) if draws is None else draws
    x = fam.transform(lam, s, z)
    lp, g = target(x)
    value = -(fam.entropy(lam) + np.mean(lp))
    zt = z / s[:, None]
    GS = -(zt.T @ g) / n_samples
    return value, _grad_from_GS(fam, lam, GS, -0.5, -np.mean(g, axis=0))


def klvi_pd_value_grad(fam, target, lam, n_samples, draws=None):
    """black_box_klvi_pd (vb.py:268-278): value -(mean log p - mean log q(x)); the
    gradient equals KLVI's (log q's total derivative is -1/2 d log det Sigma)."""
    s, z = fam.draw(n_samples) if draws is None else draws
    x = fam.transform(lam, s, z)
    value = -(np.mean(target(x)[0]) - np.mean(fam.logdensity(x, lam)))
    return value, klvi_value_grad(fam, target, lam, n_samples, draws=(s, z))[1]


def chivi_value_grad(fam, target, lam, n_samples, alpha, draws=None):
    """black_box_chivi (vb.py:248-266) for the full-rank t family."""
    if draws is None:
        seed = np.random.randint(2 ** 32)
        draws = fam.draw(n_samples, seed)
    s, z = draws
    x = fam.transform(lam, s, z)
    lp, g = target(x)
    lw = lp - fam.logdensity(x, lam)
    top = np.max(lw)
    w = np.exp(lw - top) ** alpha
    value = np.log(np.mean(w)) / alpha + top
    zt = z / s[:, None]
    c = alpha / w.size
    GS = c * (zt.T @ (w[:, None] * g))
    return value, _grad_from_GS(fam, lam, GS, 0.5 * c * np.sum(w), c * np.sum(w[:, None] * g, axis=0))


def target_fn(name, D):
    if name == 'corr_gauss':
        return targets_oracle.CorrGauss(D)
    return targets_oracle.TARGETS[name]
