"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Target log densities log p(x) and gradients d log p / dx for x of shape (N, D).
Definitions follow SURVEY.md §8a row a19:
  isogauss   N(0, I_D)                                  (synthetic, config 3)
  mixture    per coordinate logaddexp(N(x;-2,1), N(x;2,1)) - log 2
             (notebooks/normal-mixture.ipynb cell 2, applied per coordinate)
  funnel     notebooks/funnel-distribution.ipynb cell 2 generalised to D:
             x[:,1] ~ N(0, 1.35^2), every other x[:,d] ~ N(0, exp(x[:,1])^2)
  eight_schools_ncp   notebooks/eight_schools_ncp.stan log_prob on the
             unconstrained space [mu, log tau, theta_tilde(8)] (pystan's
             log_prob drops the constants of ~ statements and adds log|J|).
"""
import numpy as np

LOG2PI = np.log(2 * np.pi)

ES_Y = np.array([28., 8., -3., 7., -1., 1., 18., 12.])
ES_SIGMA = np.array([15., 10., 16., 11., 9., 11., 10., 18.])


def _norm_logpdf(x, loc, scale):
    z = (x - loc) / scale
    return -0.5 * z * z - np.log(scale) - 0.5 * LOG2PI


def isogauss(x):
    x = np.atleast_2d(x)
    return np.sum(-0.5 * x * x - 0.5 * LOG2PI, axis=1), -x


def mixture(x):
    x = np.atleast_2d(x)
    a = _norm_logpdf(x, -2.0, 1.0)
    b = _norm_logpdf(x, 2.0, 1.0)
    lp = np.sum(np.logaddexp(a, b) - np.log(2), axis=1)
    wb = 1.0 / (1.0 + np.exp(a - b))
    return lp, -(x + 2.0) + 4.0 * wb


def funnel(x, s0=1.35):
    x = np.atleast_2d(x)
    v = x[:, 1]
    lp = _norm_logpdf(v, 0.0, s0)
    g = np.empty_like(x)
    scale = np.exp(v)
    others = [d for d in range(x.shape[1]) if d != 1]
    gv = -v / s0 ** 2
    for d in others:
        lp = lp + _norm_logpdf(x[:, d], 0.0, scale)
        g[:, d] = -x[:, d] * np.exp(-2 * v)
        gv = gv + (x[:, d] / scale) ** 2 - 1.0
    g[:, 1] = gv
    return lp, g


def eight_schools_ncp(x):
    x = np.atleast_2d(x)
    mu, u, th = x[:, 0], x[:, 1], x[:, 2:]
    tau = np.exp(u)
    t5 = tau / 5.0
    r = (ES_Y[None, :] - mu[:, None] - tau[:, None] * th) / ES_SIGMA[None, :]
    lp = (-0.5 * (mu / 5.0) ** 2 - np.log1p(t5 ** 2) + u
          - 0.5 * np.sum(th ** 2, axis=1) - 0.5 * np.sum(r ** 2, axis=1))
    g = np.empty_like(x)
    g[:, 0] = -mu / 25.0 + np.sum(r / ES_SIGMA[None, :], axis=1)
    g[:, 1] = (-2.0 * t5 ** 2 / (1.0 + t5 ** 2) + 1.0
               + np.sum(r * tau[:, None] * th / ES_SIGMA[None, :], axis=1))
    g[:, 2:] = -th + r * tau[:, None] / ES_SIGMA[None, :]
    return lp, g


TARGETS = {
    'isogauss': isogauss,
    'mixture': mixture,
    'funnel': funnel,
    'eight_schools_ncp': eight_schools_ncp,
}


class CorrGauss:
    """corr_gauss target: N(0, Sigma*) with
    Sigma* = A A^T / D + I, A = RandomState(seed).randn(D, D)."""

    def __init__(self, dim, seed=512):
        a = np.random.RandomState(seed).randn(dim, dim)
        self.sigma = a @ a.T / dim + np.eye(dim)
        self.prec = np.linalg.inv(self.sigma)
        self.prec = 0.5 * (self.prec + self.prec.T)
        sign, logdet = np.linalg.slogdet(self.sigma)
        self.const = -0.5 * logdet - 0.5 * dim * LOG2PI

    def __call__(self, x):
        x = np.atleast_2d(x)
        px = x @ self.prec
        return -0.5 * np.sum(x * px, axis=1) + self.const, -px
