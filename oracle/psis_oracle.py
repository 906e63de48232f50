"""ORACLE -- TEST INFRASTRUCTURE ONLY.

numpy restatement of notebooks/psis.py (PSIS smoothing, Zhang-Stephens GPD
fit, GPD inverse CDF, log-sum-exp).  Pinned against golden outputs of the
reference (tests/golden/psis_golden.npz).  Additionally returns the tail
order tailinds[x2si] (psis.py:182, 196) so tests can check the device sort
bit-exactly.
"""
import numpy as np

EPS = np.finfo(float).eps


def sumlogs(x, axis=None):
    """psis.py:379-395."""
    top = np.max(x, axis=axis, keepdims=True)
    s = np.log(np.sum(np.exp(x - top), axis=axis))
    return s + np.squeeze(top)


def gpinv(p, k, sigma):
    """psis.py:334-376."""
    p = np.asarray(p, dtype=float)
    out = np.full(p.shape, np.nan)
    if sigma <= 0:
        return out
    inside = (p > 0) & (p < 1)
    t = np.log1p(-p[inside])
    if np.abs(k) < EPS:
        v = -t
    else:
        v = np.expm1(t * -k) / k
    out[inside] = v * sigma
    if not np.all(inside):
        out[p == 0] = 0
        out[p == 1] = np.inf if k >= 0 else -sigma / k
    return out


def gpdfit(x, order=None, return_quadrature=False):
    """gpdfitnew, psis.py:211-331 (empirical-Bayes estimate of the GPD)."""
    if x.ndim != 1 or len(x) <= 1:
        raise ValueError("Invalid input array.")
    if order is None:
        order = np.argsort(x)
    n = len(x)
    m = 30 + int(np.sqrt(n))
    grid = 1 - np.sqrt(m / (np.arange(1, m + 1, dtype=float) - 0.5))
    grid = grid / (3 * x[order[int(n / 4 + 0.5) - 1]]) + 1 / x[order[-1]]
    kq = np.mean(np.log1p(-grid[:, None] * x), axis=1)
    L = n * ((np.log(-(grid / kq)) - kq) - 1)
    with np.errstate(over='ignore'):
        w = 1 / np.sum(np.exp(L[None, :] - L[:, None]), axis=1)
    keep = w >= 10 * EPS
    w, grid = w[keep], grid[keep]
    w = w / w.sum()
    b = np.sum(grid * w)
    k = np.mean(np.log1p(-b * x))
    sigma = -k / b * n / (n - 0)
    a = 10
    k = k * n / (n + a) + a * 0.5 / (n + a)
    if return_quadrature:
        ks = np.mean(np.log1p(grid[:, None] * -x), axis=1)
        ks = ks * n / (n + a) + a * 0.5 / (n + a)
        return k, sigma, ks, w
    return k, sigma


def psislw(lw, Reff=1.0, return_tail=False):
    """psislw, psis.py:112-208.  Returns (lw_out, k) and, if return_tail, the
    list of tailinds[x2si] per column."""
    if lw.ndim == 2:
        n, m = lw.shape
    elif lw.ndim == 1:
        n, m = len(lw), 1
    else:
        raise ValueError("Argument `lw` must be 1 or 2 dimensional.")
    if n <= 1:
        raise ValueError("More than one log-weight needed.")
    out = np.copy(lw, order='F')
    ks = np.empty(m)
    tails = []
    ncut = int(np.ceil(min(0.2 * n, 3 * np.sqrt(n / Reff))))
    floor = np.log(np.finfo(float).tiny)
    cols = out.T if out.ndim == 2 else out[None, :]
    for c, x in enumerate(cols):
        x -= np.max(x)
        srt = np.argsort(x)
        cut = max(x[srt[-ncut - 1]], floor)
        ecut = np.exp(cut)
        tidx = np.flatnonzero(x > cut)
        tv = x[tidx]
        if len(tv) <= 4:
            k, sigma, o = np.inf, None, np.arange(len(tv))
        else:
            o = np.argsort(tv)
            y = np.exp(tv) - ecut
            k, sigma = gpdfit(y, order=o)
        tails.append(tidx[o])
        if k >= 1 / 3 and not np.isinf(k):
            q = np.log(gpinv((np.arange(len(tv)) + 0.5) / len(tv), k, sigma) + ecut)
            x[tidx[o]] = q
            x[x > 0] = 0
        x -= sumlogs(x)
        ks[c] = k
    if out.ndim == 1:
        ks = ks[0]
    return (out, ks, tails) if return_tail else (out, ks)
