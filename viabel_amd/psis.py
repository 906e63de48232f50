"""Pareto-smoothed importance sampling on the GPU (API of notebooks/psis.py).

  psislw(lw, Reff=1.0, overwrite_lw=False) -> (lw_out, kss)    psis.py:112-208
  gpdfitnew(x, sort=True, sort_in_place=False, return_quadrature=False)
                                                               psis.py:211-331
  gpinv(p, k, sigma)                                           psis.py:334-376
  sumlogs(x, axis=None, out=None)                              psis.py:379-395

All arithmetic runs in libviabel_amd.so (vb_psislw, vb_gpdfit, vb_gpinv,
vb_sumlogs).  ``psislw_with_tail`` additionally returns the tail order
tailinds[x2si] the device used, for bit-exact checks.
"""
import numpy as np

from . import _native as nat

__all__ = ['psislw', 'psislw_with_tail', 'gpdfitnew', 'gpinv', 'sumlogs']


def _tail_cap(n, Reff):
    return int(np.ceil(min(0.2 * n, 3 * np.sqrt(n / Reff))))


def _colmajor(lw):
    """The (m, n) C-contiguous storage of a 2-D Fortran-ordered log-weight matrix
    (n, m): an F-contiguous numpy array or a transposed contiguous float64
    device tensor; None otherwise."""
    if getattr(lw, 'ndim', 0) != 2 or lw.shape[1] < 2:
        return None
    if getattr(lw, 'is_cuda', False):
        import torch
        t = lw.t()
        if lw.dtype == torch.float64 and not lw.is_contiguous() and t.is_contiguous():
            return t
        return None
    if (isinstance(lw, np.ndarray) and lw.dtype == np.float64 and lw.flags.f_contiguous
            and not lw.flags.c_contiguous):
        return lw.T
    return None


def psis_khat(lw, Reff=1.0):
    """The Pareto shape estimates kss of `psislw(lw, Reff)` alone (ndarray [m],
    or a scalar for 1-D input): the device pipeline stops after the GPD fit --
    the smoothed log weights, which only the first output of psislw carries, are
    never formed (vb_psislw with a null lw_out)."""
    cm = _colmajor(lw)
    src, rs_cm = cm, True
    if cm is None:
        dev = nat.device_tensor(lw)
        src, rs_cm = (dev if dev is not None else nat.as_f64(np.asarray(lw, dtype=float))), False
    if lw.ndim == 2:
        n, m = lw.shape
    elif lw.ndim == 1:
        n, m = len(lw), 1
    else:
        raise ValueError("Argument `lw` must be 1 or 2 dimensional.")
    if n <= 1:
        raise ValueError("More than one log-weight needed.")
    k = np.empty(m)
    fn = nat.lib().vb_psislw_colmajor if rs_cm else nat.lib().vb_psislw
    nat.check(fn(nat.context().handle, nat.dptr(src), n, m, float(Reff), None, nat.dptr(k),
                 None, 0, None))
    return k[0] if lw.ndim == 1 else k


def psislw_with_tail(lw, Reff=1.0):
    """psislw plus the tail order of each column.  A float64 device tensor
    input stays in HBM: the smoothed log weights come back as a device tensor
    of shape (n, m); k and the tail orders are host arrays.  Fortran-ordered
    input (psis.py:146 works on such a copy), i.e. an F-contiguous array or the
    transpose of a contiguous device tensor, is read in place and gives output
    of the same order.  All columns run through the device pipeline together."""
    cm = _colmajor(lw)
    dev = None
    if cm is None:
        dev = nat.device_tensor(lw)
        if dev is None:
            lw = np.asarray(lw, dtype=float)
    if lw.ndim == 2:
        n, m = lw.shape
    elif lw.ndim == 1:
        n, m = len(lw), 1
    else:
        raise ValueError("Argument `lw` must be 1 or 2 dimensional.")
    if n <= 1:
        raise ValueError("More than one log-weight needed.")
    k = np.empty(m)
    cap = _tail_cap(n, Reff)
    tail = np.empty((m, max(cap, 1)), dtype=np.int64)
    ntail = np.empty(m, dtype=np.int64)
    if cm is not None:
        if getattr(cm, 'is_cuda', False):
            import torch
            out_cm = torch.empty((m, n), dtype=torch.float64, device=cm.device)
        else:
            out_cm = np.empty((m, n))
        nat.check(nat.lib().vb_psislw_colmajor(nat.context().handle, nat.dptr(cm), n, m,
                                               float(Reff), nat.dptr(out_cm), nat.dptr(k),
                                               nat.i64ptr(tail), max(cap, 1), nat.i64ptr(ntail)))
        out = out_cm.T
    else:
        if dev is None:
            src = nat.as_f64(lw.reshape(n, m))
            out = np.empty((n, m))
        else:
            import torch
            src = dev.reshape(n, m)
            out = torch.empty((n, m), dtype=torch.float64, device=dev.device)
        nat.check(nat.lib().vb_psislw(nat.context().handle, nat.dptr(src), n, m, float(Reff),
                                      nat.dptr(out), nat.dptr(k), nat.i64ptr(tail), max(cap, 1),
                                      nat.i64ptr(ntail)))
    tails = [tail[c, :ntail[c]].copy() for c in range(m)]
    return out, k, tails


def psislw(lw, Reff=1.0, overwrite_lw=False):
    """Pareto smoothed importance sampling (PSIS).  Returns (lw_out, kss);
    kss is a scalar for 1-D input (psis.py:204-206)."""
    out, k, _ = psislw_with_tail(lw, Reff)
    if getattr(lw, 'is_cuda', False):       # device in, device out (no copy to the host)
        return (out[:, 0], k[0]) if lw.ndim == 1 else (out, k)
    lw_arr = np.asarray(lw)
    if lw_arr.ndim == 1:
        res = out[:, 0]
        if overwrite_lw and isinstance(lw, np.ndarray) and lw.flags.f_contiguous:
            lw[...] = res
            res = lw
        return res, k[0]
    if overwrite_lw and isinstance(lw, np.ndarray) and lw.flags.f_contiguous:
        lw[...] = out
        return lw, k
    return np.asfortranarray(out), k


def gpdfitnew(x, sort=True, sort_in_place=False, return_quadrature=False):
    """Zhang-Stephens empirical-Bayes GPD fit; returns (k, sigma[, ks, w])."""
    x = np.asarray(x)
    if x.ndim != 1 or len(x) <= 1:
        raise ValueError("Invalid input array.")
    if sort is True and sort_in_place:
        x.sort()                      # the reference's documented side effect
    xx = nat.as_f64(x)
    n = xx.size
    m = 30 + int(np.sqrt(n))
    k, sigma = np.empty(1), np.empty(1)
    ks, w = np.empty(m), np.empty(m)
    nw = np.empty(1, dtype=np.int64)
    nat.check(nat.lib().vb_gpdfit(nat.context().handle, nat.dptr(xx), n, nat.dptr(k),
                                  nat.dptr(sigma), nat.dptr(ks), nat.dptr(w), nat.i64ptr(nw)))
    if return_quadrature:
        return k[0], sigma[0], ks[:nw[0]].copy(), w[:nw[0]].copy()
    return k[0], sigma[0]


def gpinv(p, k, sigma):
    """Inverse generalised Pareto distribution function."""
    p = np.asarray(p, dtype=float)
    pp = nat.as_f64(p.ravel())
    out = np.empty(pp.size)
    nat.check(nat.lib().vb_gpinv(nat.context().handle, nat.dptr(pp), pp.size, float(k),
                                 float(sigma), nat.dptr(out)))
    return out.reshape(p.shape)


def _sumlogs_1d(v):
    v = nat.as_f64(v)
    r = np.empty(1)
    nat.check(nat.lib().vb_sumlogs(nat.context().handle, nat.dptr(v), v.size, nat.dptr(r)))
    return r[0]


def sumlogs(x, axis=None, out=None):
    """log(sum(exp(x), axis)) computed stably."""
    x = np.asarray(x, dtype=float)
    if axis is None:
        res = _sumlogs_1d(x.ravel())
    else:
        moved = np.moveaxis(x, axis, -1)
        flat = nat.as_f64(moved.reshape(-1, moved.shape[-1]))
        res = np.empty(flat.shape[0])
        nat.check(nat.lib().vb_sumlogs_rows(nat.context().handle, nat.dptr(flat), flat.shape[0],
                                            flat.shape[1], nat.dptr(res)))
        res = res.reshape(moved.shape[:-1])
    if out is not None:
        out[...] = res
        return out
    return res
