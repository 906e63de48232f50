"""Convergence diagnostics of viabel/functions.py:8-77 on the device.

  compute_R_hat                  functions.py:8-31
  compute_R_hat_adaptive_numpy   functions.py:44-52
  compute_R_hat_halfway          functions.py:54-65
  stochastic_iterate_averaging   functions.py:68-77
  safe_root, flat_to_triang, triang_to_flat, compute_posterior_moments
                                 functions.py:80-150 (host helpers of the IA
                                 notebooks: index reshapes and a d x d
                                 conjugate-Gaussian posterior; no Monte Carlo)

Chains are [n_chains, n_iters, K] float64 (host or torch device tensors).  Every
R-hat of a call is one segment of a single batched kernel launch (vb_rhat);
the segment bookkeeping below mirrors the reference's slicing, including its
odd-length quirk (two iterations dropped, then the reshape fails).
"""
import numpy as np

from . import _native as nat

__all__ = ['compute_R_hat', 'compute_R_hat_adaptive_numpy', 'compute_R_hat_halfway',
           'adaptive_segments', 'halfway_segments', 'rhat_stats', 'rhat_combine',
           'stochastic_iterate_averaging', 'safe_root', 'flat_to_triang', 'triang_to_flat',
           'compute_posterior_moments']


def _chains(chains):
    c = nat.as_f64(chains)
    if c.ndim != 3:
        raise ValueError('chains must have shape (n_chains, n_iters, K)')
    return c


def _segment(n_chains, n_iters, K, warmup):
    """(start, length) of compute_R_hat(chains[:, warmup:, :]) (functions.py:12-21)."""
    start = min(max(int(warmup), 0), n_iters) if warmup >= 0 else max(n_iters + int(warmup), 0)
    n = n_iters - start
    if n % 2 == 1:
        # the reference drops two iterations here, then its reshape cannot succeed
        raise ValueError('cannot reshape array of size %d into shape (%d,%d,%d)'
                         % (n_chains * (n - 2) * K, 2 * n_chains, (n - 1) // 2, K))
    return start, n


def _rhat_batch(c, segs, return_var=False):
    n_chains, n_iters, K = c.shape
    starts = np.array([s for s, _ in segs], dtype=np.int64)
    lens = np.array([n for _, n in segs], dtype=np.int64)
    out = np.empty((len(segs), K))
    var = np.empty((len(segs), K)) if return_var else None
    nat.check(nat.lib().vb_rhat(nat.context().handle, nat.dptr(c), n_chains, n_iters, K, len(segs),
                                nat.i64ptr(starts), nat.i64ptr(lens), nat.dptr(var),
                                nat.dptr(out)))
    return var, out


def compute_R_hat(chains, warmup=500):
    """Split-chain R-hat; returns (var_hat, R_hat), each of shape (K,)."""
    c = _chains(chains)
    nc, n, K = c.shape
    seg = _segment(nc, n, K, warmup)
    if seg[1] < 2:
        raise ValueError('R-hat needs at least two iterations after warm-up')
    var, out = _rhat_batch(c, [seg], return_var=True)
    return var[0], out[0]


def adaptive_segments(n_chains, n_iters, K, window_size=100):
    """(start, length) of every window of compute_R_hat_adaptive_numpy, with the
    reference's reshape errors (functions.py:44-52)."""
    n_windows = n_iters // window_size
    if n_windows * window_size != n_iters:
        raise ValueError('cannot reshape array of size %d into shape (%d,%d,%d,newaxis)'
                         % (n_chains * n_iters * K, n_chains, n_windows, window_size))
    if window_size % 2 == 1:
        _segment(n_chains, window_size, K, 0)
    return [(i * window_size, window_size) for i in range(n_windows)]


def halfway_segments(n_chains, n_iters, K, interval=100, start=1000):
    """(start, length) of every sub-chain of compute_R_hat_halfway
    (functions.py:54-65)."""
    segs = []
    for i in range(n_iters // interval):
        sub_n = min(start + (i + 1) * interval, n_iters)
        segs.append(_segment(n_chains, sub_n, K, sub_n // 2))
    return segs


def compute_R_hat_adaptive_numpy(chains, window_size=100):
    """R-hat of consecutive windows of `window_size` iterations: (n_windows, K)."""
    c = _chains(chains)
    nc, n, K = c.shape
    return _rhat_batch(c, adaptive_segments(nc, n, K, window_size))[1]


def compute_R_hat_halfway(chains, interval=100, start=1000):
    """R-hat of chains[:, :start + (i+1) interval] after discarding its first half."""
    c = _chains(chains)
    nc, n, K = c.shape
    segs = halfway_segments(nc, n, K, interval, start)
    if not segs:
        return np.zeros((0,))
    return _rhat_batch(c, segs)[1]


def rhat_stats(chains, segs):
    """First stage of R-hat for chains held by one rank: per segment, half-chain
    (2 c + half) and parameter, the half-chain mean and centred sum of squares,
    each [n_segs][2 n_chains][K] (vb_rhat_stats)."""
    c = _chains(chains)
    nc, n, K = c.shape
    starts = np.array([s for s, _ in segs], dtype=np.int64)
    lens = np.array([m for _, m in segs], dtype=np.int64)
    mean = np.empty((len(segs), 2 * nc, K))
    ss = np.empty((len(segs), 2 * nc, K))
    nat.check(nat.lib().vb_rhat_stats(nat.context().handle, nat.dptr(c), nc, n, K, len(segs),
                                      nat.i64ptr(starts), nat.i64ptr(lens), nat.dptr(mean),
                                      nat.dptr(ss)))
    return mean, ss


def rhat_combine(mean, ss, lens, return_var=False):
    """Second stage: R-hat [n_segs][K] of the half-chains of all ranks
    (mean / ss [n_segs][n_halves][K] in chain order, vb_rhat_combine); the same
    bits as compute_R_hat on the gathered chains."""
    mean = nat.as_f64(mean)
    ss = nat.as_f64(ss)
    J, H, K = mean.shape
    lens = np.ascontiguousarray(lens, dtype=np.int64)
    out = np.empty((J, K))
    var = np.empty((J, K)) if return_var else None
    nat.check(nat.lib().vb_rhat_combine(nat.context().handle, nat.dptr(mean), nat.dptr(ss), H, K, J,
                                        nat.i64ptr(lens), nat.dptr(var), nat.dptr(out)))
    return (var, out) if return_var else out


def stochastic_iterate_averaging(estimate, start):
    """Cumulative means of estimate[start:] (rows = iterations); returns
    (estimate_iters, estimate_mean)."""
    x = nat.as_f64(estimate)
    if x.ndim == 1:
        x = x[:, None]
    N, cols = x.shape
    start = int(start)
    if N - start <= 0:
        # the reference raises a bare str (functions.py:70-71), which Python
        # turns into a TypeError; same exception type here, with the message
        raise TypeError('Start of stationary distribution must be lower than number of iterates')
    out = np.empty((N - start, cols))
    nat.check(nat.lib().vb_iterate_average(nat.context().handle, nat.dptr(x), N, cols, cols, start,
                                           nat.dptr(out)))
    return out, out[-1]


def safe_root(N):
    """Integer square root of a perfect square (functions.py:80-85)."""
    r = int(np.sqrt(N))
    if r * r != N:
        raise ValueError("N is not square!")
    return r


def flat_to_triang(flat_mat):
    """Row-major lower triangle [M(M+1)/2] -> [M, M] with zeros above the
    diagonal (functions.py:106-118: row m holds entries (m, 0..m))."""
    flat = np.asarray(flat_mat, dtype=float).ravel()
    M = int(-1 + np.sqrt(8 * flat.size + 1)) // 2
    out = np.zeros((M, M))
    out[np.tril_indices(M)] = flat[:M * (M + 1) // 2]
    return out


def triang_to_flat(L):
    """[B, M, M] stack of lower triangles -> [M(M+1)/2, B] (functions.py:126-136):
    column d holds L[d]'s lower triangle in row-major order, (m, 0..m) for m =
    0..M-1.  Not differentiable: the reference declares it an autograd
    @primitive with flat_to_triang as its VJP (functions.py:120-125); autograd
    is not part of this implementation, so code that differentiates through it
    must apply that VJP itself."""
    L = np.asarray(L)
    B, _, M = L.shape
    rows, cols = np.tril_indices(M)
    return np.ascontiguousarray(L[:, rows, cols].T).astype(float)


def compute_posterior_moments(prior_mean, prior_covariance, noise_variance, x, y):
    """Posterior mean and covariance of Bayesian linear regression with a Gaussian
    prior (functions.py:139-150): precision = prior precision + x^T x / noise,
    both inverses through Cholesky factors as the reference forms them."""
    inv_L = np.linalg.inv(np.linalg.cholesky(prior_covariance))
    prior_precision = inv_L.T @ inv_L
    inv_a = np.linalg.inv(np.linalg.cholesky(prior_precision + x.T @ x * (1. / noise_variance)))
    post_S = inv_a.T @ inv_a
    post_mu = post_S @ (prior_precision @ prior_mean + (1. / noise_variance) * x.T @ y)
    return post_mu, post_S
