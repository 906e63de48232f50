"""ORACLE -- TEST INFRASTRUCTURE ONLY.

numpy restatement of viabel/functions.py:8-77 (split-chain R-hat, windowed and
halfway R-hat, stochastic iterate averaging) and of the IA optimisers
rmsprop_IA_optimize_with_rhat / adam_IA_optimize_with_rhat (viabel/vb.py:392-712).

The reference module imports autograd (absent here), so it cannot be imported;
these restatements are pinned by independent formulas in the tests (a textbook
split-R-hat computed from per-half means and variances, closed-form cumulative
means) -- parity with a run of the reference itself is unpinned.
"""
import numpy as np

from . import vb_oracle


def compute_R_hat(chains, warmup=500):
    """functions.py:8-31 (including its odd-length handling, which drops two
    iterations and then fails the reshape like the reference)."""
    jitter = 1e-8
    chains = chains[:, warmup:, :]
    n_iters = chains.shape[1]
    n_chains = chains.shape[0]
    K = chains.shape[2]
    if n_iters % 2 == 1:
        n_iters = int(n_iters - 1)
        chains = chains[:, :n_iters - 1, :]
    n_iters = n_iters // 2
    psi = np.reshape(chains, (n_chains * 2, n_iters, K))
    n_chains2 = n_chains * 2
    psi_dot_j = np.mean(psi, axis=1)
    psi_dot_dot = np.mean(psi_dot_j, axis=0)
    s_j_2 = np.sum((psi - np.expand_dims(psi_dot_j, axis=1)) ** 2, axis=1) / (n_iters - 1)
    B = n_iters * np.sum((psi_dot_j - psi_dot_dot) ** 2, axis=0) / (n_chains2 - 1)
    W = np.nanmean(s_j_2, axis=0)
    W = W + jitter
    var_hat = (n_iters - 1) / n_iters + (B / (n_iters * W))
    return var_hat, np.sqrt(var_hat)


def compute_R_hat_adaptive_numpy(chains, window_size=100):
    """functions.py:44-52."""
    n_chains, n_iters, K = chains.shape
    n_windows = n_iters // window_size
    cr = np.transpose(np.reshape(chains, [n_chains, n_windows, window_size, -1]), [1, 0, 2, 3])
    return np.array([compute_R_hat(cr[i, :], warmup=0)[1] for i in range(cr.shape[0])])


def compute_R_hat_halfway(chains, interval=100, start=1000):
    """functions.py:54-65."""
    n_chains, n_iters, K = chains.shape
    out = []
    for i in range(n_iters // interval):
        sub = chains[:, :start + (i + 1) * interval, :]
        out.append(compute_R_hat(sub, warmup=sub.shape[1] // 2)[1])
    return np.array(out)


def stochastic_iterate_averaging(estimate, start):
    """functions.py:68-77."""
    N = estimate.shape[0]
    if N - start <= 0:
        # the reference raises a bare str (functions.py:70-71), which Python
        # turns into a TypeError; same exception type here, with the message
        raise TypeError('Start of stationary distribution must be lower than number of iterates')
    window_lengths = np.reshape(np.arange(start, N) - start + 1, [-1, 1])
    estimate_iters = np.cumsum(estimate[start:, :], axis=0) / window_lengths
    return estimate_iters, estimate_iters[-1]


def _ia_optimize(kind, n_iters, objective_and_grad, init_param, K, window=500,
                 learning_rate=.01, epsilon=.000001, rhat_window=500, n_optimisers=1,
                 r_mean_threshold=1.15, r_sigma_threshold=1.20, tail_avg_iters=2000,
                 learning_rate_end=None, perturb=None, has_log_norm=False, avg_grad_norm=False):
    """vb.py:392-553 (rmsprop; avg_grad_norm: the scalar sum of squares, or
    exp(log_norm), normalises every coordinate, vb.py:443-451) and vb.py:556-712
    (adam).  has_log_norm: the objective returns (value, grad, log_norm).
    `perturb(o, P)` replaces the global-RNG init perturbation draw
    (stats.norm.rvs after np.random.seed(o)) when given."""
    value_history = []
    log_norm_history = []
    lam = init_param.copy()
    hist_list, final_list = [], []
    scale = 0.5 if kind == 'rmsprop' else 0.2
    for o in range(n_optimisers):
        hist = []
        np.random.seed(seed=o)
        if o >= 1:
            z = perturb(o, len(init_param)) if perturb else np.random.randn(len(init_param))
            lam = init_param + z * (o + 1) * scale
        sched = vb_oracle.learning_rate_schedule(n_iters, learning_rate, learning_rate_end)
        for i, lr in zip(range(n_iters), sched):
            if has_log_norm:
                val, g, ln = objective_and_grad(lam)
            else:
                val, g = objective_and_grad(lam)
                ln = 0
            value_history.append(val)
            log_norm_history.append(ln)
            old = lam.copy()
            if kind == 'rmsprop':
                if avg_grad_norm:
                    gn = np.exp(ln) if has_log_norm else np.sum(g ** 2, axis=0)
                    sgs = gn if i == 0 else gn * 0.9 + (1. - 0.9) * gn
                else:
                    sgs = g ** 2 if i == 0 else sgs * 0.9 + (1. - 0.9) * g ** 2
                lam = lam - lr * g / np.sqrt(epsilon + sgs)
            else:
                if i == 0:
                    v = 0.9 * g ** 2
                    m = 0.9 * g
                else:
                    v = v * 0.999 + (1. - 0.999) * g ** 2
                    m = m * 0.9 + (1. - 0.9) * g
                m_hat = m / (1 - np.power(0.9, i + 2))
                v_hat = v / (1 - np.power(0.999, i + 2))
                lam = lam - lr * m_hat / np.sqrt(epsilon + v_hat)
            hist.append(old)
            if len(hist) > 100 * window:
                hist.pop(0)
        hist_list.append(np.array(hist))
        final_list.append(lam)
    chains = np.stack(hist_list, axis=0)
    rhats = compute_R_hat_adaptive_numpy(chains, window_size=rhat_window)
    rhats_halfway = compute_R_hat_halfway(chains, interval=100, start=200)
    rm, rs = rhats[:, :K], rhats[:, K:]
    start_m = start_s = n_iters - tail_avg_iters
    for ee in range(rm.shape[0] - 1):
        if (rm[ee] < r_mean_threshold).all() and (rm[ee + 1] < r_mean_threshold).all():
            start_m = ee * rhat_window
            break
    for ee in range(rs.shape[0] - 1):
        if (rs[ee] < r_sigma_threshold).all() and (rs[ee + 1] < r_sigma_threshold).all():
            start_s = ee * rhat_window
            break
    means, sigmas = [], []
    for o in range(n_optimisers):
        means.append(stochastic_iterate_averaging(chains[o, :, :K], start_m)[0])
        sigmas.append(stochastic_iterate_averaging(chains[o, :, K:], start_s)[0])
    log = {'start_avg_mean_iters': start_m, 'start_avg_sigma_iters': start_s,
           'r_hat_mean': rm, 'r_hat_sigma': rs,
           'r_hat_mean_halfway': rhats_halfway[:, :K], 'r_hat_sigma_halfway': rhats_halfway[:, K:]}
    return (lam, chains, means, sigmas, np.array(value_history),
            np.array(log_norm_history, dtype=float), log)


def rmsprop_IA_optimize_with_rhat(*args, **kw):
    return _ia_optimize('rmsprop', *args, **kw)


def adam_IA_optimize_with_rhat(*args, **kw):
    return _ia_optimize('adam', *args, **kw)
