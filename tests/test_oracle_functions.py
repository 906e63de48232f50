"""Pin the R-hat / iterate-averaging restatement (oracle/functions_oracle.py)
by independent formulas: split-R-hat from per-half-chain means and variances
written out directly (Gelman et al., BDA3 §11.4, with the reference's jitter
and its (n-1)/n + B/(nW) form), and cumulative means by explicit loops."""
import numpy as np
import pytest

from oracle import functions_oracle as fo


def _split_rhat(chains):
    nc, n, K = chains.shape
    h = n // 2
    halves = [chains[c, :h] for c in range(nc)] + [chains[c, h:2 * h] for c in range(nc)]
    out = np.empty(K)
    for k in range(K):
        means = np.array([x[:, k].mean() for x in halves])
        vars_ = np.array([x[:, k].var(ddof=1) for x in halves])
        B = h * means.var(ddof=1)
        W = vars_.mean() + 1e-8
        out[k] = np.sqrt((h - 1) / h + B / (h * W))
    return out


@pytest.mark.parametrize('nc,n,K', [(2, 100, 3), (4, 1000, 2), (1, 64, 5)])
def test_rhat_matches_split_formula(nc, n, K):
    rs = np.random.RandomState(0)
    chains = rs.randn(nc, n, K) + rs.randn(nc, 1, K) * 0.3
    _, r = fo.compute_R_hat(chains, warmup=0)
    np.testing.assert_allclose(r, _split_rhat(chains), rtol=1e-12)
    _, r2 = fo.compute_R_hat(chains, warmup=n // 4 * 2)
    np.testing.assert_allclose(r2, _split_rhat(chains[:, n // 4 * 2:]), rtol=1e-12)


def test_rhat_odd_length_raises_like_reference():
    with pytest.raises(ValueError):
        fo.compute_R_hat(np.zeros((2, 101, 1)), warmup=0)


def test_rhat_windows_and_halfway():
    rs = np.random.RandomState(1)
    chains = rs.randn(3, 1000, 2)
    w = fo.compute_R_hat_adaptive_numpy(chains, window_size=200)
    assert w.shape == (5, 2)
    for i in range(5):
        np.testing.assert_allclose(w[i], _split_rhat(chains[:, 200 * i:200 * (i + 1)]), rtol=1e-12)
    hw = fo.compute_R_hat_halfway(chains, interval=100, start=200)
    assert hw.shape == (10, 2)
    for i in range(10):
        sub = chains[:, :min(1000, 200 + (i + 1) * 100)]
        s = sub.shape[1]
        np.testing.assert_allclose(hw[i], _split_rhat(sub[:, s // 2:]), rtol=1e-12)


def test_iterate_averaging():
    x = np.random.RandomState(2).randn(50, 3)
    it, last = fo.stochastic_iterate_averaging(x, 10)
    for t in range(40):
        np.testing.assert_allclose(it[t], x[10:11 + t].mean(axis=0), rtol=1e-13)
    np.testing.assert_allclose(last, x[10:].mean(axis=0), rtol=1e-13)
    with pytest.raises(TypeError):          # the reference raises a str (functions.py:70-71)
        fo.stochastic_iterate_averaging(x, 50)
