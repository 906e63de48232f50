"""Would a warm eigenbasis replace Newton-Schulz + PCG on config 4?  (VERDICT r03
next-round 1c.)  Runs the oracle's config-4 trajectory (full-rank t D = 512, CHIVI,
corr_gauss, adagrad, Philox draws) for a few steps and, for each step, measures how
far the previous step's eigenbasis V is from diagonalising the new Sigma:
A = V^T Sigma_new V; first-order perturbation (V' = V (I + E), E_ij = A_ij / (w_j -
w_i)) is only valid where |A_ij| << |w_i - w_j|.  Prints the off-diagonal size, the
eigen-gap distribution and the fraction of pairs where the first-order correction
is not small (|A_ij| / |w_i - w_j| > 0.1) -- there the warm basis must be refreshed
by a full (Jacobi / dsyevd) eigensolve.

  python scripts/eig_warm_analysis.py [steps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from oracle import fullrank_oracle as fo, rng_oracle as ro, vb_oracle as vo
    sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
    import make_cfg4_trajectory as m
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    D = m.D
    lam0 = m.problem()
    ofam = fo.FullRankT(D, m.DF)
    otgt = fo.target_fn('corr_gauss', D)
    lams = [lam0]
    step = [0]

    def f(lam):
        draws = ro.fr_noise(0, 1, step[0], m.N, D, m.DF)
        step[0] += 1
        lams.append(None)
        return fo.chivi_value_grad(ofam, otgt, lam, m.N, m.ALPHA, draws=draws)
    # adagrad_optimize returns only the tail; rerun step by step to keep each lambda
    lam = lam0.copy()
    hist_g = []
    sig = []
    for k in range(steps):
        _, _, S = fo.unpack(lam, D)
        sig.append(S)
        _, g = f(lam)
        hist_g.append(g)
        win = np.array(hist_g[-m.W:])
        lam = lam - m.LR * g / np.sqrt(m.EPS + np.sum(win ** 2, axis=0))
    for k in range(1, steps):
        w0, V = np.linalg.eigh(sig[k - 1])
        w1 = np.linalg.eigvalsh(sig[k])
        A = V.T @ sig[k] @ V
        off = A - np.diag(np.diag(A))
        d = np.diag(A)
        gap = np.abs(d[:, None] - d[None, :])
        iu = np.triu_indices(D, 1)
        ratio = np.abs(off[iu]) / np.maximum(gap[iu], 1e-300)
        print('step %d: ||Sigma_k - Sigma_k-1||_F / ||Sigma||_F = %.2e; off-diag of V^T Sigma_k V: '
              'max %.2e rms %.2e; eigen-gaps: min %.2e median %.2e; pairs with |A_ij|/gap > 0.1: '
              '%.1f %%, > 1: %.1f %%; max |w_k - w_k-1| %.2e'
              % (k, np.linalg.norm(sig[k] - sig[k - 1]) / np.linalg.norm(sig[k]), np.max(np.abs(off)),
                 np.sqrt(np.mean(off[iu] ** 2)), np.min(np.diff(w1)), np.median(np.diff(w1)),
                 100 * np.mean(ratio > 0.1), 100 * np.mean(ratio > 1), np.max(np.abs(w1 - w0))),
              flush=True)


if __name__ == '__main__':
    main()
