"""Oracle trajectory of config 4 (full-rank t, D = 512, df = 100, CHIVI alpha = 2,
N = 128, corr_gauss target, adagrad W = 10 lr .01 eps .1; Philox seed 0 stream 1,
the bench's workload) for tests/test_gpu_configs.py.

The oracle's step (scipy sqrtm + the solve_sylvester VJP, oracle/fullrank_oracle.py)
costs ~1 s at D = 512, too slow to recompute 120 steps inside a GPU test, so the
trajectory is computed here once, on the C oracle's Philox draws, and stored:

  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_cfg4_trajectory.py

Stored (cfg4_trajectory.npz): the objective value of every step, and at fixed
sampled parameter indices (the 512 means, the 512 log-diagonal entries and 1 024
off-diagonal entries) lambda after every third of the last 30 steps.  Data only; no
reference code is involved (the oracle restates vb.py:192-266, pinned by the
robust-regression notebook's full-rank run, tests/test_oracle_notebooks.py).
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

D, N, DF, ALPHA, W, LR, EPS = 512, 128, 100.0, 2.0, 10, 0.01, 0.1
N_ITERS, TAIL = 120, 30


def problem():
    """bench.py _cfg4_problem: the config-4 initial parameters."""
    rs = np.random.RandomState(4)
    tri = np.tril_indices(D)
    free = rs.randn(len(tri[0])) * 0.01
    free[tri[0] == tri[1]] = rs.randn(D) * 0.1
    return np.concatenate([np.zeros(D), free])


def sample_index():
    tri = np.tril_indices(D)
    diag = D + np.nonzero(tri[0] == tri[1])[0]
    off = D + np.nonzero(tri[0] != tri[1])[0]
    pick = np.sort(np.random.RandomState(77).choice(off, 3072, replace=False))[::3]
    return np.concatenate([np.arange(D), diag, pick])


TAIL_ROWS = np.arange(2, TAIL, 3)     # lambda after steps 92, 95, ..., 119


def main():
    from oracle import fullrank_oracle as fo, rng_oracle as ro, vb_oracle as vo
    lam0 = problem()
    ofam = fo.FullRankT(D, DF)
    otgt = fo.target_fn('corr_gauss', D)
    step = [0]
    t0 = time.time()

    def f(lam):
        draws = ro.fr_noise(0, 1, step[0], N, D, DF)
        step[0] += 1
        if step[0] % 10 == 0:
            print('step %d  %.0f s' % (step[0], time.time() - t0), flush=True)
        return fo.chivi_value_grad(ofam, otgt, lam, N, ALPHA, draws=draws)
    _, hist, vals, _ = vo.adagrad_optimize(N_ITERS, f, lam0, window=W, learning_rate=LR,
                                           epsilon=EPS)
    idx = sample_index()
    # hist holds the tail quarter: row k = lambda after step 3 N_ITERS / 4 + k
    assert hist.shape[0] == N_ITERS - 3 * N_ITERS // 4 == TAIL
    np.savez_compressed(os.path.join(HERE, 'cfg4_trajectory.npz'), values=vals, index=idx,
                        tail_rows=TAIL_ROWS, tail=hist[TAIL_ROWS][:, idx], n_iters=N_ITERS)
    print('wrote cfg4_trajectory.npz', vals[:3], vals[-3:])


if __name__ == '__main__':
    main()
