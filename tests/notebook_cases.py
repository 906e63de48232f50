"""The reproducible KLVI runs of the reference's notebooks (settings restated
from the notebook cells cited in tests/golden/notebook_outputs.json), shared by
the oracle test (CPU) and the device test.  Every quantity the notebooks print
is invariant to a constant shift of log p, so Stan's dropped constants do not
matter."""
import json
import os

import numpy as np

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'notebook_outputs.json')))

FUNNEL = dict(D=2, df=40.0, init=np.array([0., -1., 1., 1.]), n_iters=10000, N=100,
              kw=dict(learning_rate=.01, learning_rate_end=.001), M_bounds=1000000,
              M_psis=1000000)
RR_MF = dict(D=2, df=40.0, init=np.array([0., 0., 1., 1.]), n_iters=5000, N=100,
             kw=dict(learning_rate=.01), M_bounds=1000000, M_psis=1000000)
RR_FR = dict(D=2, df=100.0, init=np.zeros(5), n_iters=5000, N=100,
             kw=dict(learning_rate=.1, learning_rate_end=.001), M_bounds=1000000,
             M_psis=1000000)


def robust_regression_data():
    """robust-regression.ipynb cell 6: N = 25 points, t(40) noise, centred y."""
    rs_state = np.random.get_state()
    np.random.seed(5039)
    x = np.random.randn(25, 2).dot(np.array([[1, .75], [.75, 1]]))
    y_raw = x.dot(np.array([-2, 1])) + np.random.standard_t(40, 25)
    np.random.set_state(rs_state)
    return x, y_raw - np.mean(y_raw)


def robust_regression_target():
    """The notebook's Stan model (cell 3): beta ~ normal(0, 10);
    y ~ student_t(40, x beta, 1); log p up to constants and its gradient."""
    x, y = robust_regression_data()
    nu = 40.0

    def f(b):
        b = np.atleast_2d(b)
        r = y[None, :] - b @ x.T
        lp = (-0.5 * np.sum((b / 10.0) ** 2, axis=1)
              - (nu + 1) / 2 * np.sum(np.log1p(r ** 2 / nu), axis=1))
        g = -b / 100.0 + ((nu + 1) * r / (nu + r ** 2)) @ x
        return lp, g
    return f


def check(case, mean, stdevs, bounds, khat, psis_mean, psis_stdevs):
    """Compare with the printed values: 8-significant-digit arrays within half a
    unit of the last printed digit (+ a 1e-8 allowance for a different but
    exact-to-rounding reduction order), 3-significant-digit scalars as printed."""
    g = GOLDEN[case]
    for got, want in ((mean, g['mean']), (stdevs, g['stdevs']), (psis_mean, g['psis_mean']),
                      (psis_stdevs, g['psis_stdevs'])):
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-8)
    shown = {'W2': bounds['W2'], 'd2': bounds['d2'], 'mean_error': bounds['mean_error'],
             'std_error': bounds['std_error'], 'sqrt_cov_error': np.sqrt(bounds['cov_error'])}
    assert {k: '{:.3g}'.format(v) for k, v in shown.items()} == g['bounds_3g']
    assert '{:.3g}'.format(khat) == g['khat_3g']
