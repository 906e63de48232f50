"""The t family's Philox log-weight draws (Bailey's trigonometric t, vb_device.hpp
bailey_t; oracle/vbrng.c family 2) on every log-weight path: the row kernel (D <=
16, config 5's bound draws), the separable wave-per-row kernel (D > 16) and the
materialised path (non-separable wide targets).  Samples equal the C oracle's
draws scaled by the family (1e-13), log weights the oracle's log_weights on
those draws (1e-12 relative to the largest); the batched rows launch equals the
per-row calls (test_gpu_restarts.py)."""
import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]


def _close(a, b, rtol):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    assert a.shape == b.shape
    err = float(np.max(np.abs(a - b))) / max(1.0, float(np.max(np.abs(b))))
    assert err <= rtol, 'max scaled error %.3e > %.1e' % (err, rtol)


@pytest.mark.parametrize('target,D,df', [('eight_schools_ncp', 10, 40.0), ('isogauss', 3, 3.5),
                                         ('mixture', 1, 8.0), ('isogauss', 40, 40.0),
                                         ('funnel', 20, 40.0)])
def test_bailey_log_weights_equal_oracle(target, D, df):
    from viabel_amd import vb, targets, experiments
    from oracle import vb_oracle as vo, rng_oracle as ro
    fam = vb.mean_field_t_variational_family(D, df, rng='philox')
    fam.stream = 321
    tgt = {'eight_schools_ncp': lambda: targets.eight_schools_ncp(),
           'isogauss': lambda: targets.isogauss(D), 'mixture': lambda: targets.mixture(D),
           'funnel': lambda: targets.funnel(D)}[target]()
    lam = np.random.RandomState(D).randn(2 * D) * 0.3
    m = 4000
    for call in range(2):
        x, lw = experiments.log_weights(tgt, fam, lam, m)
        eps = ro.noise(fam.seed, fam.stream, call, m, D, 't_bailey', df)
        ox, olw = vo.log_weights(vo.Family('t', D, df), target, lam, m, eps=eps)
        _close(x, ox, 1e-13)
        _close(lw, olw, 1e-12)
