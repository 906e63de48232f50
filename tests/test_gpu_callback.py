"""User-model boundary (make_stan_log_density, vb.py:314-321): a host callback
target gives the same estimator values, gradients and trajectories as the
built-in device target of the same model on identical numpy-stream draws.
Tolerance 1e-11 relative (only the target's evaluation order differs)."""
import math

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]


def _close(a, b, rtol):
    a, b = np.asarray(a), np.asarray(b)
    scale = max(1.0, float(np.max(np.abs(b))))
    assert float(np.max(np.abs(a - b))) / scale <= rtol


def _iso(x):
    return np.sum(-0.5 * x * x - 0.5 * math.log(2 * math.pi), axis=1), -x


class _MockStanFit:
    """Stands in for a pystan fit: log_prob / grad_log_prob of one row (the
    eight-schools NCP restatement from the oracle, test infrastructure)."""

    def log_prob(self, row):
        from oracle import targets_oracle
        return targets_oracle.eight_schools_ncp(row[None, :])[0][0]

    def grad_log_prob(self, row):
        from oracle import targets_oracle
        return targets_oracle.eight_schools_ncp(row[None, :])[1][0]


@pytest.mark.parametrize('D,objective', [(5, 'klvi'), (40, 'klvi'), (40, 'chivi'), (3000, 'klvi')])
def test_callback_matches_device_target(D, objective):
    from viabel_amd import vb, targets
    f1 = vb.mean_field_gaussian_variational_family(D, rng='numpy')
    f2 = vb.mean_field_gaussian_variational_family(D, rng='numpy')
    if objective == 'klvi':
        o1 = vb.black_box_klvi(f1, targets.isogauss(D), 64)
        o2 = vb.black_box_klvi(f2, targets.callback(_iso, D), 64)
    else:
        o1 = vb.black_box_chivi(2.0, f1, targets.isogauss(D), 64)
        o2 = vb.black_box_chivi(2.0, f2, targets.callback(_iso, D), 64)
    lam = np.concatenate([np.linspace(-1, 1, D), np.linspace(-0.5, 0.2, D)])
    np.random.seed(1)
    v1, g1 = o1(lam)
    np.random.seed(1)
    v2, g2 = o2(lam)
    np.testing.assert_allclose(v2, v1, rtol=1e-11)
    _close(g2, g1, 1e-11)


def test_stan_adapter_adagrad():
    from viabel_amd import vb, targets
    f1 = vb.mean_field_t_variational_family(10, 40.0, rng='numpy')
    f2 = vb.mean_field_t_variational_family(10, 40.0, rng='numpy')
    o1 = vb.black_box_klvi(f1, targets.eight_schools_ncp(), 30)
    o2 = vb.black_box_klvi(f2, targets.from_stan(_MockStanFit(), 10), 30)
    init = np.zeros(20)
    r1 = vb.adagrad_optimize(40, o1, init)
    r2 = vb.adagrad_optimize(40, o2, init)
    _close(r2[1], r1[1], 1e-10)
    _close(r2[2], r1[2], 1e-10)


def test_torch_target_fullrank_and_log_weights():
    import torch
    from viabel_amd import vb, targets, experiments
    D = 6
    tg = targets.corr_gauss(D)
    P = torch.tensor(tg.params[:-1].reshape(D, D), device='cuda')
    c = float(tg.params[-1])
    tt = targets.torch_target(lambda x: -0.5 * torch.sum(x * (x @ P), dim=1) + c, D)
    f1 = vb.t_variational_family(D, 100.0, rng='numpy')
    f2 = vb.t_variational_family(D, 100.0, rng='numpy')
    lam = np.concatenate([np.zeros(D), np.random.RandomState(0).randn(D * (D + 1) // 2) * 0.05])
    v1, g1 = vb.black_box_klvi(f1, tg, 50)(lam)
    v2, g2 = vb.black_box_klvi(f2, tt, 50)(lam)
    np.testing.assert_allclose(v2, v1, rtol=1e-11)
    _close(g2, g1, 1e-10)
    fm1 = vb.mean_field_gaussian_variational_family(3, rng='numpy')
    fm2 = vb.mean_field_gaussian_variational_family(3, rng='numpy')
    lam3 = np.array([0.1, -0.2, 0.3, 0.0, -0.1, 0.2])
    x1, lw1 = experiments.log_weights(targets.isogauss(3), fm1, lam3, 1000)
    x2, lw2 = experiments.log_weights(targets.callback(_iso, 3), fm2, lam3, 1000)
    _close(x2, x1, 1e-14)
    _close(lw2, lw1, 1e-11)


def test_callback_exception_propagates():
    from viabel_amd import vb, targets

    def bad(x):
        raise ValueError('model failed')
    fam = vb.mean_field_gaussian_variational_family(4, rng='numpy')
    obj = vb.black_box_klvi(fam, targets.callback(bad, 4), 10)
    with pytest.raises(ValueError, match='model failed'):
        obj(np.zeros(8))


def test_make_stan_log_density_dimension_from_family():
    """vb.make_stan_log_density(fit) (vb.py:314-321, no dimension argument): the
    target takes the family's dimension, here through adagrad and log weights."""
    from viabel_amd import vb, targets, experiments
    f1 = vb.mean_field_t_variational_family(10, 40.0, rng='numpy')
    f2 = vb.mean_field_t_variational_family(10, 40.0, rng='numpy')
    stan = vb.make_stan_log_density(_MockStanFit())
    assert stan.dim is None
    r1 = vb.adagrad_optimize(30, vb.black_box_klvi(f1, targets.eight_schools_ncp(), 20), np.zeros(20))
    r2 = vb.adagrad_optimize(30, vb.black_box_klvi(f2, stan, 20), np.zeros(20))
    _close(r2[1], r1[1], 1e-10)
    _, lw1 = experiments.log_weights(targets.eight_schools_ncp(), f1, r1[0], 500)
    _, lw2 = experiments.log_weights(stan, f2, r1[0], 500)
    _close(lw2, lw1, 1e-11)
    lp, g = stan.logdensity_and_grad(np.zeros((3, 10)))
    assert lp.shape == (3,) and g.shape == (3, 10)
