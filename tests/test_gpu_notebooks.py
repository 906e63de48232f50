"""The reference notebooks' reproducible KLVI runs through viabel_amd on the GPU
(numpy-stream draws, so the same samples as the notebooks): every printed digit
of tests/golden/notebook_outputs.json — the fitted means and stdevs, the
bounds, k-hat and the PSIS-corrected moments — is reproduced."""
import warnings

import numpy as np
import pytest

from tests import notebook_cases as nc
from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]


def _run(case, fam, target, spec):
    from viabel_amd import vb, experiments, bounds
    obj = vb.black_box_klvi(fam, target, spec['N'])
    opt = vb.adagrad_optimize(spec['n_iters'], obj, spec['init'], **spec['kw'])[0]
    mean, cov = fam.mean_and_cov(opt)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        _, lw = experiments.get_samples_and_log_weights(target, fam, opt, spec['M_bounds'])
        b = bounds.all_bounds(lw, q_var=cov, moment_bound_fn=lambda p: fam.pth_moment(p, opt))
        D = spec['D']
        res, am, ac = experiments.improve_with_psis(target, fam, opt, spec['M_psis'],
                                                    np.zeros(D), np.eye(D))
    nc.check(case, mean, np.sqrt(np.diag(cov)), b, res['khat'], am, np.sqrt(np.diag(ac)))


def test_funnel_klvi_notebook():
    from viabel_amd import vb, targets
    s = nc.FUNNEL
    _run('funnel_klvi', vb.mean_field_t_variational_family(s['D'], s['df'], rng='numpy'),
         targets.funnel(s['D']), s)


def test_robust_regression_mean_field_klvi_notebook():
    from viabel_amd import vb, targets
    s = nc.RR_MF
    _run('robust_regression_mf_klvi',
         vb.mean_field_t_variational_family(s['D'], s['df'], rng='numpy'),
         targets.callback(nc.robust_regression_target(), s['D']), s)


def test_robust_regression_full_rank_klvi_notebook():
    from viabel_amd import vb, targets
    s = nc.RR_FR
    _run('robust_regression_fullrank_klvi', vb.t_variational_family(s['D'], s['df'], rng='numpy'),
         targets.callback(nc.robust_regression_target(), s['D']), s)
