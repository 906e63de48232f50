"""Pins the oracle on the reference's own published outputs: the notebooks'
reproducible KLVI runs (funnel, robust regression mean-field t and full-rank t)
re-run on the oracle reproduce every printed digit (tests/golden/
notebook_outputs.json)."""
import warnings

import numpy as np

from tests import notebook_cases as nc


def _summaries(target, fam, opt, mean_cov, pth, M_b, M_p, sample_lw):
    from oracle import bounds_oracle as bo, psis_oracle as po
    _, lw = sample_lw(M_b)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        b = bo.all_bounds(lw, q_var=mean_cov[1], moment_bound_fn=pth)
        x2, lw2 = sample_lw(M_p)
        slw, k = po.psislw(lw2.copy())
    slw = slw - np.max(slw)
    w = np.exp(slw)
    w /= np.sum(w)
    am = np.sum(w[None, :] * x2.T, axis=1)
    ac = np.cov(x2.T, aweights=w, ddof=0)
    return b, k, am, np.sqrt(np.diag(ac))


def _mf(case, target, spec):
    from oracle import vb_oracle as vo
    D, df = spec['D'], spec['df']
    fam = vo.Family('t', D, df)
    opt = vo.adagrad_optimize(spec['n_iters'], lambda l: vo.klvi_value_grad(fam, target, l, spec['N']),
                              spec['init'], **spec['kw'])[0]
    c = df / (df - 2)
    s = np.exp(opt[D:])
    pth = lambda p: (c * np.sum(s ** 2) if p == 2
                     else c ** 2 * (2 * (df - 1) / (df - 4) * np.sum(s ** 4) + np.sum(s ** 2) ** 2))
    b, k, am, asd = _summaries(target, fam, opt, (opt[:D], c * np.diag(s ** 2)), pth,
                               spec['M_bounds'], spec['M_psis'],
                               lambda m: vo.log_weights(fam, target, opt, m))
    nc.check(case, opt[:D], np.sqrt(c) * s, b, k, am, asd)


def test_funnel_klvi_notebook():
    _mf('funnel_klvi', 'funnel', nc.FUNNEL)


def test_robust_regression_mean_field_klvi_notebook():
    _mf('robust_regression_mf_klvi', nc.robust_regression_target(), nc.RR_MF)


def test_robust_regression_full_rank_klvi_notebook():
    from oracle import vb_oracle as vo, fullrank_oracle as fr
    spec, target = nc.RR_FR, nc.robust_regression_target()
    fam = fr.FullRankT(spec['D'], spec['df'])
    opt = vo.adagrad_optimize(spec['n_iters'], lambda l: fr.klvi_value_grad(fam, target, l, spec['N']),
                              spec['init'], **spec['kw'])[0]
    m, C = fam.mean_and_cov(opt)

    def sample_lw(n):
        xs = fam.sample(opt, n)
        return xs, target(xs)[0] - fam.logdensity(xs, opt)
    b, k, am, asd = _summaries(target, fam, opt, (m, C), lambda p: fam.pth_moment(p, opt),
                               spec['M_bounds'], spec['M_psis'], sample_lw)
    nc.check('robust_regression_fullrank_klvi', m, np.sqrt(np.diag(C)), b, k, am, asd)
