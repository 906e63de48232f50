"""Generate golden vectors from the REFERENCE implementation (run in the build
container only; /root/reference does not exist on the GPU box).

  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference's viabel.bounds and notebooks/psis.py are numpy-only and are
loaded by file path under distinct module names (our own package is
`viabel_amd`, but the reference package is named `viabel`; loading by path
keeps the two apart).  viabel.vb is NOT importable here (autograd / paragami
absent), so no vb golden comes from the reference; the vb restatement is
pinned by independent AD instead (tests/test_oracle_vb.py).

Outputs (small .npz files next to this script):
  bounds_golden.npz   divergence / Wasserstein / all_bounds outputs
  psis_golden.npz     psislw / gpdfitnew / gpinv / sumlogs outputs
  rng_golden.npz      numpy legacy RandomState draws used by the reference
Inputs are stored when small; large inputs are stored as the seed recipe
(`recipe_*`) that regenerates them with numpy's frozen legacy stream.
"""
import importlib.util
import os
import sys
import warnings

import numpy as np
from scipy.stats import norm
from scipy.special import factorial2

REF = os.environ.get('VIABEL_REFERENCE', '/root/reference')
HERE = os.path.dirname(os.path.abspath(__file__))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    sys.dont_write_bytecode = True
    bounds = _load('viabel_ref_bounds', os.path.join(REF, 'viabel', 'bounds.py'))
    psis = _load('psis_ref', os.path.join(REF, 'notebooks', 'psis.py'))
    return bounds, psis


def mixture_inputs():
    """normal-mixture.ipynb cells 2, 8: q = N(0, 5), seed 918, 50 000 draws."""
    q_var = 5
    np.random.seed(918)
    samples = norm(scale=np.sqrt(q_var)).rvs(50000)
    log_p = np.logaddexp(norm.logpdf(samples, loc=-2), norm.logpdf(samples, loc=2)) - np.log(2)
    lw = log_p - norm(scale=np.sqrt(q_var)).logpdf(samples)
    return samples, lw, q_var


def gauss_ratio_inputs(seed, n, var1, var2):
    """test_bounds.py style: samples ~ N(0, var2), lw = log N(0,var1) - log N(0,var2)."""
    np.random.seed(seed)
    s = norm(scale=np.sqrt(var2)).rvs(n)
    lw = norm(scale=np.sqrt(var1)).logpdf(s) - norm(scale=np.sqrt(var2)).logpdf(s)
    return s, lw


def make_bounds(bounds):
    out = {}
    samples, lw, q_var = mixture_inputs()
    mb = lambda order: factorial2(order - 1) ** (1 / order) * np.sqrt(q_var)
    cases = {
        'mix_a': bounds.all_bounds(lw, samples),
        'mix_b': bounds.all_bounds(lw, samples, q_var=q_var, log_norm_bound=0),
        'mix_c': bounds.all_bounds(lw, moment_bound_fn=mb, q_var=q_var),
    }
    for cname, res in cases.items():
        for k, v in res.items():
            out['%s_%s' % (cname, k)] = np.float64(v)
    # divergence bound over alpha x elbo on a smaller test_bounds-like sample
    _, lw2 = gauss_ratio_inputs(846, 20000, 4.0, 16.0)
    out['div_lw'] = lw2
    for a in (1.5, 2.0, 3.0):
        for e in (None, 0.0):
            with warnings.catch_warnings(record=True):
                warnings.simplefilter('always')
                d, lnb = bounds.divergence_bound(lw2, a, e, return_log_norm_bound=True)
            tag = 'div_a%g_%s' % (a, 'none' if e is None else 'zero')
            out[tag] = np.array([d, lnb])
    # Wasserstein from samples, 1-D and 3-D
    rs = np.random.RandomState(341)
    s1 = rs.randn(20000) * 3.5
    s3 = rs.randn(5000, 3) * np.array([1.0, 2.0, 0.5]) + np.array([1.0, -1.0, 0.0])
    out['w_s1'] = s1
    out['w_s3'] = s3
    for tag, s in (('w1d', s1), ('w3d', s3)):
        r = bounds.wasserstein_bounds(5.0, s)
        out[tag] = np.array([r['W1'], r['W2']])
    # all_bounds with a 3-D sample covariance (np.cov + spectral norm)
    _, lw3 = gauss_ratio_inputs(1639, 5000, 2.5, 9.3)
    out['ab3_lw'] = lw3
    r = bounds.all_bounds(lw3, s3)
    for k, v in r.items():
        out['ab3_%s' % k] = np.float64(v)
    # the Monte Carlo error warning text
    small = np.array([-40.0, 0.0, -3.0, -1.0])
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        bounds.divergence_bound(small)
    out['warn_lw'] = small
    out['warn_msgs'] = np.array([str(x.message) for x in w])
    return out


def make_psis(psis):
    out = {}
    rs = np.random.RandomState(2024)
    cases = {
        'normal1000': rs.randn(1000),
        't3_1000': rs.standard_t(3, 1000) * 1.5,
        'n5': rs.randn(5),
        'n128': rs.standard_t(2, 128) * 2.0,
        'heavy2e4': np.random.RandomState(7).randn(20000) * 1.7 + np.random.RandomState(8).standard_t(4, 20000),
        'cols': rs.randn(2000, 3) * np.array([0.5, 1.5, 3.0]),
    }
    for name, lw in cases.items():
        lw_out, k = psis.psislw(lw.copy())
        out[name + '_in'] = lw
        out[name + '_out'] = np.asarray(lw_out)
        out[name + '_k'] = np.atleast_1d(k)
    x = np.sort(rs.exponential(2.0, 400)) * rs.uniform(0.5, 1.5, 400)
    out['gpd_x'] = x
    k, sigma, ks, w = psis.gpdfitnew(x.copy(), return_quadrature=True)
    out['gpd_k'] = np.array([k, sigma])
    out['gpd_ks'] = ks
    out['gpd_w'] = w
    p = np.array([0.0, 0.25, 0.5, 0.999, 1.0])
    for tag, (kk, ss) in {'gpinv_pos': (0.4, 1.3), 'gpinv_neg': (-0.3, 2.0),
                          'gpinv_zero': (1e-18, 0.7), 'gpinv_badsig': (0.2, -1.0)}.items():
        out[tag] = psis.gpinv(p, kk, ss)
    out['gpinv_p'] = p
    out['gpinv_open'] = psis.gpinv(np.array([0.1, 0.5, 0.9]), 0.4, 1.3)
    s = rs.randn(777) * 30
    out['sumlogs_x'] = s
    out['sumlogs'] = np.array([psis.sumlogs(s)])
    return out


def make_rng():
    out = {}
    rs = np.random.RandomState(0)
    out['randn_4x5'] = rs.randn(4, 5)
    rs = np.random.RandomState(0)
    out['t40_4x5'] = rs.standard_t(40, size=(4, 5))
    rs = np.random.RandomState(0)
    out['chisq100_4'] = rs.chisquare(100, 4)
    out['randn_after_chisq_4x3'] = rs.randn(4, 3)
    np.random.seed(0)
    out['global_randint'] = np.array([np.random.randint(2 ** 32) for _ in range(3)], dtype=np.int64)
    return out


def main():
    bounds, psis = load_reference()
    np.savez_compressed(os.path.join(HERE, 'bounds_golden.npz'), **make_bounds(bounds))
    np.savez_compressed(os.path.join(HERE, 'psis_golden.npz'), **make_psis(psis))
    np.savez_compressed(os.path.join(HERE, 'rng_golden.npz'), **make_rng())
    for f in ('bounds_golden.npz', 'psis_golden.npz', 'rng_golden.npz'):
        print(f, os.path.getsize(os.path.join(HERE, f)), 'bytes')


if __name__ == '__main__':
    main()
