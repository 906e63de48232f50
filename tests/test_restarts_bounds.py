"""Host logic: restarts.bounds_records (the bound algebra of all restarts as
arrays) equals bounds.all_bounds_from_divergence row by row with the family's
own pth_moment / mean_and_cov (bounds.py:13-61, vb.py:72-82, 168-182)."""
import warnings

import numpy as np
import pytest

from viabel_amd import bounds, restarts, vb


@pytest.mark.parametrize('make', [
    lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox'),
    lambda: vb.mean_field_t_variational_family(3, 6.5, rng='philox'),
    lambda: vb.mean_field_gaussian_variational_family(7, rng='philox'),
])
def test_bounds_records_match_per_restart(make):
    fam = make()
    rs = np.random.RandomState(3)
    R, P = 17, fam.var_param_dim
    lams = rs.randn(R, P) * 0.5
    div = np.column_stack([rs.rand(R) * 3, rs.randn(R), rs.randn(R), rs.rand(R) * 0.05,
                           rs.randn(R), rs.rand(R) * 0.05, rs.randn(R)])
    ids = list(range(5, 5 + 2 * R, 2))
    with warnings.catch_warnings(record=True) as w_new:
        warnings.simplefilter('always')
        new = np.array(restarts.bounds_records(ids, div, lams, fam))
    old = []
    with warnings.catch_warnings(record=True) as w_old:
        warnings.simplefilter('always')
        for j, r in enumerate(ids):
            opt = lams[j]
            res = bounds.all_bounds_from_divergence(
                div[j], moment_bound_fn=lambda p, opt=opt: fam.pth_moment(p, opt),
                q_var=fam.mean_and_cov(opt)[1])
            old.append([r, res['log_norm_bound'], res['d2'], res['W1'], res['W2'],
                        res['mean_error'], res['std_error'], res['cov_error']])
    np.testing.assert_allclose(new, np.array(old), rtol=1e-14, atol=0)
    assert [str(x.message) for x in w_new] == [str(x.message) for x in w_old]


def test_default_inits_are_the_per_restart_randomstate_streams():
    """default_inits re-seeds one generator per restart: bit for bit
    base + RandomState(r).randn(P) * scale."""
    import numpy as np
    from viabel_amd import restarts
    base = np.linspace(-1, 1, 6)
    want = np.stack([base + np.random.RandomState(r).randn(6) * 0.3 for r in range(9)])
    np.testing.assert_array_equal(restarts.default_inits(9, 6, scale=0.3, base=base), want)
