"""Device block cache (vb_capi.hip devpool): runs dropped and made again reuse
cached blocks instead of hipFree / hipMalloc.  A reused block must not carry
anything into its next run: the same optimisation repeated around runs of other
shapes (which return and take blocks of other size classes, and of the same
ones) gives bitwise the same trajectory, values and smoothed parameters."""
import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]


def _fit(D, n, iters, chivi=False):
    from viabel_amd import vb, targets
    if chivi:
        fam = vb.mean_field_t_variational_family(D, 40.0, rng='philox')
        obj = vb.black_box_chivi(2.0, fam, targets.funnel(D), n)
    else:
        fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
        obj = vb.black_box_klvi(fam, targets.isogauss(D), n)
    fam.stream, fam.step = 7, 0      # the same Philox draws in every call
    lam0 = np.concatenate([np.zeros(D), np.ones(D) * 0.1])
    return vb.adagrad_optimize(iters, obj, lam0, learning_rate_end=.001)


def test_reused_blocks_give_the_same_runs():
    ref = _fit(2, 100, 500)
    for D, n, iters, chivi in [(10, 128, 300, True), (2, 100, 500, False), (64, 32, 37, False),
                               (2, 100, 500, False)]:
        other = _fit(D, n, iters, chivi)
        assert np.all(np.isfinite(other[0]))
        again = _fit(2, 100, 500)
        for a, b in zip(ref, again):
            if a is None:
                assert b is None
                continue
            np.testing.assert_array_equal(np.asarray(a), np.asarray(b))


def test_restart_tables_repeat_bitwise():
    from viabel_amd import vb, targets, restarts
    fac = lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox')
    tgt = targets.eight_schools_ncp()
    a = restarts.run_restarts(fac, tgt, 8, 200, n_bounds=20000)
    restarts.run_restarts(fac, tgt, 5, 50, n_bounds=3000)
    b = restarts.run_restarts(fac, tgt, 8, 200, n_bounds=20000)
    np.testing.assert_array_equal(a, b)
