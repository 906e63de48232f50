"""The drop-in namespace: every name the reference notebooks import from
``viabel``, ``viabel.vb``, ``viabel.functions``, ``psis`` and ``experiments``
resolves (names the reference itself defines; the notebooks also name
black_box_chivi_neff / perturbed_black_box_vi / adagrad_perturb_optimize, which
/root/reference/viabel/vb.py does not define either, so those imports fail there
too).  Out-of-scope names import and raise NotImplementedError on call.  No GPU."""
import importlib

import numpy as np
import pytest

# (module, names) as in the import cells of /root/reference/notebooks/*.ipynb
NOTEBOOK_IMPORTS = [
    ('viabel', ['all_bounds']),
    ('viabel.functions', ['compute_posterior_moments']),
    ('viabel.vb', ['mean_field_gaussian_variational_family', 'mean_field_t_variational_family',
                   'full_rank_gaussian_variational_family', 't_variational_family',
                   'black_box_klvi', 'black_box_klvi_pd', 'black_box_klvi_pd2', 'black_box_chivi',
                   'make_stan_log_density', 'adagrad_optimize',
                   'rmsprop_IA_optimize_with_rhat', 'adam_IA_optimize_with_rhat']),
    ('experiments', ['get_samples_and_log_weights', 'improve_with_psis', 'plot_history',
                     'plot_approx_and_exact_contours', 'plot_dist_to_opt_param',
                     'check_approx_accuracy', 'print_bounds', 'run_experiment']),
    ('psis', ['psislw']),
]


@pytest.mark.parametrize('mod,names', NOTEBOOK_IMPORTS)
def test_notebook_import_cells_resolve(mod, names):
    m = importlib.import_module(mod)
    missing = [n for n in names if not hasattr(m, n)]
    assert not missing, (mod, missing)


def test_star_import_of_experiments():
    ns = {}
    exec('from experiments import *', ns)
    for n in ('print_bounds', 'improve_with_psis', 'check_accuracy'):
        assert n in ns


@pytest.mark.parametrize('name', ['plot_history', 'plot_approx_and_exact_contours',
                                  'plot_dist_to_opt_param', 'run_experiment'])
def test_out_of_scope_experiment_helpers_raise_on_call(name):
    import experiments
    with pytest.raises(NotImplementedError):
        getattr(experiments, name)(None)


def test_full_rank_gaussian_raises_on_call():
    from viabel.vb import full_rank_gaussian_variational_family
    with pytest.raises(NotImplementedError):
        full_rank_gaussian_variational_family(3)


def test_print_bounds(capsys):
    from experiments import print_bounds
    print_bounds(dict(W2=1.23456, d2=0.5, mean_error=2e-3, std_error=3.0, cov_error=4.0))
    out = capsys.readouterr().out.splitlines()
    assert out == ['Bounds on...', '  2-Wasserstein   1.23', '  2-divergence    0.5',
                   '  mean error      0.002', '  stdev error     3', '  sqrt cov error  2',
                   '  cov error       4']


def test_safe_root():
    from viabel.functions import safe_root
    assert safe_root(49) == 7 and safe_root(1) == 1
    with pytest.raises(ValueError, match='N is not square!'):
        safe_root(50)


def test_flat_triang_round_trip():
    """functions.py:106-136: row m of the triangle holds flat entries in order."""
    from viabel.functions import flat_to_triang, triang_to_flat
    M = 4
    flat = np.arange(1.0, M * (M + 1) // 2 + 1)
    T = flat_to_triang(flat)
    expect = np.zeros((M, M))
    c = 0
    for m in range(M):
        for mm in range(m + 1):
            expect[m, mm] = flat[c]
            c += 1
    np.testing.assert_array_equal(T, expect)
    stack = np.stack([T, 2 * T, -T])
    F = triang_to_flat(stack)
    assert F.shape == (M * (M + 1) // 2, 3)
    np.testing.assert_array_equal(F[:, 0], flat)
    np.testing.assert_array_equal(F[:, 1], 2 * flat)
    np.testing.assert_array_equal(F[:, 2], -flat)


def test_triang_to_flat_follows_the_reference_loops():
    """triang_to_flat on a random stack with a non-zero upper triangle (ignored)
    against the reference's index loops restated (functions.py:126-136):
    flat[count, d] = L[d, m, mm] for m = 0..M-1, mm = 0..m; shape [N, B]."""
    from viabel.functions import triang_to_flat
    rs = np.random.RandomState(3)
    for B, M in ((1, 1), (2, 5), (7, 3)):
        L = rs.randn(B, M, M)
        flat = np.empty((M * (M + 1) // 2, B))
        for d in range(B):
            count = 0
            for m in range(M):
                for mm in range(m + 1):
                    flat[count, d] = L[d, m, mm]
                    count += 1
        np.testing.assert_array_equal(triang_to_flat(L), flat)


def test_compute_posterior_moments_is_the_conjugate_posterior():
    from viabel.functions import compute_posterior_moments
    rs = np.random.RandomState(3)
    d, n = 5, 40
    A = rs.randn(d, d)
    prior_cov = A @ A.T + d * np.eye(d)
    prior_mean = rs.randn(d)
    x = rs.randn(n, d)
    y = x @ rs.randn(d) + 0.3 * rs.randn(n)
    mu, S = compute_posterior_moments(prior_mean, prior_cov, 0.09, x, y)
    P = np.linalg.inv(prior_cov) + x.T @ x / 0.09
    S_ref = np.linalg.inv(P)
    np.testing.assert_allclose(S, S_ref, rtol=1e-10, atol=1e-14)
    np.testing.assert_allclose(mu, S_ref @ (np.linalg.solve(prior_cov, prior_mean) + x.T @ y / 0.09),
                               rtol=1e-10)
