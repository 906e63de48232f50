"""Config 5's sharded restarts with the NATIVE per-rank compute.

* a world_size-1 NCCL (RCCL) group: run_restarts binds the rank's GPU, fits all
  restarts in one device launch chain, computes log weights / bounds / PSIS on
  the device and all-gathers the records over RCCL; the table must equal the
  oracle's per-restart recomputation on the same Philox streams
  (tests/test_restarts_dist.oracle_compute);
* a world_size-2 gloo group whose two ranks both compute on the box's GPU: the
  gathered table must equal the single-process table (restart r draws from
  stream 1 + r whatever the sharding, so the split changes nothing).
"""
import os
import socket
import warnings

import numpy as np
import pytest

from tests.conftest import gpu_available
from tests.test_restarts_dist import (D, N_ITERS, N_RESTARTS, N_SAMPLES, _factory,
                                      oracle_compute)

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]

M = 2000   # log weights per restart (oracle_compute's size)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _native_table():
    from viabel_amd import restarts, targets
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        return restarts.run_restarts(_factory, targets.eight_schools_ncp(), N_RESTARTS, N_ITERS,
                                     n_samples=N_SAMPLES, n_bounds=M)


def test_nccl_world1_native_matches_oracle():
    import torch
    import torch.distributed as dist
    os.environ.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % _free_port(), rank=0,
                            world_size=1, device_id=torch.device('cuda', 0))
    try:
        from viabel_amd import restarts
        table = _native_table()
        assert dist.get_backend() == 'nccl'
        assert torch.cuda.current_device() == 0
    finally:
        dist.destroy_process_group()
    expect = oracle_compute(list(range(N_RESTARTS)),
                            restarts.default_inits(N_RESTARTS, 2 * D))
    assert table.shape == expect.shape == (N_RESTARTS, len(restarts.RECORD_HEAD) + 2 * D)
    np.testing.assert_array_equal(table[:, 0], np.arange(N_RESTARTS))
    # fitted lambda* and final values: trajectories of 30 steps (<= 1e-7 bar)
    np.testing.assert_allclose(table[:, 9:], expect[:, 9:], rtol=1e-8, atol=1e-10)
    # bounds and k-hat from M log weights at those lambda*
    np.testing.assert_allclose(table[:, 1:9], expect[:, 1:9], rtol=1e-6, atol=1e-9)


def _gloo_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    table = _native_table()
    from viabel_amd import _native as nat
    np.save(os.path.join(out_dir, 'table_%d.npy' % rank), table)
    np.save(os.path.join(out_dir, 'dev_%d.npy' % rank), np.array([nat.context().device]))
    dist.destroy_process_group()


def test_gloo_world2_native_compute_matches_single_process(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_gloo_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    t0 = np.load(tmp_path / 'table_0.npy')
    t1 = np.load(tmp_path / 'table_1.npy')
    np.testing.assert_array_equal(t0, t1)
    single = _native_table()
    np.testing.assert_allclose(t0, single, rtol=1e-13, atol=1e-15)
    # both ranks bound a GPU (LOCAL_RANK mod the visible count: one GPU here)
    import torch
    n = torch.cuda.device_count()
    assert [int(np.load(tmp_path / ('dev_%d.npy' % r))[0]) for r in range(2)] == [0 % n, 1 % n]


def test_numpy_rng_factory_is_rejected():
    from viabel_amd import restarts, targets, vb
    with pytest.raises(ValueError, match='philox'):
        restarts.run_restarts(lambda: vb.mean_field_t_variational_family(D, 40, rng='numpy'),
                              targets.eight_schools_ncp(), 2, 5, n_bounds=100)


@pytest.mark.parametrize('case', ['t_eight_schools', 'gauss_mixture', 'gauss_isogauss_wide'])
def test_log_weights_rows_equal_per_row_calls(case):
    """vb_log_weights_rows (one launch for every restart's bound draws) gives the
    per-restart vb_log_weights results bit for bit (row r: stream base + r * stride)."""
    from viabel_amd import vb, targets, experiments
    if case == 't_eight_schools':
        D, fam_fn, tgt = 10, lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox'), \
            targets.eight_schools_ncp()
    elif case == 'gauss_mixture':
        D = 3
        fam_fn, tgt = lambda: vb.mean_field_gaussian_variational_family(3, rng='philox'), targets.mixture(3)
    else:
        D = 40
        fam_fn, tgt = lambda: vb.mean_field_gaussian_variational_family(40, rng='philox'), targets.isogauss(40)
    R, m = 5, 20000
    lams = np.random.RandomState(3).randn(R, 2 * D) * 0.3
    rows = experiments.log_weights_rows(tgt, fam_fn(), lams, m, stream=100, stream_stride=3)
    for r in range(R):
        f = fam_fn()
        f.stream = 100 + 3 * r
        _, lw = experiments.log_weights(tgt, f, lams[r], m, return_samples=False)
        np.testing.assert_array_equal(rows[r], lw)


def _per_restart_records(fac, tgt, R, n_iters, N, M):
    """The fallback path spelled out with the single-call API: one DeviceRun
    for all restarts (restart r: Philox stream 1 + r), then per restart
    log_weights on stream 2^20 + r, all_bounds with the family's own moments
    and covariance (bounds.py:13-61) and psislw."""
    from viabel_amd import vb, experiments, bounds, psis, restarts
    fam = fac()
    P = fam.var_param_dim
    inits = restarts.default_inits(R, P)
    run = vb.DeviceRun(vb.black_box_klvi(fam, tgt, N), n_iters, inits, learning_rate=.01,
                       learning_rate_end=.001)
    run.advance_philox(n_iters, 0, 1, 0)
    _, _, vals, smooth = run.result()
    out = []
    for r in range(R):
        f = fac()
        f.stream = (1 << 20) + r
        _, lw = experiments.log_weights(tgt, f, smooth[r], M, return_samples=False)
        res = bounds.all_bounds(lw, moment_bound_fn=lambda p, l=smooth[r]: fam.pth_moment(p, l),
                                q_var=fam.mean_and_cov(smooth[r])[1])
        k = psis.psislw(lw)[1]
        out.append(np.concatenate([[r, np.mean(lw), res['d2'], res['W1'], res['W2'],
                                    res['mean_error'], res['std_error'], res['cov_error'], k,
                                    vals[r, -1]], smooth[r]]))
    return np.array(out)


@pytest.mark.parametrize('case', ['full_rank_t', 'callback_target'])
def test_run_restarts_fallback_families_and_targets(case):
    """Families / targets the batched bound kernel does not cover (full-rank q,
    host-callback targets) take the per-restart log-weight path and the
    family's own moments (no VB_EUNSUPPORTED after the fit, no mean-field
    moment formulas applied to a full-rank q)."""
    from viabel_amd import vb, targets, restarts
    R, n_iters, N, M = 3, 25, 16, 3000
    if case == 'full_rank_t':
        fac = lambda: vb.t_variational_family(3, 10.0, rng='philox')
        tgt = targets.isogauss(3)
    else:
        fac = lambda: vb.mean_field_t_variational_family(3, 10.0, rng='philox')
        tgt = targets.callback(lambda x: (-0.5 * np.sum(x ** 2, axis=1), -x), 3)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        table = restarts.run_restarts(fac, tgt, R, n_iters, n_samples=N, n_bounds=M)
        expect = _per_restart_records(fac, tgt, R, n_iters, N, M)
    assert table.shape == expect.shape
    np.testing.assert_allclose(table, expect, rtol=1e-12, atol=1e-14)
