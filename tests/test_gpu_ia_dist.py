"""The rank-sharded IA / R-hat path with the NATIVE per-rank work
(restarts.run_ia_chains, vb.rmsprop_IA_optimize_with_rhat(sharded=True);
vb.py:392-712, functions.py:8-77):

* the two R-hat stages (vb_rhat_stats, vb_rhat_combine) equal vb_rhat bit for
  bit and the oracle's compute_R_hat to 1e-12;
* the sharded driver without torch.distributed equals the one-process
  optimiser (same Philox chains, R-hat diagnostics bit for bit);
* a world_size-2 gloo group whose two ranks both run their chains on the box's
  GPU: r_hat_mean / r_hat_sigma / the halfway R-hats and start_avg_* equal the
  one-process run's to 1e-12 on both ranks.
"""
import os
import pickle
import socket

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]

D, N, N_ITERS, N_OPT = 10, 50, 1200, 5
KW = dict(window=20, learning_rate=.01, rhat_window=100, n_optimisers=N_OPT,
          tail_avg_iters=400, learning_rate_end=.001)
LOG_KEYS = ('r_hat_mean', 'r_hat_sigma', 'r_hat_mean_halfway', 'r_hat_sigma_halfway')


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rhat_stages_equal_vb_rhat_and_oracle():
    from viabel_amd import functions
    from oracle import functions_oracle as fo
    rs = np.random.RandomState(11)
    chains = rs.randn(6, 2000, 7).cumsum(axis=1) * 0.01 + rs.randn(6, 1, 7)
    segs = functions.adaptive_segments(6, 2000, 7, 200) + functions.halfway_segments(6, 2000, 7,
                                                                                     100, 200)
    whole = functions._rhat_batch(chains, segs, return_var=True)
    lens = [n for _, n in segs]
    # stats of the chains in two groups (as two ranks would), interleaved back
    ma, sa = functions.rhat_stats(chains[0::2], segs)
    mb, sb = functions.rhat_stats(chains[1::2], segs)
    J = len(segs)
    mean = np.empty((J, 12, 7))
    ss = np.empty((J, 12, 7))
    for i, c in enumerate(range(0, 6, 2)):
        mean[:, 2 * c:2 * c + 2], ss[:, 2 * c:2 * c + 2] = ma[:, 2 * i:2 * i + 2], sa[:, 2 * i:2 * i + 2]
    for i, c in enumerate(range(1, 6, 2)):
        mean[:, 2 * c:2 * c + 2], ss[:, 2 * c:2 * c + 2] = mb[:, 2 * i:2 * i + 2], sb[:, 2 * i:2 * i + 2]
    var, out = functions.rhat_combine(mean, ss, lens, return_var=True)
    np.testing.assert_array_equal(out, whole[1])
    np.testing.assert_array_equal(var, whole[0])
    for j, (s, n) in enumerate(segs):
        ov, orr = fo.compute_R_hat(chains[:, s:s + n], warmup=0)
        np.testing.assert_allclose(out[j], orr, rtol=1e-12)
        np.testing.assert_allclose(var[j], ov, rtol=1e-12)


def _objective():
    from viabel_amd import vb, targets
    fam = vb.mean_field_t_variational_family(D, 40.0, rng='philox')
    fam.stream = 500      # (families get distinct default streams): the same chains every call
    return vb.black_box_klvi(fam, targets.eight_schools_ncp(), N)


@pytest.mark.parametrize('which', ['rmsprop', 'adam'])
def test_sharded_driver_one_process_equals_optimizer(which):
    from viabel_amd import vb
    run = getattr(vb, which + '_IA_optimize_with_rhat')
    init = np.zeros(2 * D)
    a = run(N_ITERS, _objective(), init, D, **KW)
    b = run(N_ITERS, _objective(), init, D, sharded=True, **KW)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[4], b[4])
    for k in LOG_KEYS:
        np.testing.assert_array_equal(a[6][k], b[6][k])
    for k in ('start_avg_mean_iters', 'start_avg_sigma_iters'):
        assert a[6][k] == b[6][k]
    for x, y in zip(a[2] + a[3], b[2] + b[3]):
        np.testing.assert_array_equal(x, y)


def _gloo_worker(rank, world, port, out_dir, which):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), LOCAL_RANK=str(rank),
                      VIABEL_AMD_PROGRESS='0')
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from viabel_amd import vb
    run = getattr(vb, which + '_IA_optimize_with_rhat')
    res = run(N_ITERS, _objective(), np.zeros(2 * D), D, sharded=True, **KW)
    with open(os.path.join(out_dir, 'res_%d.pkl' % rank), 'wb') as f:
        pickle.dump(res, f)
    dist.destroy_process_group()


@pytest.mark.parametrize('which', ['rmsprop', 'adam'])
def test_gloo_world2_sharded_rhat_matches_single_process(tmp_path, which):
    import torch.multiprocessing as mp
    from viabel_amd import vb
    mp.spawn(_gloo_worker, args=(2, _free_port(), str(tmp_path), which), nprocs=2, join=True)
    single = getattr(vb, which + '_IA_optimize_with_rhat')(N_ITERS, _objective(), np.zeros(2 * D),
                                                           D, **KW)
    for rank, ids in ((0, [0, 2, 4]), (1, [1, 3])):
        res = pickle.load(open(tmp_path / ('res_%d.pkl' % rank), 'rb'))
        log = res[6]
        assert log['chain_ids'] == ids
        for k in LOG_KEYS:
            np.testing.assert_allclose(log[k], single[6][k], rtol=1e-12, atol=0)
        for k in ('start_avg_mean_iters', 'start_avg_sigma_iters'):
            assert log[k] == single[6][k]
        np.testing.assert_allclose(res[0], single[0], rtol=1e-12)
        np.testing.assert_allclose(res[4], single[4], rtol=1e-12)
        np.testing.assert_allclose(res[1], single[1][ids], rtol=1e-12)
