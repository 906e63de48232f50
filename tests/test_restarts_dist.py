"""Multi-process path of the sharded restarts: world_size 2 over
gloo on the CPU.  The per-rank compute is injected (the oracle fits each
restart on its own Philox stream 1 + r, exactly as the device run does), so
the test checks the sharding and the all_gather without a GPU: the gathered
table must equal the single-process table bit for bit."""
import os
import socket
import warnings

import numpy as np
import pytest
import torch.multiprocessing as mp

N_RESTARTS, N_ITERS, N_SAMPLES, D = 5, 30, 16, 10


def oracle_compute(ids, inits):
    from oracle import vb_oracle, rng_oracle, bounds_oracle, psis_oracle
    recs = []
    for r, init in zip(ids, inits):
        fam = vb_oracle.Family('t', D, 40.0)
        step = [0]

        def f(lam):
            eps = rng_oracle.noise(0, 1 + r, step[0], N_SAMPLES, D, 't', 40.0)
            step[0] += 1
            return vb_oracle.klvi_value_grad(fam, 'eight_schools_ncp', lam, N_SAMPLES, eps=eps)
        opt, hist, vals, _ = vb_oracle.adagrad_optimize(N_ITERS, f, init, learning_rate=.01,
                                                        learning_rate_end=.001)
        eps = rng_oracle.noise(0, (1 << 20) + r, 0, 2000, D, 't_bailey', 40.0)
        _, lw = vb_oracle.log_weights(fam, 'eight_schools_ncp', opt, 2000, eps=eps)
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            res = bounds_oracle.all_bounds(lw, q_var=fam.mean_and_cov(opt)[1],
                                           moment_bound_fn=lambda p: fam.pth_moment(p, opt))
            _, khat = psis_oracle.psislw(lw)
        recs.append(np.concatenate([[r, np.mean(lw), res['d2'], res['W1'], res['W2'],
                                     res['mean_error'], res['std_error'], res['cov_error'],
                                     khat, vals[-1]], opt]))
    return np.array(recs)


def _factory():
    from viabel_amd import vb
    return vb.mean_field_t_variational_family(D, 40, rng='philox')


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from viabel_amd import restarts, targets
    table = restarts.run_restarts(_factory, targets.eight_schools_ncp(), N_RESTARTS, N_ITERS,
                                  n_samples=N_SAMPLES, compute=oracle_compute)
    np.save(os.path.join(out_dir, 'table_%d.npy' % rank), table)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_assignment():
    from viabel_amd.restarts import shard
    assert shard(5, 0, 2) == [0, 2, 4] and shard(5, 1, 2) == [1, 3]
    assert sorted(shard(64, 0, 8) + sum((shard(64, r, 8) for r in range(1, 8)), [])) == list(range(64))


def test_gloo_world2_gather_matches_single_process(tmp_path):
    from viabel_amd import restarts, targets
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    t0 = np.load(tmp_path / 'table_0.npy')
    t1 = np.load(tmp_path / 'table_1.npy')
    single = restarts.run_restarts(_factory, targets.eight_schools_ncp(), N_RESTARTS, N_ITERS,
                                   n_samples=N_SAMPLES, compute=oracle_compute)
    assert t0.shape == (N_RESTARTS, len(restarts.RECORD_HEAD) + 2 * D)
    np.testing.assert_array_equal(t0, t1)
    np.testing.assert_array_equal(t0, single)
    np.testing.assert_array_equal(t0[:, 0], np.arange(N_RESTARTS))
