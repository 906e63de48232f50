"""Every A/B environment switch of the library (README "Environment switches")
against the default path, on the GPU.  Switches are read once per process, so
each side runs in a child process; the child writes its run's result
(lambda, history, values) and the test compares.

* VIABEL_AMD_BLOCK_PF=0 (block kernel: device-noise rows from HBM instead of the
  copy wave's LDS ring): the same draws; the copy-wave layout splits each sample
  over two lanes (split rows), so the sums run in another order -> equal to
  rounding (1e-12 of the largest entry over 400 steps).
* VIABEL_AMD_FR_FUSE=0 / GEMM_SYM=0 / FR_SCHED_FUSE=0 / FR_WEIGHTS_FUSE=0 /
  FR_PCG_SS=0 (full rank: separate launches, full symmetric products, the schedule
  and the weights in their own kernels, the PCG's products and vector updates as
  separate launches): other reduction / contraction orders -> equal to 1e-9
  of the largest entry over a short trajectory.  VIABEL_AMD_GEMM_SK=0 (the
  Newton-Schulz Y|Z pair without stream-K) likewise, at D = 512.
* VIABEL_AMD_HOST_TRACE=1 (host timestamps of the column-pair launch path on
  stderr): the same bits, and the trace lines are there.
* VIABEL_AMD_PSIS_WORKER=1 (restart table: the PSIS k-hats on a worker thread):
  the same bits.
* VIABEL_AMD_DIV_TWO_PASS=0 (divergence statistics in numpy's three passes at every
  size): equal to the two-pass Welford / Chan form to rounding.
(VIABEL_AMD_PREDRAW, _BLOCK_SPLIT, _PREDRAW_OVERLAP, _GEMM_EPI_EXACT,
_PSIS_FAST_SELECT and _FR_NS_START have their own tests in test_gpu_vb.py,
test_gpu_configs.py, test_gpu_fullrank.py and test_gpu_bounds_psis.py.)
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason='needs an MI355X')]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = '''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import viabel_amd.vb as vb
from viabel_amd import targets
kind = sys.argv[3]
if kind == 'block':
    D, N = 10, 128
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj = vb.black_box_klvi(fam, targets.funnel(D), N)
    rs = np.random.RandomState(5)
    init = np.stack([np.concatenate([rs.randn(D) * 0.3, rs.randn(D) * 0.2 - 0.5]) for _ in range(3)])
    run = vb.DeviceRun(obj, 400, init, learning_rate=0.01)
    run.advance_philox(7, 3, 2, 0)
    run.advance_philox(393, 3, 2, 7)
elif kind in ('fullrank', 'fullrank512'):
    D, N = (512, 128) if kind == 'fullrank512' else (64, 32)
    rs = np.random.RandomState(9)
    tri = np.tril_indices(D)
    free = rs.randn(len(tri[0])) * 0.01
    free[tri[0] == tri[1]] = rs.randn(D) * 0.1
    lam0 = np.concatenate([rs.randn(D) * 0.1, free])
    fam = vb.t_variational_family(D, 30.0, rng='philox')
    obj = vb.black_box_chivi(2.0, fam, targets.corr_gauss(D), N)
    run = vb.DeviceRun(obj, 12, lam0, learning_rate=0.02)
    run.advance_philox(5, 1, 4, 0)
    run.advance_philox(7, 1, 4, 5)
else:
    D, N = 40, 128
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    run = vb.DeviceRun(obj, 45, init[None, :])
    run.advance_philox(5, 0, 1, 0)
    run.advance_philox(20, 0, 1, 5)
    run.advance_philox(20, 0, 1, 25)
lam, hist, vals, smooth = run.result()
np.savez(sys.argv[2], lam=lam, hist=hist, vals=vals)
'''


def _run(tmp_path, kind, env_extra, tag):
    f = str(tmp_path / ('%s_%s.npz' % (kind, tag)))
    env = dict(os.environ)
    for k in [k for k in env if k.startswith('VIABEL_AMD_') and k not in ('VIABEL_AMD_LIB',
                                                                        'VIABEL_AMD_DEVICE')]:
        if k != 'VIABEL_AMD_PROGRESS':
            del env[k]
    env.update(env_extra)
    r = subprocess.run([sys.executable, '-c', _CHILD, ROOT, f, kind], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return dict(np.load(f)), r.stderr


def _close(a, b, rtol):
    scale = max(1.0, float(np.max(np.abs(b))))
    err = float(np.max(np.abs(a - b))) / scale
    assert err <= rtol, 'max scaled error %.3e > %.1e' % (err, rtol)


def test_block_pf_off_matches_default(tmp_path):
    ref, _ = _run(tmp_path, 'block', {}, 'default')
    out, _ = _run(tmp_path, 'block', {'VIABEL_AMD_BLOCK_PF': '0'}, 'pf0')
    for k in ('lam', 'hist', 'vals'):
        _close(out[k], ref[k], 1e-12)


@pytest.mark.parametrize('switch', ['VIABEL_AMD_FR_FUSE', 'VIABEL_AMD_GEMM_SYM',
                                    'VIABEL_AMD_FR_SCHED_FUSE', 'VIABEL_AMD_FR_WEIGHTS_FUSE',
                                    'VIABEL_AMD_FR_PCG_SS'])
def test_full_rank_switch_off_matches_default(tmp_path, switch):
    ref, _ = _run(tmp_path, 'fullrank', {}, 'default')
    out, _ = _run(tmp_path, 'fullrank', {switch: '0'}, 'off')
    for k in ('lam', 'hist', 'vals'):
        _close(out[k], ref[k], 1e-9)


def test_gemm_sk_off_matches_default(tmp_path):
    """VIABEL_AMD_GEMM_SK=0 (the Newton-Schulz Y|Z pair as one block per tile) against
    the default stream-K launch at D = 512, where the pair's 272 tiles exceed the 256
    CUs and stream-K runs: the split tiles add their two k parts in another order ->
    equal to 1e-9 of the largest entry over 12 steps (as the other full-rank
    switches)."""
    ref, _ = _run(tmp_path, 'fullrank512', {}, 'default')
    out, _ = _run(tmp_path, 'fullrank512', {'VIABEL_AMD_GEMM_SK': '0'}, 'off')
    assert np.all(np.isfinite(ref['vals']))
    for k in ('lam', 'hist', 'vals'):
        _close(out[k], ref[k], 1e-9)


def test_host_trace_is_bitwise_default_and_prints(tmp_path):
    ref, _ = _run(tmp_path, 'sep', {}, 'default')
    out, err = _run(tmp_path, 'sep', {'VIABEL_AMD_HOST_TRACE': '1'}, 'trace')
    for k in ('lam', 'hist', 'vals'):
        np.testing.assert_array_equal(out[k], ref[k])
    assert 'sep advance' in err, err[-2000:]


_RESTARTS_CHILD = '''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from viabel_amd import vb, targets, restarts
fac = lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox')
tab = restarts.run_restarts(fac, targets.eight_schools_ncp(), 6, 200, n_samples=100,
                            n_bounds=200_000, learning_rate=.01, learning_rate_end=.001)
np.save(sys.argv[2], tab)
'''


def test_psis_worker_switch_is_bitwise(tmp_path):
    """VIABEL_AMD_PSIS_WORKER=1 (the restart table's PSIS k-hats on a worker thread
    beside the host bound algebra) against the default serial order: the same calls
    on the same device buffers, so the same table bit for bit."""
    out = {}
    for tag, env in (('serial', {}), ('worker', {'VIABEL_AMD_PSIS_WORKER': '1'})):
        path = str(tmp_path / ('%s.npy' % tag))
        e = dict(os.environ)
        e.pop('VIABEL_AMD_PSIS_WORKER', None)
        e.update(env)
        subprocess.check_call([sys.executable, '-c', _RESTARTS_CHILD, ROOT, path], env=e,
                              timeout=300)
        out[tag] = np.load(path)
    assert np.all(np.isfinite(out['serial'][:, 8]))
    np.testing.assert_array_equal(out['worker'], out['serial'])


_DIV_CHILD = '''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from viabel_amd import bounds
rs = np.random.RandomState(17)
lw = np.stack([rs.standard_t(5.0, 300_000) * 0.7 - 3.0, rs.randn(300_000) * 2.0 + 1.0])
np.save(sys.argv[2], bounds.divergence_rows(lw))
'''


def test_div_two_pass_switch(tmp_path):
    """VIABEL_AMD_DIV_TWO_PASS=0 (the three-pass divergence statistics at every
    size) against the default two-pass Welford / Chan form at n = 3e5: equal to
    rounding (1e-12 relative), and both equal to the oracle's divergence_bound
    statistics (bounds.py:142-192, numpy's definitions) to 1e-12."""
    from oracle import bounds_oracle
    out = {}
    for tag, env in (('two', {}), ('three', {'VIABEL_AMD_DIV_TWO_PASS': '0'})):
        path = str(tmp_path / ('%s.npy' % tag))
        subprocess.check_call([sys.executable, '-c', _DIV_CHILD, ROOT, path],
                              env=dict(os.environ, **env), timeout=300)
        out[tag] = np.load(path)
    np.testing.assert_allclose(out['two'], out['three'], rtol=1e-12, atol=1e-14)
    rs = np.random.RandomState(17)
    lw = np.stack([rs.standard_t(5.0, 300_000) * 0.7 - 3.0, rs.randn(300_000) * 2.0 + 1.0])
    import warnings
    for j in range(2):
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            d, lnb = bounds_oracle.divergence_bound(lw[j], return_log_norm_bound=True)
        np.testing.assert_allclose(out['two'][j, :2], [d, lnb], rtol=1e-12)
        r = np.exp(2 * (lw[j] - lw[j].max()))
        np.testing.assert_allclose(out['two'][j, 2:7],
                                   [r.mean(), r.std() / np.sqrt(r.size), lw[j].mean(),
                                    lw[j].std() / np.sqrt(lw[j].size), lw[j].max()], rtol=1e-12)
