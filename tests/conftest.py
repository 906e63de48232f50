import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP kernels)')
    # adagrad_optimize's progress bar (vb.py:354) off in tests; tests that check it
    # turn it back on
    os.environ.setdefault('VIABEL_AMD_PROGRESS', '0')
    _build_missing()


def _build_missing():
    """Build the oracle's C library and the HIP library if a fresh checkout
    lacks them (hipcc cross-compiles without a GPU)."""
    import subprocess
    if not os.path.exists(os.path.join(ROOT, 'oracle', 'liboracle_rng.so')):
        subprocess.call(['make', '-s', '-C', os.path.join(ROOT, 'oracle')])
    if not os.path.exists(os.path.join(ROOT, 'viabel_amd', 'libviabel_amd.so')):
        subprocess.call(['make', '-s', '-j8', '-C', os.path.join(ROOT, 'viabel_amd', 'csrc')])


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope='session')
def golden():
    import numpy as np
    d = os.path.join(ROOT, 'tests', 'golden')
    return {k: np.load(os.path.join(d, k + '_golden.npz')) for k in ('bounds', 'psis', 'rng')}
