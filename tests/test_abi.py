"""C-ABI checks that need no GPU: the library loads, exports every function
declared in include/viabel_amd.h, the ctypes descriptors match the header's
struct layouts, and the product fails loudly (no CPU fallback) without a GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT, gpu_available

HEADER = os.path.join(ROOT, 'include', 'viabel_amd.h')


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(vb_[a-z0-9_]+)\s*\(', src)))


def test_header_declares_the_hot_path():
    fns = header_functions()
    for f in ('vb_objective_value_grad', 'vb_run_create', 'vb_run_advance', 'vb_log_weights',
              'vb_divergence_bound', 'vb_centered_moments', 'vb_psislw', 'vb_gpdfit'):
        assert f in fns


def test_library_exports_every_header_symbol():
    from viabel_amd import _native
    lib = _native.lib()
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing
    # and the ctypes binding covers all of them
    assert set(header_functions()) == set(_native._SIGNATURES)
    assert lib.vb_abi_version() == 1


def source_hash():
    """sha256 prefix of the library sources in Makefile HASH_SRCS order (the
    recipe vb_build_id() was made with)."""
    import hashlib
    csrc = os.path.join(ROOT, 'viabel_amd', 'csrc')
    mk = open(os.path.join(csrc, 'Makefile')).read()
    names = re.search(r'HASH_SRCS = (.*?)\nSRC_HASH', mk, re.S).group(1).replace('\\\n', ' ').split()
    h = hashlib.sha256()
    for n in names:
        h.update(open(os.path.join(csrc, n), 'rb').read())
    return h.hexdigest()[:16]


def test_library_was_built_from_these_sources():
    """The loaded libviabel_amd.so carries the hash of the sources it was built
    from (vb_build_id): it equals the hash of the tree the tests run in, so the
    binary under test is the source under review (GPU box: the same check runs
    as test_gpu_vb.py::test_gpu_library_was_built_from_these_sources)."""
    from viabel_amd import _native
    assert _native.lib().vb_build_id().decode() == source_hash()


def test_exported_symbols_are_c_linkage():
    so = os.path.join(ROOT, 'viabel_amd', 'libviabel_amd.so')
    out = subprocess.check_output(['nm', '-D', '--defined-only', so]).decode()
    syms = set(re.findall(r' T (vb_[a-z0-9_]+)$', out, flags=re.M))
    assert set(header_functions()) <= syms


def _struct_sizes_from_c():
    """Compile a tiny C program against the header to get sizeof/offsetof."""
    import tempfile
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "viabel_amd.h"
int main(void){
  printf("%zu %zu %zu %zu %zu\n", sizeof(vb_family), sizeof(vb_target), sizeof(vb_objective),
         sizeof(vb_noise), sizeof(vb_adagrad_config));
  printf("%zu %zu %zu\n", offsetof(vb_noise, eps), offsetof(vb_objective, n_samples),
         offsetof(vb_adagrad_config, epsilon));
  return 0; }
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, 'p.c')
        exe = os.path.join(d, 'p')
        open(c, 'w').write(prog)
        subprocess.check_call(['gcc', '-I', os.path.join(ROOT, 'include'), c, '-o', exe])
        lines = subprocess.check_output([exe]).decode().split('\n')
    return [int(v) for v in lines[0].split()], [int(v) for v in lines[1].split()]


def test_ctypes_layouts_match_header():
    from viabel_amd import _native as n
    sizes, offs = _struct_sizes_from_c()
    assert sizes == [ctypes.sizeof(n.Family), ctypes.sizeof(n.Target), ctypes.sizeof(n.Objective),
                     ctypes.sizeof(n.Noise), ctypes.sizeof(n.AdagradConfig)]
    assert offs == [n.Noise.eps.offset, n.Objective.n_samples.offset,
                    n.AdagradConfig.epsilon.offset]


@pytest.mark.skipif(gpu_available(), reason='checks the no-GPU failure mode')
def test_no_gpu_fails_loudly():
    from viabel_amd import _native, vb, targets
    _native._ctx.clear()
    with pytest.raises(RuntimeError):
        _native.Context(0)
    fam = vb.mean_field_gaussian_variational_family(3)
    obj = vb.black_box_klvi(fam, targets.isogauss(3), 10)
    with pytest.raises(RuntimeError):
        obj(np.zeros(6))


def test_api_argument_errors_without_gpu():
    """Argument validation that the reference performs before any compute."""
    from viabel_amd import vb, targets
    with pytest.raises(ValueError, match='df must be greater than 2'):
        vb.mean_field_t_variational_family(3, 2)
    fam = vb.mean_field_gaussian_variational_family(3)
    with pytest.raises(ValueError, match='only p = 2 or 4 supported'):
        fam.pth_moment(3, np.zeros(6))
    # a callable torch cannot differentiate (vb.py:236-241 takes any autograd
    # callable; only torch-differentiable ones can be wrapped here)
    with pytest.raises(TypeError, match='viabel_amd.targets'):
        vb.black_box_klvi(fam, lambda x: np.asarray(x).sum(1), 10)
    # a torch-differentiable callable is wrapped as a host-callback target
    obj = vb.black_box_klvi(fam, lambda x: -0.5 * (x ** 2).sum(1), 10)
    assert obj.target.kind == targets.callback(lambda x: None, 3).kind
    with pytest.raises(ValueError, match='learning rate must be positive'):
        vb.adagrad_optimize(10, vb.black_box_klvi(fam, targets.isogauss(3), 5), np.zeros(6),
                            learning_rate=0)
    with pytest.raises(ValueError, match='initial learning rate must be greater'):
        list(vb.learning_rate_schedule(10, 0.01, 0.1))
    tfam = vb.mean_field_t_variational_family(3, 3.5)
    with pytest.raises(ValueError, match='df must be greater than p'):
        tfam.pth_moment(4, np.zeros(6))


def test_host_side_closed_forms():
    """entropy / mean_and_cov / pth_moment follow vb.py:59-79, 153-179."""
    from viabel_amd import vb
    from oracle import vb_oracle
    lam = np.array([0.1, -0.3, 0.2, -0.5, 0.4, 0.05])
    for kind, df in (('gauss', None), ('t', 7.0)):
        fam = (vb.mean_field_gaussian_variational_family(3) if kind == 'gauss'
               else vb.mean_field_t_variational_family(3, df))
        ofam = vb_oracle.Family(kind, 3, df)
        assert fam.entropy(lam) == pytest.approx(ofam.entropy(lam), rel=1e-15)
        for p in (2, 4):
            assert fam.pth_moment(p, lam) == pytest.approx(ofam.pth_moment(p, lam), rel=1e-14)
        m, c = fam.mean_and_cov(lam)
        om, oc = ofam.mean_and_cov(lam)
        np.testing.assert_array_equal(m, om)
        np.testing.assert_allclose(c, oc, rtol=1e-15)
        assert fam.var_param_dim == 6


def test_viabel_namespace_is_the_device_implementation():
    """`from viabel import ...` (reference tests/test_bounds.py:1-2,
    viabel/__init__.py:1), `viabel.vb`, `viabel.bounds`, `viabel.functions` and
    the notebooks' top-level `psis` / `experiments` resolve to viabel_amd."""
    import importlib
    import viabel
    import viabel_amd
    from viabel import all_bounds, error_bounds, wasserstein_bounds, divergence_bound
    assert all_bounds is viabel_amd.bounds.all_bounds
    assert divergence_bound is viabel_amd.divergence_bound
    assert (error_bounds, wasserstein_bounds) == (viabel_amd.error_bounds,
                                                  viabel_amd.wasserstein_bounds)
    vbm = importlib.import_module('viabel.vb')
    assert vbm is viabel_amd.vb is viabel.vb
    assert importlib.import_module('viabel.bounds') is viabel_amd.bounds
    assert importlib.import_module('viabel.functions') is viabel_amd.functions
    from viabel.vb import (mean_field_gaussian_variational_family, black_box_klvi,  # noqa: F401
                           black_box_chivi, adagrad_optimize, t_variational_family)
    from viabel.bounds import mean_and_check_mc_error  # noqa: F401
    psis = importlib.import_module('psis')
    assert psis is viabel_amd.psis
    from psis import psislw, gpdfitnew, gpinv, sumlogs  # noqa: F401
    assert importlib.import_module('experiments') is viabel_amd.experiments
    # the same errors as the reference, before any device work
    with pytest.raises(ValueError, match='alpha must be greater than 1'):
        divergence_bound(np.zeros(3), alpha=1.0)
    with pytest.raises(ValueError, match='must provides samples'):
        wasserstein_bounds(1.0)
