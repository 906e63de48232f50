"""ctypes binding of libviabel_amd.so (include/viabel_amd.h).

The product path has no CPU fallback: if the HIP library is missing, or no
GPU is visible when a computation is requested, this module raises.
"""
import atexit
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# VIABEL_AMD_LIB selects another in-tree build (e.g. an instrumented one)
LIB_PATH = os.environ.get('VIABEL_AMD_LIB') or os.path.join(_HERE, 'libviabel_amd.so')

VB_OK, VB_EINVAL, VB_EDEVICE, VB_ENOMEM, VB_EUNSUPPORTED = 0, -1, -2, -3, -4
FAMILY_MF_GAUSSIAN, FAMILY_MF_T, FAMILY_FR_T = 0, 1, 2
TARGET_ISOGAUSS, TARGET_MIXTURE, TARGET_FUNNEL, TARGET_EIGHT_SCHOOLS_NCP = 0, 1, 2, 3
TARGET_CORR_GAUSS = 4
TARGET_CALLBACK = 5
OBJ_KLVI, OBJ_CHIVI, OBJ_KLVI_PD = 0, 1, 2
OPT_ADAGRAD, OPT_RMSPROP_IA, OPT_ADAM_IA, OPT_RMSPROP_IA_NORM = 0, 1, 2, 3
NOISE_HOST, NOISE_PHILOX = 0, 1

c_double_p = ctypes.POINTER(ctypes.c_double)
c_int64_p = ctypes.POINTER(ctypes.c_int64)


class Family(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32), ('reserved', ctypes.c_int32),
                ('dim', ctypes.c_int64), ('df', ctypes.c_double)]


# vb_target_callback: (user, x, n, d, logp, grad) -> int, host pointers
TARGET_CALLBACK_T = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, c_double_p, ctypes.c_int64,
                                     ctypes.c_int64, c_double_p, c_double_p)


class Target(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32), ('reserved', ctypes.c_int32), ('dim', ctypes.c_int64),
                ('params', c_double_p), ('n_params', ctypes.c_int64),
                ('callback', TARGET_CALLBACK_T), ('user', ctypes.c_void_p)]


class Objective(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32), ('reserved', ctypes.c_int32),
                ('alpha', ctypes.c_double), ('n_samples', ctypes.c_int64)]


class Noise(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32), ('stream', ctypes.c_uint32),
                ('seed', ctypes.c_uint64), ('step', ctypes.c_uint64), ('eps', c_double_p),
                ('stream_stride', ctypes.c_uint32), ('reserved', ctypes.c_uint32)]


class AdagradConfig(ctypes.Structure):
    _fields_ = [('n_iters', ctypes.c_int64), ('window', ctypes.c_int32),
                ('optimizer', ctypes.c_int32), ('learning_rate', ctypes.c_double),
                ('learning_rate_end', ctypes.c_double), ('epsilon', ctypes.c_double)]


P = ctypes.POINTER
_SIGNATURES = {
    'vb_abi_version': ([], ctypes.c_int),
    'vb_last_error': ([], ctypes.c_char_p),
    'vb_build_id': ([], ctypes.c_char_p),
    'vb_flop_tally': ([ctypes.c_int], ctypes.c_double),
    'vb_ctx_create': ([ctypes.c_int, ctypes.c_void_p, P(ctypes.c_void_p)], ctypes.c_int),
    'vb_ctx_destroy': ([ctypes.c_void_p], ctypes.c_int),
    'vb_ctx_synchronize': ([ctypes.c_void_p], ctypes.c_int),
    'vb_ctx_stream': ([ctypes.c_void_p], ctypes.c_void_p),
    'vb_family_sample': ([ctypes.c_void_p, P(Family), c_double_p, ctypes.c_int64, P(Noise),
                          c_double_p], ctypes.c_int),
    'vb_family_logdensity': ([ctypes.c_void_p, P(Family), c_double_p, c_double_p,
                              ctypes.c_int64, c_double_p], ctypes.c_int),
    'vb_family_moments': ([ctypes.c_void_p, P(Family), c_double_p, c_double_p, c_double_p],
                          ctypes.c_int),
    'vb_target_logdensity': ([ctypes.c_void_p, P(Target), c_double_p, ctypes.c_int64,
                              c_double_p, c_double_p], ctypes.c_int),
    'vb_objective_value_grad': ([ctypes.c_void_p, P(Family), P(Target), P(Objective),
                                 c_double_p, P(Noise), c_double_p, c_double_p], ctypes.c_int),
    'vb_run_create': ([ctypes.c_void_p, P(Family), P(Target), P(Objective), P(AdagradConfig),
                       ctypes.c_int64, c_double_p, P(ctypes.c_void_p)], ctypes.c_int),
    'vb_run_advance': ([ctypes.c_void_p, ctypes.c_int64, P(Noise)], ctypes.c_int),
    'vb_run_steps_done': ([ctypes.c_void_p, c_int64_p], ctypes.c_int),
    'vb_run_values_async': ([ctypes.c_void_p, ctypes.c_int64], ctypes.c_int),
    'vb_run_values_wait': ([ctypes.c_void_p, c_double_p, c_int64_p], ctypes.c_int),
    'vb_run_fr_retries': ([ctypes.c_void_p, c_int64_p], ctypes.c_int),
    'vb_peak_probe': ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                       c_double_p], ctypes.c_int),
    'vb_run_set_timing': ([ctypes.c_void_p, ctypes.c_int], ctypes.c_int),
    'vb_run_launch_times': ([ctypes.c_void_p, ctypes.c_int64, c_int64_p,
                             P(ctypes.c_float), c_int64_p], ctypes.c_int),
    'vb_block_floor': ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                        ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, c_double_p], ctypes.c_int),
    'vb_run_result': ([ctypes.c_void_p, c_double_p, c_double_p, c_double_p, c_double_p],
                      ctypes.c_int),
    'vb_run_destroy': ([ctypes.c_void_p], ctypes.c_int),
    'vb_adagrad_update': ([ctypes.c_void_p, ctypes.c_int64, c_double_p, c_double_p, c_double_p,
                           ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_double],
                          ctypes.c_int),
    'vb_adagrad_update_scaled': ([ctypes.c_void_p, ctypes.c_int64, c_double_p, c_double_p,
                                  c_double_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double,
                                  ctypes.c_double, c_double_p], ctypes.c_int),
    'vb_ia_update': ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, c_double_p, c_double_p,
                      c_double_p, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                      ctypes.c_double, c_double_p], ctypes.c_int),
    'vb_log_weights': ([ctypes.c_void_p, P(Family), P(Target), c_double_p, ctypes.c_int64,
                        P(Noise), c_double_p, c_double_p], ctypes.c_int),
    'vb_log_weights_rows': ([ctypes.c_void_p, P(Family), P(Target), c_double_p, ctypes.c_int64,
                             ctypes.c_int64, P(Noise), c_double_p], ctypes.c_int),
    'vb_divergence_bound': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_double,
                             ctypes.c_int32, ctypes.c_double, c_double_p], ctypes.c_int),
    'vb_divergence_bound_rows': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_int64,
                                  ctypes.c_int64, ctypes.c_double, ctypes.c_int32, ctypes.c_double,
                                  c_double_p], ctypes.c_int),
    'vb_centered_moments': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_int64,
                             c_double_p, c_double_p], ctypes.c_int),
    'vb_covariance': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_int64, c_double_p,
                       c_double_p], ctypes.c_int),
    'vb_weighted_covariance': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_int64,
                                c_double_p, ctypes.c_int32, c_double_p, c_double_p], ctypes.c_int),
    'vb_weighted_covariance_logw': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_int64,
                                     c_double_p, ctypes.c_int32, c_double_p, c_double_p],
                                    ctypes.c_int),
    'vb_psislw': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
                   c_double_p, c_double_p, c_int64_p, ctypes.c_int64, c_int64_p], ctypes.c_int),
    'vb_psislw_colmajor': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_int64,
                            ctypes.c_double, c_double_p, c_double_p, c_int64_p, ctypes.c_int64,
                            c_int64_p], ctypes.c_int),
    'vb_gpdfit': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, c_double_p, c_double_p,
                   c_double_p, c_double_p, c_int64_p], ctypes.c_int),
    'vb_gpinv': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                  c_double_p], ctypes.c_int),
    'vb_sumlogs': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, c_double_p], ctypes.c_int),
    'vb_sumlogs_rows': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_int64, c_double_p],
                        ctypes.c_int),
    'vb_rhat': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                 ctypes.c_int64, c_int64_p, c_int64_p, c_double_p, c_double_p], ctypes.c_int),
    'vb_rhat_stats': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                       ctypes.c_int64, c_int64_p, c_int64_p, c_double_p, c_double_p], ctypes.c_int),
    'vb_rhat_combine': ([ctypes.c_void_p, c_double_p, c_double_p, ctypes.c_int64, ctypes.c_int64,
                         ctypes.c_int64, c_int64_p, c_double_p, c_double_p], ctypes.c_int),
    'vb_iterate_average': ([ctypes.c_void_p, c_double_p, ctypes.c_int64, ctypes.c_int64,
                            ctypes.c_int64, ctypes.c_int64, c_double_p], ctypes.c_int),
}

_lib = None
_lock = threading.Lock()


def _load_torch_runtime():
    """PyTorch bundles its own HIP / HSA runtime (torch/lib/libamdhip64.so,
    libhsa-runtime64.so) with the same sonames as the ROCm runtime this library
    links (libamdhip64.so.7, libhsa-runtime64.so.1), so whichever loads first
    serves the whole process.  Device tensors are how callers hand this library
    HBM-resident data, and torch works only on its own runtime: load torch first
    so that this library binds to it (with the ROCm runtime loaded first, torch
    reports "No HIP GPUs are available")."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    """Load libviabel_amd.so (raises ImportError when it was not built)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(
                        'viabel_amd: HIP library %s not found; build it with '
                        '`python -c "import __graft_entry__ as g; g.build()"` or '
                        '`make -C viabel_amd/csrc`' % LIB_PATH)
                _load_torch_runtime()
                L = ctypes.CDLL(LIB_PATH)
                for name, (args, res) in _SIGNATURES.items():
                    fn = getattr(L, name)
                    fn.argtypes = args
                    fn.restype = res
                _lib = L
    return _lib


# exceptions raised inside a Python target callback, re-raised after the call
PENDING_CALLBACK_ERRORS = []


def check(rc):
    if PENDING_CALLBACK_ERRORS:
        err = PENDING_CALLBACK_ERRORS.pop()
        PENDING_CALLBACK_ERRORS.clear()
        raise err
    if rc == VB_OK:
        return
    msg = lib().vb_last_error().decode('utf-8', 'replace')
    if rc == VB_EINVAL:
        raise ValueError(msg)
    if rc == VB_ENOMEM:
        raise MemoryError(msg)
    if rc == VB_EUNSUPPORTED:
        raise NotImplementedError(msg)
    raise RuntimeError(msg)


class Context:
    """One vb_ctx (device + HIP stream)."""

    def __init__(self, device=0, stream=None):
        h = ctypes.c_void_p()
        check(lib().vb_ctx_create(int(device), stream, ctypes.byref(h)))
        self.handle = h
        self.device = device

    def synchronize(self):
        check(lib().vb_ctx_synchronize(self.handle))

    @property
    def stream(self):
        return lib().vb_ctx_stream(self.handle)

    def __del__(self):
        try:
            if self.handle and _lib is not None and not _SHUTDOWN[0]:
                _lib.vb_ctx_destroy(self.handle)
        except Exception:
            pass
        self.handle = None


# At interpreter exit every context is destroyed while the HIP runtime is alive
# (release_all, registered with atexit below); native objects still referenced
# then are left to process teardown: their finalizers run after the HIP / rocBLAS
# runtimes' own static destructors may have, so they skip the native release.
# The library also releases what live contexts hold from its own exit handler
# (vb_capi.hip release_live_contexts) for callers that never destroy them.
_SHUTDOWN = [False]


def shutting_down():
    return _SHUTDOWN[0]


def release_all():
    """Collect the objects no longer referenced (their native release runs first),
    then synchronize and destroy every context (its stream, the CU-masked pre-draw
    streams and the full-rank workspace) while the HIP runtime is still alive.
    The library is not used afterwards (later finalizers skip their native
    release).  Runs at interpreter exit; a program may call it earlier.  Round 5:
    with CU-masked streams still alive at exit, the process's teardown crashed
    under rocprofv3."""
    import gc
    gc.collect()
    for d, c in list(_ctx.items()):
        try:
            c.synchronize()
        except Exception:
            pass
        try:
            if c.handle and _lib is not None:
                _lib.vb_ctx_destroy(c.handle)
        finally:
            c.handle = None
            _ctx.pop(d, None)
    _SHUTDOWN[0] = True


atexit.register(release_all)


_ctx = {}
_default_device = [int(os.environ.get('VIABEL_AMD_DEVICE', '0'))]


def set_device(device):
    _default_device[0] = int(device)


def context(device=None):
    d = _default_device[0] if device is None else int(device)
    c = _ctx.get(d)
    if c is None:
        c = Context(d)
        _ctx[d] = c
    return c


def dptr(a):
    """double* of a C-contiguous float64 numpy array, or of a torch tensor's data."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if a.dtype != np.float64 or not a.flags.c_contiguous:
            raise TypeError('expected a C-contiguous float64 array')
        return a.ctypes.data_as(c_double_p)
    # torch tensor (device or host): pass the raw pointer
    return ctypes.cast(ctypes.c_void_p(a.data_ptr()), c_double_p)


def device_tensor(a):
    """`a` if it is a torch tensor in device memory (checked: contiguous
    float64), else None.  Device tensors go to the C ABI as device pointers,
    so chained calls (log weights -> bounds -> PSIS) stay in HBM."""
    if not getattr(a, 'is_cuda', False) or not hasattr(a, 'data_ptr'):
        return None
    import torch
    if a.dtype != torch.float64 or not a.is_contiguous():
        raise TypeError('expected a contiguous float64 device tensor')
    return a


def i64ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(c_int64_p)


def as_f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


NAN = float('nan')


def use_stream(device, stream_handle):
    """Make the default context of `device` launch on an existing HIP stream
    (e.g. torch.cuda.current_stream().cuda_stream) so torch events time it."""
    c = Context(device, ctypes.c_void_p(stream_handle))
    _ctx[int(device)] = c
    _default_device[0] = int(device)
    return c


def block_floor_us(D, N, chivi=False, host_layout=False, n_steps=2000, n_problems=1):
    """Device microseconds per step of the block kernel's step skeleton (same
    block shape, barriers, reductions and adagrad update; no draws, no target):
    the latency floor of configs 1, 2 and 5's fit (vb_block_floor)."""
    out = ctypes.c_double()
    check(lib().vb_block_floor(context().handle, int(D), int(N), 1 if chivi else 0,
                               1 if host_layout else 0, int(n_steps), int(n_problems),
                               ctypes.byref(out)))
    return out.value


PROBE_KINDS = {'hbm_copy': 0, 'hbm_read': 1, 'mfma_f64': 2, 'valu_fma_f64': 3, 'valu_mad_u64': 4}


def peak_probe(kind, n, reps=5):
    """Measured peak of one resource (vb_peak_probe): 'hbm_copy' / 'hbm_read' over n
    bytes (GB/s), 'mfma_f64' (TFLOP/s), 'valu_fma_f64' / 'valu_mad_u64' (G
    wave-instructions/s) over n iterations; best of `reps` launches."""
    out = ctypes.c_double()
    check(lib().vb_peak_probe(context().handle, PROBE_KINDS[kind], int(n), int(reps),
                              ctypes.byref(out)))
    return out.value
