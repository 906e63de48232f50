"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/vbrng.c, the C restatement of the device Philox noise
(counter = (column pair, sample, step, stream | purpose << 24), key = seed).
Build with ``make -C oracle`` (``__graft_entry__.build()`` does it).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, 'liboracle_rng.so')
        if not os.path.exists(path):
            raise ImportError('oracle RNG library missing: run `make -C oracle`')
        lib = ctypes.CDLL(path)
        lib.vbo_philox.argtypes = [ctypes.POINTER(ctypes.c_uint32)] * 3
        lib.vbo_fill.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                                 ctypes.POINTER(ctypes.c_double)]
        lib.vbo_fr_scale.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_int64, ctypes.c_double,
                                     ctypes.POINTER(ctypes.c_double)]
        _LIB = lib
    return _LIB


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    _lib().vbo_philox(c, k, o)
    return list(o)


def noise(seed, stream, step, n, dim, family='gauss', df=0.0):
    """Standardized draws eps[n, dim] of one step: N(0,1) ('gauss'), t(df) as
    N / sqrt(Gamma) ('t', the estimators' draws) or by Bailey's trigonometric
    method ('t_bailey', the log-weight draws of the t family)."""
    out = np.empty((n, dim))
    _lib().vbo_fill(seed, stream & 0xFFFFFF, step & 0xFFFFFFFF, n, dim,
                    {'gauss': 0, 't': 1, 't_bailey': 2}[family], float(df),
                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return out


def fr_noise(seed, stream, step, n, dim, df):
    """Full-rank t draws of one step: (s [n], z [n, dim]) (vb_fr.hip fr_noise_kernel)."""
    s = np.empty(n)
    _lib().vbo_fr_scale(seed, stream & 0xFFFFFF, step & 0xFFFFFFFF, n, float(df),
                        s.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return s, noise(seed, stream, step, n, dim, 'gauss')
