"""ctypes wrapper of oracle/tpe_score.c -- TEST INFRASTRUCTURE / CPU BASELINE
ONLY (the C restatement of the reference's scoring, OpenMP over candidates).
Built by `make -C oracle` (hyperopt_amd._build.build_oracle, __graft_entry__.build).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, 'libtpe_score.so')
_lib = None

_P = ctypes.c_void_p
_D = ctypes.c_double


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise OSError('C oracle not built: run `make -C oracle`')
        lib = ctypes.CDLL(LIB)
        lib.ora_mixture_lpdf.argtypes = [ctypes.c_int, _P, ctypes.c_int64, _P, _P, _P, ctypes.c_int,
                                         ctypes.c_int, _D, _D, _D, _P]
        lib.ora_mixture_lpdf.restype = None
        lib.ora_categorical_lpdf.argtypes = [_P, ctypes.c_int64, _P, _P]
        lib.ora_categorical_lpdf.restype = None
        lib.ora_broadcast_best.argtypes = [_P, _P, ctypes.c_int64]
        lib.ora_broadcast_best.restype = ctypes.c_int64
        lib.ora_threads.restype = ctypes.c_int
        _lib = lib
    return _lib


def available():
    return os.path.exists(LIB)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _flags(low, high, q):
    return (1 if low is not None else 0) | (2 if high is not None else 0) | (4 if q is not None else 0)


def mixture_lpdf(log_space, samples, weights, mus, sigmas, low=None, high=None, q=None):
    x = np.ascontiguousarray(samples, dtype=np.float64).ravel()
    w, m, s = (np.ascontiguousarray(a, dtype=np.float64) for a in (weights, mus, sigmas))
    out = np.empty_like(x)
    load().ora_mixture_lpdf(int(log_space), _p(x), len(x), _p(w), _p(m), _p(s), len(w),
                            _flags(low, high, q), float(low or 0.0), float(high or 0.0),
                            float(q or 0.0), _p(out))
    return out


def gmm1_lpdf(samples, weights, mus, sigmas, low=None, high=None, q=None):
    return mixture_lpdf(0, samples, weights, mus, sigmas, low, high, q)


def lgmm1_lpdf(samples, weights, mus, sigmas, low=None, high=None, q=None):
    return mixture_lpdf(1, samples, weights, mus, sigmas, low, high, q)


def categorical_lpdf(sample, p):
    s = np.ascontiguousarray(sample, dtype=np.int64).ravel()
    p = np.ascontiguousarray(p, dtype=np.float64)
    out = np.empty(len(s))
    load().ora_categorical_lpdf(_p(s), len(s), _p(p), _p(out))
    return out


def broadcast_best_index(below, above):
    b = np.ascontiguousarray(below, dtype=np.float64)
    a = np.ascontiguousarray(above, dtype=np.float64)
    return int(load().ora_broadcast_best(_p(b), _p(a), len(b)))


def threads():
    return int(load().ora_threads())
