"""ctypes binding of the C ABI in include/hyperopt_tpe.h.

The shared library `libhyperopt_tpe.so` is built in-tree (see
`hyperopt_amd/_build.py`).  There is no fallback: if it is missing or a
symbol is absent, importing the engine raises.

PyTorch, when importable, is imported BEFORE the library is loaded so that the
process holds exactly one HIP runtime (torch's bundled libamdhip64.so.7 has
the same SONAME, so the dynamic loader binds our library to it).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libhyperopt_tpe.so')
HEADER = os.path.join(os.path.dirname(HERE), 'include', 'hyperopt_tpe.h')

ABI_VERSION = 4

TPE_OK = 0
TPE_ERR_VALUE = -1
TPE_ERR_TYPE = -2
TPE_ERR_ARG = -3
TPE_STATUS_VALUE_ONLY = 1   # tpe_label_result.status of a value-only cell
TPE_ERR_HIP = -4
TPE_ERR_SAMPLE = -5

TPE_F64 = 0
TPE_F32 = 1

TPE_GMM1 = 0
TPE_LGMM1 = 1
TPE_CATEGORICAL = 2

TPE_HAS_LOW = 1
TPE_HAS_HIGH = 2
TPE_HAS_Q = 4
TPE_HAS_STREAM = 8

TPE_OPT_SCREEN = 1
TPE_OPT_SPLITK = 2
TPE_OPT_DEDUP = 3
TPE_OPT_CHUNKS = 4
TPE_OPT_WHOLE_N = 5
TPE_OPT_WHOLE_ROUNDS = 6
TPE_OPT_TIMING = 7
TPE_OPT_WINDOW = 8
TPE_OPT_WIN_T = 9
TPE_OPT_WIN_GROUPS = 10
TPE_OPT_EXPAND = 11
TPE_OPT_HOT = 12
TPE_OPT_EARLY = 13
TPE_OPT_HOT_DIV = 14
TPE_OPT_ZERO_WIN = 15
TPE_OPT_VALUE_ONLY = 16
TPE_OPT_RESCORE_CAP = 17
TPE_OPT_MODE_MASK = 18
TPE_OPT_AUX_FAMILIES = 19
TPE_OPT_BX_SPLIT = 21
TPE_OPT_BX_T = 22
TPE_OPT_PK_SLICED = 23
TPE_OPT_DEFER_REPORT = 24
TPE_OPT_LABEL_SHARDS = 25

TPE_OBS_IDENTITY = 0
TPE_OBS_LOG = 1
TPE_OBS_LOG_FLOOR = 2


class LabelDesc(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32), ('flags', ctypes.c_int32),
                ('low', ctypes.c_double), ('high', ctypes.c_double), ('q', ctypes.c_double),
                ('below_off', ctypes.c_int64), ('above_off', ctypes.c_int64),
                ('n_below', ctypes.c_int32), ('n_above', ctypes.c_int32)]


class LabelSpec(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32), ('flags', ctypes.c_int32),
                ('low', ctypes.c_double), ('high', ctypes.c_double), ('q', ctypes.c_double),
                ('prior_mu', ctypes.c_double), ('prior_sigma', ctypes.c_double),
                ('upper', ctypes.c_int32), ('randint', ctypes.c_int32), ('p_off', ctypes.c_int64),
                ('stream', ctypes.c_int32), ('reserved', ctypes.c_int32)]


class LabelResult(ctypes.Structure):
    _fields_ = [('value', ctypes.c_double), ('score', ctypes.c_double),
                ('lpdf_below', ctypes.c_double), ('lpdf_above', ctypes.c_double),
                ('index', ctypes.c_int64), ('label', ctypes.c_int32), ('status', ctypes.c_int32)]


assert ctypes.sizeof(LabelDesc) == 56
assert ctypes.sizeof(LabelResult) == 48
assert ctypes.sizeof(LabelSpec) == 72

_P = ctypes.c_void_p
_I32, _I64, _U32, _U64, _D = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                              ctypes.c_uint64, ctypes.c_double)
_PD = ctypes.POINTER(ctypes.c_double)

# name -> (restype, argtypes); every function declared in include/hyperopt_tpe.h
SIGNATURES = {
    'tpe_abi_version': (ctypes.c_int, []),
    'tpe_source_hash': (ctypes.c_char_p, []),
    'tpe_ctx_create': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P)]),
    'tpe_ctx_create_multi': (ctypes.c_int, [_P, _I32, ctypes.c_int, ctypes.POINTER(_P)]),
    'tpe_ctx_devices': (ctypes.c_int32, [_P, _P, _I32]),
    'tpe_label_device': (ctypes.c_int32, [_P, _I32]),
    'tpe_ctx_destroy': (None, [_P]),
    'tpe_last_error': (ctypes.c_char_p, [_P]),
    'tpe_gmm1_lpdf': (ctypes.c_int, [_P, _P, _I64, _P, _P, _P, _I32, _I32, _D, _D, _D, _P]),
    'tpe_lgmm1_lpdf': (ctypes.c_int, [_P, _P, _I64, _P, _P, _P, _I32, _I32, _D, _D, _D, _P]),
    'tpe_categorical_lpdf': (ctypes.c_int, [_P, _P, _I64, _P, _I32, _P]),
    'tpe_broadcast_best': (ctypes.c_int, [_P, _P, _P, _I64, _P]),
    'tpe_gmm1_sample': (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _D, _D, _D, _U64, _U32, _U32,
                                       _I64, _I64, _P]),
    'tpe_lgmm1_sample': (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _D, _D, _D, _U64, _U32, _U32,
                                        _I64, _I64, _P]),
    'tpe_categorical_sample': (ctypes.c_int, [_P, _P, _I32, _U64, _U32, _U32, _I64, _I64, _P]),
    'tpe_set_posterior': (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _I64]),
    'tpe_suggest': (ctypes.c_int, [_P, _U64, _U32, _I64, _I64, _P]),
    'tpe_suggest_batch': (ctypes.c_int, [_P, _U64, _P, _I32, _I64, _I64, _P]),
    'tpe_score': (ctypes.c_int, [_P, _I32, _P, _I64, _P, _P, _P]),
    'tpe_merge_results': (ctypes.c_int, [_P, _I32, _I32, _P]),
    'tpe_suggest_batch_device': (ctypes.c_int, [_P, _U64, _P, _I32, _I64, _I64, _P, _P]),
    'tpe_merge_results_device': (ctypes.c_int, [_P, _P, _I32, _I32, _P]),
    'tpe_last_timing': (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_float),
                                       ctypes.POINTER(ctypes.c_float)]),
    'tpe_last_evals': (ctypes.c_int64, [_P]),
    'tpe_last_mode_stats': (ctypes.c_int, [_P, _P, _P]),
    'tpe_build_posterior': (ctypes.c_int, [_P, _P, _I32, _P, _I64, _P, _I64, _P, _P, _P, _D, _D,
                                           _I32, _P]),
    'tpe_get_mixture': (ctypes.c_int, [_P, _I32, _I32, _P, _P, _P, _I32, _P]),
    'tpe_resident_labels': (ctypes.c_int32, [_P]),
    'tpe_history_reset': (ctypes.c_int, [_P, _P, _I32, _P, _I64]),
    'tpe_history_append': (ctypes.c_int, [_P, _P, _P, _P]),
    'tpe_build_posterior_resident': (ctypes.c_int, [_P, _P, _I64, _I64, _D, _D, _I32, _P]),
    'tpe_build_posterior_resident_ordered': (ctypes.c_int, [_P, _P, _I64, _I64, _D, _D, _I32, _P, _P, _P,
                                                            _P, _P]),
    'tpe_rebuild_labels': (ctypes.c_int, [_P, _P, _I64, _I64, _D, _D, _I32, _P, _P, _P, _I32, _P, _P]),
    'tpe_last_build_ms': (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_float)]),
    'tpe_build_report': (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int32), ctypes.c_void_p]),
    'tpe_last_screen': (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(ctypes.c_float)]),
    'tpe_set_option': (ctypes.c_int, [_P, _I32, _I64]),
    'tpe_last_screen_terms': (ctypes.c_int, [_P, _P]),
    'tpe_last_rescore_terms': (ctypes.c_int, [_P, _P]),
    'tpe_last_drawn': (ctypes.c_int, [_P, _P, _P]),
    'tpe_device_bytes': (ctypes.c_int64, []),
    'tpe_prepare': (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int32]),
    'tpe_arm_prepare': (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int32]),
    'tpe_last_screen_mode': (ctypes.c_int32, [_P]),
    'tpe_last_hot': (ctypes.c_int, [_P, _P, _P]),
    'tpe_last_prepare': (ctypes.c_int, [_P, _P]),
    'tpe_hot_probe': (ctypes.c_int, [_P, ctypes.c_int32, _P, ctypes.c_int64, _P, _P, _P]),
    'tpe_screen_probe': (ctypes.c_int, [_P, _I32, _P, _I64, _P, _P]),
    'tpe_export_posterior': (ctypes.c_int, [_P, _P, _I64, _P]),
    'tpe_import_posterior': (ctypes.c_int, [_P, _P, _I64, _P, _I32, _P, _P]),
}

_lib = None


def load():
    """Load and bind the library once.  Raises OSError / AttributeError if the
    native build is missing or stale -- there is no Python fallback."""
    global _lib
    if _lib is not None:
        return _lib
    try:  # one HIP runtime per process: let torch bring its libamdhip64 first
        import torch  # noqa: F401
    except Exception:
        pass
    variant = os.environ.get('HYPEROPT_AMD_VARIANT')
    path = LIB_PATH
    if variant:   # timing experiments only (tools/build_variant.py): explicit opt-in
        import sys
        path = os.path.abspath(variant)
        sys.stderr.write('hyperopt_amd: loading the experiment variant %s, not the product '
                         'library\n' % path)
    if not os.path.exists(path):
        raise OSError('hyperopt_amd native library not built: %s (run '
                      '`python -m hyperopt_amd._build` or __graft_entry__.build())' % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if variant and not hasattr(lib, name):   # (a variant of an older commit: fewer entry points)
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.tpe_abi_version() != ABI_VERSION:
        raise OSError('ABI version mismatch')
    if variant:
        if not lib.tpe_source_hash().decode().startswith('v:'):
            raise OSError('%s is not a variant build (tools/build_variant.py)' % path)
    else:
        check_stamp(lib)
    _lib = lib
    return lib


def check_stamp(lib):
    """Refuse a library that was not built from the sources in this tree
    (its embedded hash, hyperopt_amd/_build.py, must match theirs)."""
    from . import _build
    want = _build.source_hash()
    got = lib.tpe_source_hash().decode()
    if got != want:
        raise OSError('hyperopt_amd native library %s is stale: built from sources %s, tree '
                      'has %s (run `python -m hyperopt_amd._build`)' % (LIB_PATH, got, want))


def header_functions(path=HEADER):
    """Names of the functions declared in the C header (for export checks)."""
    import re
    txt = open(path).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(tpe_[a-z0-9_]+)\s*\(', txt)))
