"""C-ABI checks that need no GPU: the in-tree library loads, exports every
function include/hyperopt_tpe.h declares, struct layouts match, and the
host-only merge follows broadcast_best's order (tpe.py:769-778)."""
import ctypes
import os

import numpy as np
import pytest

from hyperopt_amd import _lib as L


def test_library_built_and_exports_header():
    assert os.path.exists(L.LIB_PATH), 'run hyperopt_amd._build first'
    lib = L.load()
    declared = L.header_functions()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
        assert name in L.SIGNATURES, 'binding missing for ' + name
    assert lib.tpe_abi_version() == L.ABI_VERSION == 4


def test_struct_layouts():
    assert ctypes.sizeof(L.LabelDesc) == 56
    assert ctypes.sizeof(L.LabelResult) == 48
    assert ctypes.sizeof(L.LabelSpec) == 72
    assert L.LabelSpec.stream.offset == 64
    assert L.LabelDesc.n_below.offset == 48
    assert L.LabelResult.index.offset == 32


def _res(score, index, value=0.0):
    from hyperopt_amd.engine import RESULT_DTYPE
    r = np.zeros(1, dtype=RESULT_DTYPE)
    r['score'], r['index'], r['value'] = score, index, value
    return r


def test_merge_results_order():
    from hyperopt_amd.engine import merge_results
    cases = [
        ([1.0, 3.0, 2.0], [0, 1, 2], 1),             # larger score wins
        ([3.0, 3.0], [7, 2], 1),                       # tie -> lowest global index
        ([np.inf, np.nan, 5.0], [0, 9, 1], 1),         # NaN beats +inf
        ([np.nan, np.nan], [4, 3], 1),                 # first NaN (lowest index)
        ([-0.0, 0.0], [2, 1], 1),                      # -0 == +0
        ([-np.inf, -np.inf], [5, 6], 0),
    ]
    for scores, idx, want in cases:
        parts = np.stack([_res(s, i) for s, i in zip(scores, idx)])
        out = merge_results(parts)
        assert int(out['index'][0]) == idx[want], (scores, idx)
    # shards with no candidates (index -1) are ignored
    parts = np.stack([_res(np.nan, -1), _res(1.0, 3)])
    assert int(merge_results(parts)['index'][0]) == 3


def test_ctx_create_reports_missing_device():
    lib = L.load()
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip('GPU present')
    except ImportError:
        pass
    h = ctypes.c_void_p()
    rc = lib.tpe_ctx_create(0, L.TPE_F64, ctypes.byref(h))
    assert rc == L.TPE_ERR_HIP
    assert b'device' in lib.tpe_last_error(None)
    from hyperopt_amd.engine import Engine, EngineError
    with pytest.raises(EngineError):
        Engine(0)


def test_bad_precision_rejected():
    lib = L.load()
    h = ctypes.c_void_p()
    assert lib.tpe_ctx_create(0, 7, ctypes.byref(h)) == L.TPE_ERR_ARG


def test_merge_results_refuses_value_only():
    """A TPE_STATUS_VALUE_ONLY record (index and value, no score) cannot be
    ranked by broadcast_best's order: the host merge refuses it; records
    without a winner (index -1) are skipped as before."""
    from hyperopt_amd.engine import EngineError, merge_results
    a, b = _res(1.0, 3), _res(float('nan'), 7)
    b['status'] = L.TPE_STATUS_VALUE_ONLY
    with pytest.raises(EngineError):
        merge_results(np.stack([a, b]))
    b['index'] = -1
    assert merge_results(np.stack([a, b]))['index'][0] == 3
