"""Shared helpers: turn golden label cases (reference-built posteriors) into
C-ABI label descriptors, and tolerance checks with the bars stated in
DESIGN.md."""
import numpy as np

from hyperopt_amd import _lib as L
from hyperopt_amd.engine import DESC_DTYPE


def desc_from_case(meta, rec, off=0):
    """One tpe_label_desc + flat component arrays from a golden case."""
    kw = meta['lpdf_kwargs']
    if meta['sampler'] == 'categorical':
        pb, pa = rec['p_below'], rec['p_above']
        d = np.zeros(1, dtype=DESC_DTYPE)
        d['kind'] = L.TPE_CATEGORICAL
        d['below_off'], d['n_below'] = off, len(pb)
        d['above_off'], d['n_above'] = off + len(pb), len(pa)
        w = np.concatenate([pb, pa])
        return d, w, np.zeros_like(w), np.zeros_like(w)
    low, high, q = kw.get('low'), kw.get('high'), kw.get('q')
    d = np.zeros(1, dtype=DESC_DTYPE)
    d['kind'] = L.TPE_GMM1 if meta['sampler'] == 'GMM1' else L.TPE_LGMM1
    f = 0
    if low is not None:
        f |= L.TPE_HAS_LOW
        d['low'] = low
    if high is not None:
        f |= L.TPE_HAS_HIGH
        d['high'] = high
    if q is not None:
        f |= L.TPE_HAS_Q
        d['q'] = q
    d['flags'] = f
    nb, na = len(rec['w_b']), len(rec['w_a'])
    d['below_off'], d['n_below'] = off, nb
    d['above_off'], d['n_above'] = off + nb, na
    w = np.concatenate([rec['w_b'], rec['w_a']])
    m = np.concatenate([rec['mu_b'], rec['mu_a']])
    s = np.concatenate([rec['sigma_b'], rec['sigma_a']])
    return d, w, m, s


def stack_cases(pairs):
    """Concatenate several (meta, rec) cases into one multi-label posterior."""
    ds, ws, ms, ss = [], [], [], []
    off = 0
    for meta, rec in pairs:
        d, w, m, s = desc_from_case(meta, rec, off)
        ds.append(d)
        ws.append(w)
        ms.append(m)
        ss.append(s)
        off += len(w)
    return np.concatenate(ds), np.concatenate(ws), np.concatenate(ms), np.concatenate(ss)


def is_quantized(meta):
    return meta['lpdf_kwargs'].get('q') is not None


def assert_lpdf_close(got, ref, quantized=False, rtol=1e-9, atol=1e-9, w_sum=1.0):
    """fp64 bar: rtol 1e-9 (+atol 1e-9 for values near 0).  Quantized lpdfs
    are log(sum of differences of CDFs) computed in linear space by the
    reference, whose own rounding error is ~K ulp(1) in the probability; for
    those the bar is rtol 1e-9 on the log OR |exp(got) - exp(ref)| <= 1e-13,
    i.e. the two probabilities agree to the reference's own accuracy."""
    got = np.asarray(got, float)
    ref = np.asarray(ref, float)
    assert got.shape == ref.shape
    both_nan = np.isnan(got) & np.isnan(ref)
    same_inf = np.isinf(got) & (got == ref)
    with np.errstate(invalid='ignore', over='ignore'):
        ok = both_nan | same_inf | (np.abs(got - ref) <= atol + rtol * np.abs(ref))
        abs_only = np.zeros_like(ok)
        if quantized:
            abs_only = ~ok & (np.abs(np.exp(got) - np.exp(ref)) <= 1e-13 * w_sum)
            ok |= abs_only
    if not ok.all():
        bad = np.where(~ok)[0][:8]
        raise AssertionError('lpdf mismatch at %s: got %s ref %s' % (
            bad.tolist(), got[bad].tolist(), ref[bad].tolist()))
    return abs_only
