"""Exact early exit of quantized and categorical tile rounds (TPE_OPT_EARLY,
tpe_engine.hip k_qfused_tiles / k_cat_tiles): a label's candidates are
drawn in index order and the round stops once a candidate holds the best
score any draw can have.  The first index holding that score is the
np.argmax winner (reference broadcast_best, hyperopt/tpe.py:769-778: the
first maximum), so every result field must equal the full scan's bit for
bit -- on the config-3 posterior at 2^20 and 2^24 candidates, and on
posteriors whose best value is rare (the second, full-grid phase has to
find it), and with per-candidate quantized evaluation (dedup off)."""
import numpy as np
import pytest

from hyperopt_amd import _lib as L
from hyperopt_amd.engine import DESC_DTYPE

pytestmark = pytest.mark.gpu


def _bytes(res):
    return np.ascontiguousarray(res).view(np.uint8).tobytes()


def _rounds(eng, C, seeds, early):
    eng.set_option('early', int(early))
    out, drawn = [], []
    for s in seeds:
        out.append(eng.suggest(seed=s, n_candidates=C, round=s % 7))
        drawn.append(eng.last_drawn())
    eng.set_option('early', 1)
    return out, drawn


@pytest.mark.parametrize('log2c', [20, 24])
def test_early_exit_equals_full_scan_config3(log2c):
    from hyperopt_amd import posterior as P
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(32, 10000, seed=0)
    eng = Engine(0, 'f64')
    eng.set_posterior(*P.pack(hist.posteriors()))
    C = 1 << log2c
    seeds = [11, 12] if log2c == 24 else [11, 12, 13, 14]
    fast, d_fast = _rounds(eng, C, seeds, True)
    full, d_full = _rounds(eng, C, seeds, False)
    eng.close()
    for a, b in zip(fast, full):
        assert _bytes(a) == _bytes(b)
    n_q = sum(1 for _, k, _ in hist.labels if k == 'quniform')
    n_c = sum(1 for _, k, _ in hist.labels if k == 'randint')
    first_phase = 64 * 8 * 256      # kEarlyTiles tiles of R x 256 candidates per label
    for (qf, cf), (qs, cs) in zip(d_fast, d_full):
        assert qs == n_q * C and cs == n_c * C          # the full scan draws every candidate
        # the best drawable value turns up within the first phase
        assert qf <= n_q * first_phase and cf <= n_c * first_phase


def _posterior(kind):
    """One label whose best-scoring value is rare under l(x):
    categorical: p_below = [1 - 1e-6, 1e-6], p_above = [1 - 1e-13, 1e-13]
    (category 1 first drawn around index 1e6, mostly past the first phase);
    quantized: quniform-like GMM1 on [0, 50) with q = 1, the below mixture
    piled on 10, a thin below component at 40 that the above mixture avoids."""
    d = np.zeros(1, dtype=DESC_DTYPE)
    if kind == 'categorical':
        pb = np.array([1 - 1e-6, 1e-6])
        pa = np.array([1 - 1e-13, 1e-13])
        d['kind'] = L.TPE_CATEGORICAL
        d['below_off'], d['n_below'] = 0, 2
        d['above_off'], d['n_above'] = 2, 2
        w = np.concatenate([pb, pa])
        return d, w, np.zeros_like(w), np.zeros_like(w)
    d['kind'] = L.TPE_GMM1
    d['flags'] = L.TPE_HAS_LOW | L.TPE_HAS_HIGH | L.TPE_HAS_Q
    d['low'], d['high'], d['q'] = 0.0, 50.0, 1.0
    wb, mb, sb = [1 - 2e-6, 2e-6], [10.0, 40.0], [3.0, 0.3]
    wa, ma, sa = [0.5, 0.5], [10.0, 25.0], [3.0, 3.0]
    d['below_off'], d['n_below'] = 0, 2
    d['above_off'], d['n_above'] = 2, 2
    return d, np.array(wb + wa), np.array(mb + ma), np.array(sb + sa)


@pytest.mark.parametrize('kind', ['categorical', 'quantized'])
@pytest.mark.parametrize('dedup', [1, 0])
def test_early_exit_rare_best_value(kind, dedup):
    from hyperopt_amd.engine import Engine
    if kind == 'categorical' and dedup == 0:
        pytest.skip('dedup only concerns quantized labels')
    eng = Engine(0, 'f64')
    eng.set_option('dedup', dedup)
    eng.set_posterior(*_posterior(kind))
    C = 1 << 23
    seeds = [3, 4, 5]
    fast, d_fast = _rounds(eng, C, seeds, True)
    full, d_full = _rounds(eng, C, seeds, False)
    eng.close()
    for a, b in zip(fast, full):
        assert _bytes(a) == _bytes(b)
    if kind == 'categorical':
        assert max(int(r['index'][0]) for r in fast) > 64 * 8 * 256   # a find in the second phase
        assert all(int(r['value'][0]) == 1 for r in fast)    # the rare best category wins
        assert all(f[1] < s[1] for f, s in zip(d_fast, d_full))
    elif dedup:
        assert all(f[0] < s[0] for f, s in zip(d_fast, d_full))


def test_early_exit_draw_counts_are_deterministic():
    """The drawn counts (and so the categorical evals on the bench line) are
    those of a scan in index order -- every tile starting at or before the
    first index holding the best drawable score -- whatever order the
    workgroups ran in: equal with the side families beside the dense draw on
    the second stream and without, and over repeats.
    A categorical cell's winner IS that first index, so its count is known
    exactly: min(C, (index // 2048 + 1) * 2048) (tiles of 8 x 256)."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(32, 10000, seed=0)
    eng = Engine(0, 'f64')
    eng.set_posterior(*P.pack(hist.posteriors()))
    C = 1 << 22
    cat = [i for i, (_, k, _) in enumerate(hist.labels) if k == 'randint']
    seen = {}
    for aux in (0, 1, 1, 0):
        eng.set_option('aux_families', aux)
        for s in (21, 22):
            res = eng.suggest(seed=s, n_candidates=C, round=s)
            d = eng.last_drawn()
            seen.setdefault(s, []).append(d)
            want = sum(min(C, (int(res[li]['index']) // 2048 + 1) * 2048) for li in cat)
            assert d[1] == want, (s, aux, d, want)
    eng.close()
    for s, ds in seen.items():
        assert len(set(ds)) == 1, (s, ds)
