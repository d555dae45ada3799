"""Argmax agreement of the HIP round with the reference's numpy arithmetic
at full candidate counts -- TEST INFRASTRUCTURE ONLY (tests/ and the oracle
legs of bench.py; the product never imports it).

The oracle cannot score 2^24 candidates x 10^4 components, and at that many
candidates a label's best scores are near-ties (top-2 gaps ~1e-12), where
the HIP fp64 arithmetic (table exp, 256-component summation slices) and
numpy's (np.exp, pairwise `.sum(axis=1)`, tpe.py:259-262) round differently.
So per (round, label) cell:

* dense labels (GMM1 / LGMM1 without q): every candidate of the round is
  re-drawn through the engine's sampler entry points (same Philox stream) and
  scored by the HIP fp64 lpdfs (tpe_score); the `top` best are scored by the
  numpy restatement of GMM1_lpdf / LGMM1_lpdf (oracle/tpe_oracle.py,
  tpe.py:110-172, 265-307) and numpy's broadcast_best argmax among them
  (tpe.py:769-778: first index of the largest below - above) must be the
  round's winner.  The set is wide enough when the HIP score of its last
  member is further below the best than any HIP - numpy difference seen in
  it (`span` vs `max_abs_diff`).  A cell whose numpy argmax beats the HIP
  winner, in numpy's arithmetic, by no more than the two arithmetics' own
  largest difference in the set is an arithmetic tie (`arith_tie`): the two
  scores are equal to a few ulp and the order is rounding in either
  arithmetic -- reported separately, never counted as agreement;
* quantized and categorical labels: a candidate's score is a function of its
  value, so every distinct value of the round's candidates is scored by the
  oracle and numpy's winner is the first candidate holding the best one.
"""
import numpy as np

from . import tpe_oracle as O


def posteriors_of(eng, labels):
    """The engine's resident mixtures as oracle LabelPosterior objects
    (labels: the (name, kind, args) list the posterior was built from)."""
    from hyperopt_amd import posterior as P
    posts = []
    for li, (name, kind, args) in enumerate(labels):
        b, a = eng.get_mixture(li, 0), eng.get_mixture(li, 1)
        if kind in ('randint', 'categorical'):
            posts.append(P.LabelPosterior(name, 'categorical', b[0], a[0], upper=len(b[0])))
        else:
            spec, _, _ = P.label_spec(kind, args)
            posts.append(P.LabelPosterior(name, 'GMM1' if spec['kind'] == 0 else 'LGMM1', b, a,
                                          low=args.get('low'), high=args.get('high'),
                                          q=args.get('q')))
    return posts


def _draw(eng, p, stream, seed, rnd, n):
    if p.family == 'categorical':
        return eng.categorical(p.below, seed=seed, size=(n,), stream=stream, round=rnd).astype(float)
    samp = eng.GMM1 if p.family == 'GMM1' else eng.LGMM1
    return samp(*p.below, low=p.low, high=p.high, q=p.q, seed=seed, size=(n,), stream=stream,
                round=rnd)


def _np_scores(p, x):
    if p.family == 'categorical':
        xi = x.astype(int)
        lb, la = O.categorical_lpdf(xi, p.below), O.categorical_lpdf(xi, p.above)
    else:
        f = O.gmm1_lpdf if p.family == 'GMM1' else O.lgmm1_lpdf
        lb = f(x, *p.below, low=p.low, high=p.high, q=p.q)
        la = f(x, *p.above, low=p.low, high=p.high, q=p.q)
    with np.errstate(invalid='ignore'):
        return lb - la


def _dense_cell(eng, li, p, stream, seed, rnd, C, r, top):
    x = _draw(eng, p, stream, seed, rnd, C)
    lb, la, _ = eng.score(li, x)
    s = lb - la
    del lb, la
    k = min(top, C)
    cand = np.sort(np.argpartition(-s, k - 1)[:k])          # index order: first max wins
    s_hip = s[cand]
    s_np = _np_scores(p, x[cand])
    j_np = int(np.argmax(s_np))
    order = np.sort(s_np)[::-1]
    w = int(r['index'])
    wj = np.searchsorted(cand, w)
    in_set = wj < len(cand) and cand[wj] == w
    diff = np.abs(s_hip - s_np)
    strict = int(cand[j_np]) == w
    # numpy's margin of its own argmax over the HIP winner, in numpy's
    # arithmetic: within the two arithmetics' measured disagreement (the
    # largest |HIP - numpy| of the set) the order of the two is rounding in
    # either, and the cell is an arithmetic tie, reported as such
    margin = float(s_np[j_np] - s_np[wj]) if in_set else None
    tie = bool(not strict and in_set and margin <= 2.0 * float(np.max(diff)))
    return {
        'label': int(li), 'kind': 'dense', 'agree': bool(strict), 'arith_tie': tie,
        'numpy_margin_over_winner': margin,
        'winner': w, 'numpy_winner': int(cand[j_np]),
        'hip_full_argmax': int(cand[int(np.argmax(s_hip))]),
        'numpy_top2_gap': float(order[0] - order[1]) if len(order) > 1 else None,
        'hip_minus_numpy_at_winner': float(s_hip[wj] - s_np[wj]) if in_set else None,
        'max_abs_diff': float(np.max(diff)),
        'span': float(np.max(s_hip) - np.min(s_hip)),
        'winner_value_equal': bool(x[w] == r['value']),
    }


def _valued_cell(eng, li, p, stream, seed, rnd, C, r):
    import pandas as pd
    x = _draw(eng, p, stream, seed, rnd, C)
    vals = pd.unique(x)                                      # order of first appearance
    s_np = _np_scores(p, np.asarray(vals, dtype=float))
    best = np.nanmax(s_np) if not np.all(np.isnan(s_np)) else np.nan
    # broadcast_best: NaN first, else the first index of the largest score
    if np.any(np.isnan(s_np)):
        pick = int(np.argmax(np.isnan(s_np)))
    else:
        pick = int(np.argmax(s_np))      # vals are in first-appearance order
    v = vals[pick]
    w_np = int(np.argmax(x == v))
    ties = np.sort(s_np[s_np == s_np])[::-1]
    return {
        'label': int(li), 'kind': p.family if p.family == 'categorical' else 'quantized',
        'agree': bool(w_np == int(r['index'])), 'winner': int(r['index']), 'numpy_winner': w_np,
        'distinct_values': int(len(vals)),
        'numpy_top2_gap': float(ties[0] - ties[1]) if len(ties) > 1 else None,
        'winner_value_equal': bool(x[int(r['index'])] == r['value']),
        'best_score': float(best),
    }


def round_agreement(eng, posts, res, seed, rnd, C, top=64, streams=None, dense_only=False):
    """Per-cell agreement records of one round `res` (eng.suggest(seed, C,
    round=rnd) on the posterior `posts` describes)."""
    cells = []
    for li, p in enumerate(posts):
        st = li if streams is None else int(streams[li])
        dense = p.family != 'categorical' and p.q is None
        if dense:
            cells.append(_dense_cell(eng, li, p, st, seed, rnd, C, res[li], top))
        elif not dense_only:
            cells.append(_valued_cell(eng, li, p, st, seed, rnd, C, res[li]))
    return cells


def summary(cells):
    dense = [c for c in cells if c['kind'] == 'dense']
    gaps = [c['numpy_top2_gap'] for c in dense if c['numpy_top2_gap'] is not None]
    ties = [c for c in dense if c.get('arith_tie')]
    return {
        'cells': len(cells), 'agree': sum(c['agree'] for c in cells),
        'rate': sum(c['agree'] for c in cells) / max(len(cells), 1),
        'dense_cells': len(dense), 'dense_agree': sum(c['agree'] for c in dense),
        'min_numpy_top2_gap_dense': min(gaps) if gaps else None,
        'median_numpy_top2_gap_dense': float(np.median(gaps)) if gaps else None,
        'max_abs_hip_minus_numpy_dense': max((c['max_abs_diff'] for c in dense), default=None),
        'min_span_dense': min((c['span'] for c in dense), default=None),
        # disagreements within the arithmetics' own difference (both scores
        # within a few ulp): neither argmax is the "right" one
        'arith_ties': len(ties),
        'arith_tie_margins': [c['numpy_margin_over_winner'] for c in ties],
        'agree_or_arith_tie': sum(bool(c['agree'] or c.get('arith_tie')) for c in cells),
    }


def batched_agreement(eng, posts, res, seed, ids, C, rows, streams=None):
    """Config 5's batched rounds (packed map, C = 24 candidates per (new_id,
    label) cell) against the C restatement of the reference's scoring
    (oracle/tpe_score.c, OpenMP): for every label and each row j in `rows`
    of res ([len(ids)][labels] results of suggest_batch(seed, ids, C)), the
    C candidates of round ids[j] re-drawn through the sampler entry points,
    scored under l and g in fp64, and broadcast_best's argmax (tpe.py:769-778)
    compared with the round's index and value (a value-only round reports
    those two for every cell).  Returns the per-cell agreement records."""
    from . import c_oracle as Cor
    cells = []
    for j in rows:
        rnd = int(ids[j])
        for li, p in enumerate(posts):
            stream = li if streams is None else int(streams[li])
            x = _draw(eng, p, stream, seed, rnd, C)
            if p.family == 'categorical':
                xi = x.astype(np.int64)
                lb, la = Cor.categorical_lpdf(xi, p.below), Cor.categorical_lpdf(xi, p.above)
            else:
                f = Cor.gmm1_lpdf if p.family == 'GMM1' else Cor.lgmm1_lpdf
                lb = f(x, *p.below, low=p.low, high=p.high, q=p.q)
                la = f(x, *p.above, low=p.low, high=p.high, q=p.q)
            best = Cor.broadcast_best_index(lb, la)
            r = res[j][li]
            cells.append({'row': int(j), 'label': li, 'family': p.family,
                          'agree': int(r['index']) == best and float(r['value']) == float(x[best]),
                          'hip': int(r['index']), 'oracle': best})
    return cells
