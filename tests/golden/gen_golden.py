"""Generate the golden fixtures for the TPE hot path FROM THE REFERENCE ITSELF.

Run in the survey container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

It imports the read-only reference at /root/reference (with the tiny
`future`/`past` stand-ins under tools/refshim) and, for every case, builds the
per-label posterior exactly the way `build_posterior` does
(tpe.py:670-724): `ap_filter_trials` node, the registered adaptive-Parzen
sampler for the prior's distribution (below and above), the `<sampler>_lpdf`
pair and `broadcast_best`, all evaluated by the reference's own `rec_eval`
with `np.random.RandomState(seed)`.  What it stores is DATA only: the inputs
(history, losses, gamma, prior weight, distribution args) and the outputs
(split, mixture weights/mus/sigmas, candidates, both lpdf vectors, best
index).  Nothing of the reference's source is copied.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(REPO, 'tools', 'refshim'), '/root/reference']

from hyperopt import pyll                       # noqa: E402  (reference)
from hyperopt.pyll import scope                 # noqa: E402
from hyperopt import tpe as rtpe                # noqa: E402

KINDS = {
    # kind: (pos-arg names, default args)   -- mirrors test_domains.many_dists
    'uniform': (('low', 'high'), dict(low=4.0, high=7.0)),
    'quniform': (('low', 'high', 'q'), dict(low=0.0, high=10.0, q=3.0)),
    'loguniform': (('low', 'high'), dict(low=-2.0, high=0.0)),
    'qloguniform': (('low', 'high', 'q'), dict(low=0.0, high=3.0, q=2.0)),
    'normal': (('mu', 'sigma'), dict(mu=4.0, sigma=7.0)),
    'qnormal': (('mu', 'sigma', 'q'), dict(mu=0.0, sigma=10.0, q=2.0)),
    'lognormal': (('mu', 'sigma'), dict(mu=-2.0, sigma=2.0)),
    'qlognormal': (('mu', 'sigma', 'q'), dict(mu=0.0, sigma=2.0, q=1.0)),
    'randint': (('upper',), dict(upper=10)),
    'categorical': (('p',), dict(p=[0.1, 0.9], upper=2)),
}


def prior_draw(kind, args, rng, n):
    """Observation values drawn from the prior (any values in the support are
    valid history; this only needs to be plausible)."""
    if kind == 'uniform':
        return rng.uniform(args['low'], args['high'], n)
    if kind == 'quniform':
        return np.round(rng.uniform(args['low'], args['high'], n) / args['q']) * args['q']
    if kind == 'loguniform':
        return np.exp(rng.uniform(args['low'], args['high'], n))
    if kind == 'qloguniform':
        return np.round(np.exp(rng.uniform(args['low'], args['high'], n)) / args['q']) * args['q']
    if kind == 'normal':
        return rng.normal(args['mu'], args['sigma'], n)
    if kind == 'qnormal':
        return np.round(rng.normal(args['mu'], args['sigma'], n) / args['q']) * args['q']
    if kind == 'lognormal':
        return np.exp(rng.normal(args['mu'], args['sigma'], n))
    if kind == 'qlognormal':
        return np.round(np.exp(rng.normal(args['mu'], args['sigma'], n)) / args['q']) * args['q']
    if kind == 'randint':
        return rng.randint(args['upper'], size=n)
    if kind == 'categorical':
        return rng.randint(args['upper'], size=n)
    raise ValueError(kind)


def run_reference_label(kind, args, o_idxs, o_vals, l_idxs, l_vals, gamma,
                        prior_weight, n_cand, seed):
    """One label of build_posterior, evaluated by the reference."""
    names, _ = KINDS[kind]
    aa = [args[k] for k in names]
    if kind == 'categorical':
        # the vectorized graph hands tpe_cat_pseudocounts an ndarray (tpe.py:602)
        aa = [pyll.Literal(np.asarray(args['p'], dtype=float))]
    named = {}
    if kind == 'categorical':
        named['upper'] = args['upper']
    s_oi, s_ov = pyll.Literal(list(o_idxs)), pyll.Literal(list(o_vals))
    s_li, s_lv = pyll.Literal(list(l_idxs)), pyll.Literal(list(l_vals))
    obs_below, obs_above = scope.ap_filter_trials(s_oi, s_ov, s_li, s_lv,
                                                  pyll.Literal(gamma))
    fn = rtpe.adaptive_parzen_samplers[kind]
    rng = pyll.Literal(np.random.RandomState(seed))
    size = pyll.Literal(n_cand)
    pw = pyll.Literal(float(prior_weight))
    b_post = fn(obs_below, pw, *aa, size=size, rng=rng, **named)
    a_post = fn(obs_above, pw, *aa, size=size, rng=rng, **named)
    fn_lpdf = getattr(scope, a_post.name + '_lpdf')
    a_kw = dict((n, a) for n, a in a_post.named_args if n not in ('rng', 'size'))
    b_kw = dict((n, a) for n, a in b_post.named_args if n not in ('rng', 'size'))
    below_llik = fn_lpdf(*([b_post] + b_post.pos_args), **b_kw)
    above_llik = fn_lpdf(*([b_post] + a_post.pos_args), **a_kw)
    best = scope.broadcast_best(b_post, below_llik, above_llik)
    if a_post.name == 'categorical':
        post_nodes = [b_post.pos_args[0], a_post.pos_args[0]]
    else:
        post_nodes = [scope.pos_args(*b_post.pos_args[:3]),
                      scope.pos_args(*a_post.pos_args[:3])]
    out = pyll.rec_eval(scope.pos_args(obs_below, obs_above, b_post, below_llik,
                                       above_llik, best, *post_nodes))
    below, above, samples, bl, al, bestv, pb, pa = out
    samples = np.asarray(samples)
    bl = np.asarray(bl, dtype=float)
    al = np.asarray(al, dtype=float)
    with np.errstate(invalid='ignore'):
        best_idx = int(np.argmax(bl - al)) if len(samples) else -1
    rec = dict(below=np.asarray(below, dtype=float), above=np.asarray(above, dtype=float),
               samples=samples.astype(float), lpdf_below=bl, lpdf_above=al,
               best_idx=np.int64(best_idx),
               best_val=np.float64(bestv[0]) if len(bestv) else np.float64(np.nan))
    if a_post.name == 'categorical':
        rec['p_below'] = np.asarray(pb, dtype=float)
        rec['p_above'] = np.asarray(pa, dtype=float)
    else:
        for tag, trip in (('b', pb), ('a', pa)):
            w, m, s = trip
            rec['w_' + tag] = np.asarray(w, dtype=float)
            rec['mu_' + tag] = np.asarray(m, dtype=float)
            rec['sigma_' + tag] = np.asarray(s, dtype=float)
    lpdf_kw = {k: (None if v is None else float(v)) for k, v in pyll.rec_eval(b_kw).items()}
    if a_post.name != 'categorical' and len(b_post.pos_args) > 3:
        # LGMM1(weights, mus, sigmas, low, high, q=q) passes the bounds
        # positionally (tpe.py:542); the lpdf receives them the same way
        extra = pyll.rec_eval(scope.pos_args(*b_post.pos_args[3:]))
        for name, v in zip(('low', 'high', 'q'), extra):
            lpdf_kw[name] = None if v is None else float(v)
    meta = dict(kind=kind, args=args, gamma=gamma, prior_weight=float(prior_weight),
                n_cand=n_cand, seed=seed, sampler=a_post.name, lpdf_kwargs=lpdf_kw)
    return meta, rec


def make_history(kind, args, n, rng, *, tied=False, frac_active=1.0, n_inf=0):
    tids = np.arange(n, dtype=np.int64) * 3 + 5          # sparse, sorted tids
    losses = rng.normal(size=n)
    if tied and n:
        losses = np.round(losses * 2) / 2                 # many equal losses
    if n_inf:
        losses[rng.choice(n, min(n_inf, n), replace=False)] = np.inf
    active = rng.uniform(size=n) < frac_active
    o_idxs = tids[active]
    o_vals = prior_draw(kind, args, rng, int(active.sum()))
    if tied and kind in ('uniform', 'normal', 'loguniform', 'lognormal') and len(o_vals) > 4:
        o_vals[1::4] = o_vals[0]                          # duplicate observations
    return o_idxs, o_vals, tids, losses


def gen_small():
    cases_meta, arrays = [], {}
    rng = np.random.RandomState(20240601)
    cid = 0
    for kind in KINDS:
        _, args = KINDS[kind]
        for n in (0, 1, 2, 26, 300):
            for variant in ('plain', 'tied', 'cond_inf'):
                if n < 26 and variant != 'plain':
                    continue
                kw = {}
                if variant == 'tied':
                    kw = dict(tied=True)
                elif variant == 'cond_inf':
                    kw = dict(frac_active=0.6, n_inf=max(1, n // 10))
                o_i, o_v, l_i, l_v = make_history(kind, args, n, rng, **kw)
                gamma = 0.25 if variant != 'cond_inf' else 0.15
                pw = 1.0 if variant != 'tied' else 2.5
                meta, rec = run_reference_label(kind, dict(args), o_i, o_v, l_i, l_v,
                                                gamma, pw, 64, 1000 + cid)
                meta.update(variant=variant, n_hist=n)
                for k, v in dict(o_idxs=o_i, o_vals=np.asarray(o_v, float), l_idxs=l_i,
                                 l_vals=l_v).items():
                    arrays['c%03d/%s' % (cid, k)] = v
                for k, v in rec.items():
                    arrays['c%03d/%s' % (cid, k)] = v
                cases_meta.append(meta)
                cid += 1
    arrays['meta'] = np.array(json.dumps(cases_meta))
    np.savez_compressed(os.path.join(HERE, 'labels_small.npz'), **arrays)
    print('labels_small:', cid, 'cases')


def gen_medium():
    """Larger mixtures for scoring parity: C=4096 candidates, K ~ 2k
    components (dense) / ~300 (quantized, whose reference loop is slow)."""
    cases_meta, arrays = [], {}
    rng = np.random.RandomState(7)
    specs = [('uniform', 2000, dict(low=-5.0, high=5.0)),
             ('normal', 2000, dict(mu=0.0, sigma=3.0)),
             ('loguniform', 2000, dict(low=-5.0, high=2.0)),
             ('lognormal', 1500, dict(mu=0.0, sigma=1.0)),
             ('quniform', 300, dict(low=0.0, high=100.0, q=1.0)),
             ('qloguniform', 300, dict(low=float(np.log(10)), high=float(np.log(1000)), q=1.0)),
             ('qnormal', 300, dict(mu=0.0, sigma=10.0, q=0.5)),
             ('randint', 2000, dict(upper=5))]
    for cid, (kind, n, args) in enumerate(specs):
        o_i, o_v, l_i, l_v = make_history(kind, args, n, rng)
        meta, rec = run_reference_label(kind, args, o_i, o_v, l_i, l_v, 0.25, 1.0,
                                        4096, 77 + cid)
        meta.update(variant='medium', n_hist=n)
        for k, v in dict(o_idxs=o_i, o_vals=np.asarray(o_v, float), l_idxs=l_i,
                         l_vals=l_v).items():
            arrays['c%03d/%s' % (cid, k)] = v
        for k, v in rec.items():
            arrays['c%03d/%s' % (cid, k)] = v
        cases_meta.append(meta)
    arrays['meta'] = np.array(json.dumps(cases_meta))
    np.savez_compressed(os.path.join(HERE, 'labels_medium.npz'), **arrays)
    print('labels_medium:', len(specs), 'cases')


def gen_lpdf_edges():
    """Direct calls of the reference lpdf functions on hand-picked edge inputs:
    far tails (LSE shift must not underflow), quantized tails that cancel to
    log(0) = -inf, NaN-producing inputs, bounded vs unbounded LGMM1."""
    cases, arrays = [], {}
    w = np.array([.1, .3, .4, .2])
    mu = np.array([1.0, 2.0, 3.0, 4.0])
    sg = np.array([.1, .4, .8, 2.0])
    xs = np.array([-1e3, -50.0, -3.0, 0.0, 0.999, 1.0, 2.5, 3.3, 4.0, 7.0, 40.0, 1e3])
    lxs = np.array([0.0, 1e-300, 1e-12, 0.05, 0.5, 1.0, 2.0, 7.5, 30.0, 1e5])
    calls = [('GMM1_lpdf', xs, dict()), ('GMM1_lpdf', xs, dict(low=0.5, high=3.5)),
             ('GMM1_lpdf', xs, dict(q=1.0)), ('GMM1_lpdf', xs, dict(q=0.5, low=1.0, high=4.1)),
             ('GMM1_lpdf', np.array([-1e3, 60.0, 1e3]), dict(q=2.0)),
             ('LGMM1_lpdf', lxs, dict()), ('LGMM1_lpdf', lxs, dict(low=-1.0, high=2.0)),
             ('LGMM1_lpdf', lxs, dict(q=1.0)), ('LGMM1_lpdf', lxs, dict(q=0.5, low=0.0, high=1.5)),
             ('LGMM1_lpdf', np.array([0.0, 3.0, 1e4]), dict(q=2.0, low=-1.0, high=1.0))]
    for cid, (name, x, kw) in enumerate(calls):
        f = getattr(rtpe, name)
        with np.errstate(all='ignore'):
            out = np.asarray(f(x, w, mu, sg, **kw), dtype=float)
        cases.append(dict(fn=name, kwargs=kw))
        arrays['e%03d/x' % cid] = x
        arrays['e%03d/out' % cid] = out
    # broadcast_best semantics: NaN greatest, first index wins
    bb = [np.array([1.0, 3.0, 3.0, -np.inf]), np.array([0.0, np.nan, np.inf, np.nan]),
          np.array([-np.inf, -np.inf]), np.array([np.inf, np.nan])]
    for i, s in enumerate(bb):
        arrays['bb%02d/score' % i] = s
        arrays['bb%02d/best' % i] = np.int64(np.argmax(s))
    arrays['meta'] = np.array(json.dumps(dict(w=w.tolist(), mu=mu.tolist(),
                                              sigma=sg.tolist(), calls=cases, n_bb=len(bb))))
    np.savez_compressed(os.path.join(HERE, 'lpdf_edges.npz'), **arrays)
    print('lpdf_edges:', len(calls), 'calls')


if __name__ == '__main__':
    gen_small()
    gen_medium()
    gen_lpdf_edges()
