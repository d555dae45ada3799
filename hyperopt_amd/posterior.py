"""Per-label posterior descriptors: the host half of the hot path.

Replaces the graph rewrite of `build_posterior` (hyperopt/tpe.py:651-739)
with a flat table: for every hyperparameter label, the below (l) and above (g)
Parzen mixtures as rows of a `tpe_label_desc` plus flat weight/mu/sigma
arrays, uploaded once per suggestion round to the GPU engine.

The arithmetic reproduces the reference bit-for-bit (same numpy calls in the
same order, including the default, non-stable np.argsort tie order):
  split         ap_filter_trials              tpe.py:624-648
  LF weights    linear_forgetting_weights     tpe.py:385-398
  Parzen        adaptive_parzen_normal        tpe.py:404-477
  priors        ap_*_sampler registry         tpe.py:493-576
  categorical   pseudocount posteriors        tpe.py:581-617
It is vectorised over the history (no per-trial Python loops).
"""
import threading
import time
import weakref

import numpy as np

from . import _lib as L
from .engine import DESC_DTYPE

# host-timer breakdown of the fmin step's posterior work (bench.py's
# `advance_breakdown_ms`): None, or a dict phase -> [calls, seconds]
PHASES = None


def _phase(name, t0):
    """Account perf_counter() - t0 to `name` (when PHASES is on); returns
    the new t0."""
    t = time.perf_counter()
    if PHASES is not None:
        c = PHASES.setdefault(name, [0, 0.0])
        c[0] += 1
        c[1] += t - t0
    return t

EPS = 1e-12
DEFAULT_LF = 25

CONTINUOUS = ('uniform', 'quniform', 'loguniform', 'qloguniform',
              'normal', 'qnormal', 'lognormal', 'qlognormal')
CATEGORICAL = ('randint', 'categorical')


def split_history(l_idxs, l_vals, gamma, gamma_cap=DEFAULT_LF):
    """Global loss-rank split (tpe.py:636-645): tids of the n_below best
    trials and of the rest."""
    l_idxs = np.asarray(l_idxs)
    l_vals = np.asarray(l_vals)
    n_below = min(int(np.ceil(gamma * np.sqrt(len(l_vals)))), gamma_cap)
    order = np.argsort(l_vals)
    return l_idxs[order[:n_below]], l_idxs[order[n_below:]]


def split_label(o_idxs, o_vals, below_tids, above_tids):
    """Observations of one label that belong to below / above trials, in
    their original order (tpe.py:640, :646)."""
    o_idxs = np.asarray(o_idxs)
    o_vals = np.asarray(o_vals)
    if len(o_idxs) == 0:
        return np.asarray([]), np.asarray([])
    return (o_vals[np.isin(o_idxs, below_tids)], o_vals[np.isin(o_idxs, above_tids)])


class Splitter(object):
    """split_history + split_label for many labels sharing one history: the
    membership of a tid is looked up by binary search in the sorted tids
    (one O(M log N) pass per label instead of np.isin's sorts)."""

    def __init__(self, l_idxs, l_vals, gamma, gamma_cap=DEFAULT_LF):
        below, above = split_history(l_idxs, l_vals, gamma, gamma_cap)
        tids = np.concatenate([below, above])
        side = np.concatenate([np.ones(len(below), dtype=np.int8),
                               np.full(len(above), 2, dtype=np.int8)])
        order = np.argsort(tids, kind='stable')
        self.tids = tids[order]
        self.side = side[order]

    def split(self, o_idxs, o_vals):
        o_idxs = np.asarray(o_idxs)
        o_vals = np.asarray(o_vals)
        if len(o_idxs) == 0 or len(self.tids) == 0:
            return np.asarray([]), np.asarray([])
        pos = np.searchsorted(self.tids, o_idxs)
        pos_c = np.minimum(pos, len(self.tids) - 1)
        hit = self.tids[pos_c] == o_idxs
        side = np.where(hit, self.side[pos_c], 0)
        return o_vals[side == 1], o_vals[side == 2]


def linear_forgetting_weights(n, lf):
    if n == 0:
        return np.asarray([])
    if n < lf:
        return np.ones(n)
    return np.concatenate([np.linspace(1.0 / n, 1.0, num=n - lf), np.ones(lf)], axis=0)


def adaptive_parzen_normal(mus, prior_weight, prior_mu, prior_sigma, lf=DEFAULT_LF):
    """(weights, mus, sigmas), sorted by mu, prior inserted (tpe.py:404-477)."""
    mus = np.asarray(mus, dtype=float)
    if mus.ndim != 1:
        raise TypeError('mus must be vector', mus)
    n = len(mus)
    order = None
    if n == 0:
        srtd = np.asarray([prior_mu], dtype=float)
        sigma = np.asarray([prior_sigma], dtype=float)
        pos = 0
    elif n == 1:
        pos = 0 if prior_mu < mus[0] else 1
        srtd = np.asarray([prior_mu, mus[0]] if pos == 0 else [mus[0], prior_mu], dtype=float)
        sigma = np.asarray([prior_sigma, prior_sigma * .5] if pos == 0
                           else [prior_sigma * .5, prior_sigma], dtype=float)
    else:
        order = np.argsort(mus)
        sorted_mus = mus[order]
        pos = int(np.searchsorted(sorted_mus, prior_mu))
        srtd = np.insert(sorted_mus, pos, prior_mu)
        sigma = np.empty_like(srtd)
        gaps = np.diff(srtd)
        sigma[1:-1] = np.maximum(gaps[:-1], gaps[1:])
        sigma[0] = gaps[0]
        sigma[-1] = gaps[-1]
    if lf and lf < n:
        lfw = linear_forgetting_weights(n, lf)
        weights = np.insert(lfw[order], pos, prior_weight)
    else:
        weights = np.ones(len(srtd))
        weights[pos] = prior_weight
    maxsigma = prior_sigma / 1.0
    minsigma = prior_sigma / min(100.0, (1.0 + len(srtd)))
    sigma = np.clip(sigma, minsigma, maxsigma)
    sigma[pos] = prior_sigma
    if not (prior_sigma > 0 and np.all(sigma > 0)):
        raise AssertionError('non-positive sigma in adaptive_parzen_normal')
    return weights / weights.sum(), srtd, sigma


class LabelPosterior(object):
    """Both posteriors of one label, ready to pack into a descriptor row."""
    __slots__ = ('label', 'family', 'low', 'high', 'q', 'below', 'above', 'upper')

    def __init__(self, label, family, below, above, low=None, high=None, q=None, upper=None):
        self.label, self.family = label, family
        self.below, self.above = below, above   # (w, mu, sigma) or p
        self.low, self.high, self.q, self.upper = low, high, q, upper


def label_posterior(label, kind, args, below, above, prior_weight):
    """Prior mapping of the adaptive-Parzen sampler registry."""
    pw = float(prior_weight)
    if kind in CATEGORICAL:
        upper = int(args['upper'])
        ps = []
        for obs in (below, above):
            obs = np.asarray(obs)
            lfw = linear_forgetting_weights(len(obs), DEFAULT_LF)
            counts = (np.bincount(obs.astype(int), minlength=upper, weights=lfw)
                      if len(obs) else np.zeros(upper))
            if kind == 'randint':                              # tpe.py:584-588
                pseudo = counts + pw
            else:                                              # tpe.py:605-606
                pseudo = counts + upper * (pw * np.asarray(args['p'], dtype=float))
            ps.append(pseudo / np.sum(pseudo))
        return LabelPosterior(label, 'categorical', ps[0], ps[1], upper=upper)
    if kind in ('uniform', 'quniform', 'loguniform', 'qloguniform'):
        low, high = float(args['low']), float(args['high'])
        prior_mu, prior_sigma = 0.5 * (high + low), 1.0 * (high - low)
        q = float(args['q']) if kind in ('quniform', 'qloguniform') else None
        if kind in ('uniform', 'quniform'):
            tr, fam = (lambda o: o), 'GMM1'
        elif kind == 'loguniform':
            tr, fam = np.log, 'LGMM1'
        else:
            floor = np.maximum(EPS, np.exp(low))              # tpe.py:536-540
            tr, fam = (lambda o: np.log(np.maximum(o, floor))), 'LGMM1'
        mix = [adaptive_parzen_normal(tr(np.asarray(o, dtype=float)), pw, prior_mu, prior_sigma)
               for o in (below, above)]
        return LabelPosterior(label, fam, mix[0], mix[1], low=low, high=high, q=q)
    mu, sigma = float(args['mu']), float(args['sigma'])
    q = float(args['q']) if kind in ('qnormal', 'qlognormal') else None
    if kind in ('normal', 'qnormal'):
        tr, fam = (lambda o: o), 'GMM1'
    elif kind == 'lognormal':
        tr, fam = np.log, 'LGMM1'
    elif kind == 'qlognormal':
        tr, fam = (lambda o: np.log(np.maximum(o, EPS))), 'LGMM1'
    else:
        raise ValueError('unknown distribution %r' % kind)
    mix = [adaptive_parzen_normal(tr(np.asarray(o, dtype=float)), pw, mu, sigma)
           for o in (below, above)]
    return LabelPosterior(label, fam, mix[0], mix[1], q=q)


def label_spec(kind, args):
    """The tpe_label_spec fields of one hyperparameter and its observation
    transform (the prior mapping of the ap_*_sampler registry, tpe.py:493-617):
    (spec dict, transform function, categorical p or None)."""
    if kind in CATEGORICAL:
        upper = int(args['upper'])
        p = None if kind == 'randint' else np.asarray(args['p'], dtype=float)
        return dict(kind=L.TPE_CATEGORICAL, flags=0, upper=upper,
                    randint=1 if kind == 'randint' else 0), None, p
    if kind in ('uniform', 'quniform', 'loguniform', 'qloguniform'):
        low, high = float(args['low']), float(args['high'])
        spec = dict(low=low, high=high, prior_mu=0.5 * (high + low), prior_sigma=1.0 * (high - low),
                    flags=L.TPE_HAS_LOW | L.TPE_HAS_HIGH)
        if kind in ('quniform', 'qloguniform'):
            spec['q'] = float(args['q'])
            spec['flags'] |= L.TPE_HAS_Q
        if kind in ('uniform', 'quniform'):
            spec['kind'], tr = L.TPE_GMM1, None
        elif kind == 'loguniform':
            spec['kind'], tr = L.TPE_LGMM1, np.log
        else:
            floor = np.maximum(EPS, np.exp(low))              # tpe.py:536-540
            spec['kind'], tr = L.TPE_LGMM1, (lambda o: np.log(np.maximum(o, floor)))
            tr.floor = float(floor)
        return spec, tr, None
    spec = dict(prior_mu=float(args['mu']), prior_sigma=float(args['sigma']), flags=0)
    if kind in ('qnormal', 'qlognormal'):
        spec['q'] = float(args['q'])
        spec['flags'] = L.TPE_HAS_Q
    if kind in ('normal', 'qnormal'):
        spec['kind'], tr = L.TPE_GMM1, None
    elif kind == 'lognormal':
        spec['kind'], tr = L.TPE_LGMM1, np.log
    elif kind == 'qlognormal':
        spec['kind'], tr = L.TPE_LGMM1, (lambda o: np.log(np.maximum(o, EPS)))
        tr.floor = float(EPS)
    else:
        raise ValueError('unknown distribution %r' % kind)
    return spec, tr, None


def spec_table(labels, streams=None):
    """(SPEC_DTYPE array, concatenated categorical p, per-label observation
    transform or None) for labels = [(name, kind, args)]; streams: each
    label's Philox stream (default its position) -- a subset of a space's
    labels keeps the streams, hence the candidates, it has in the whole space."""
    from .engine import SPEC_DTYPE
    specs = np.zeros(len(labels), dtype=SPEC_DTYPE)
    cat_p, p_len, trs = [], 0, []
    for i, (name, kind, args) in enumerate(labels):
        sp, tr, p = label_spec(kind, args)
        for k, v in sp.items():
            specs[i][k] = v
        if p is not None:
            specs[i]['p_off'] = p_len
            cat_p.append(p)
            p_len += len(p)
        if streams is not None:
            specs[i]['flags'] |= L.TPE_HAS_STREAM
            specs[i]['stream'] = int(streams[i])
        trs.append(tr)
    return specs, (np.concatenate(cat_p) if cat_p else np.zeros(0)), trs


def n_below_of(n_valid, gamma, gamma_cap=DEFAULT_LF):
    """min(ceil(gamma sqrt(len(l_vals))), gamma_cap), tpe.py:636 (gamma_cap
    is ap_filter_trials' default DEFAULT_LF, :626, independent of the linear
    forgetting)."""
    return int(min(np.ceil(gamma * np.sqrt(n_valid)), gamma_cap))


def reference_orders(losses, n_below, obs_of, labels):
    """The reference's own np.argsort orders, for the device builder's
    `tpe_build_posterior_resident_ordered`: the below set as
    ap_filter_trials picks it (`l_order = np.argsort(l_vals)`, tpe.py:637;
    l_vals = the losses of the trials that have one, in tid order) and, for
    each label in `labels`, np.argsort of its above observations in
    observation order (adaptive_parzen_normal's `order = np.argsort(mus)`,
    tpe.py:433) -- numpy's unstable sort on the same arrays, so equal keys
    land where the reference puts them.  obs_of(l) -> (trial position per
    observation, -1 for none; transformed value); obs_of.n_labels = L.
    Returns (below mask per trial position, order_off[L + 1], order), with
    empty ranges for the labels not in `labels`."""
    losses = np.asarray(losses, dtype=np.float64)
    T = len(losses)
    has = losses == losses
    valid = np.flatnonzero(has)
    lv = losses[valid]
    below = np.zeros(T, dtype=np.uint8)
    if 0 < n_below < len(lv):
        # the n_below smallest: unique when the boundary values differ (an
        # O(N) partition); a tie across the boundary takes np.argsort's pick
        part = np.partition(lv, (n_below - 1, n_below))
        if part[n_below - 1] < part[n_below]:
            below[valid[lv <= part[n_below - 1]]] = 1
        else:
            below[valid[np.argsort(lv)[:n_below]]] = 1      # tpe.py:637
    elif n_below > 0:
        below[valid] = 1
    # the above set per trial position: a loss, not below (tpe.py:645-646)
    above = has & (below == 0)
    n_labels = obs_of.n_labels
    off = np.zeros(n_labels + 1, dtype=np.int64)
    jobs = []   # (label, values, selection mask) in label order
    n_above = None
    for l in range(n_labels):
        n = 0
        if l in labels:
            pos, val = obs_of(l)
            val = np.asarray(val, dtype=np.float64)
            if len(pos) == T and T and pos[0] == 0 and pos[-1] == T - 1:
                sel = above                          # positions 0..T-1 (one per trial, in order)
                if n_above is None:
                    n_above = int(np.count_nonzero(above))
                n = n_above
            else:
                pos = np.asarray(pos, dtype=np.int64)
                ok = (pos >= 0) & (pos < T)
                sel = np.zeros(len(pos), dtype=bool)
                sel[ok] = above[pos[ok]]
                n = int(np.count_nonzero(sel))
            jobs.append((l, val, sel))
        off[l + 1] = off[l] + n
    order = np.empty(int(off[-1]), dtype=np.int32)

    def sort_one(job):
        # np.argsort(mus) (tpe.py:433) into the label's range of `order`
        l, val, sel = job
        order[off[l]:off[l + 1]] = np.argsort(val[sel])

    # numpy sorts (and gathers) without the GIL, so many long ones -- their
    # gathers and int32 stores too, 2/3 of the work on one thread (r5am) --
    # go to a thread pool
    if jobs and off[-1] >= _POOL_MIN:
        for _ in _sort_pool().map(sort_one, jobs):
            pass
    else:
        for job in jobs:
            sort_one(job)
    return below, off, order


EARLY_ORDERS = True   # known labels' argsorts started before the first build (build_reference_order)
_order_exec = None


def _order_thread():
    """One worker for reference_orders started ahead of the build (its
    argsorts go on to the sort pool: a separate executor, so the pool's
    workers never wait on themselves)."""
    global _order_exec
    if _order_exec is None:
        with _pool_lock:
            if _order_exec is None:
                from concurrent.futures import ThreadPoolExecutor
                _order_exec = ThreadPoolExecutor(max_workers=1)
    return _order_exec


_POOL_MIN = 1 << 14   # observations to sort (over several labels), from which the pool pays
SORT_THREADS = 16     # the argsort pool's threads at most (bench.py --sort-threads)
_pool = None
_pool_lock = threading.Lock()


def _sort_pool():
    """The process's one argsort pool (created once, also under concurrent
    tpe.suggest callers: each thread has its own engine, not its own pool)."""
    global _pool
    if _pool is None:
        with _pool_lock:
            if _pool is None:
                import os
                from concurrent.futures import ThreadPoolExecutor
                try:   # the CPUs this process may run on (a GPU box's share), at most 16
                    ncpu = len(os.sched_getaffinity(0))
                except (AttributeError, OSError):
                    ncpu = os.cpu_count() or 2
                _pool = ThreadPoolExecutor(max_workers=max(1, min(SORT_THREADS, ncpu)))
    return _pool


SUBSET_REBUILD = True   # the ordered rebuild restricted to the labels that need an order
DEFER_REPORT = True     # round_call: that rebuild's report read after the round (Engine.rebuild_labels(defer=))


def build_reference_order(eng, losses, n_valid, gamma, prior_weight, lf, obs_of, known=(), prepare=None,
                          overlap=True, round_call=None, early=None):
    """_build_reference_order (below), waiting on the early argsorts' future
    whatever happens: its worker reads (and caches into) the uploader's
    observation lists, which a failed build must not leave it writing to
    while the next call appends."""
    holder = {'early': early}
    try:
        return _build_reference_order(eng, losses, n_valid, gamma, prior_weight, lf, obs_of, known,
                                      prepare, overlap, round_call, holder)
    finally:
        if holder['early'] is not None:
            from concurrent.futures import wait
            wait([holder['early']])


def _build_reference_order(eng, losses, n_valid, gamma, prior_weight, lf, obs_of, known, prepare,
                           overlap, round_call, holder):
    """Device build whose mixtures follow the reference's tie order
    (tpe.py:433, 637): the device reports which mixtures depend on the order
    of tied observations (or a tie of losses at the split), and only for
    those the host computes numpy's own np.argsort and the build runs again
    with it.

    * prepare None: `known` -- the labels that needed an order in the
      previous build of this history -- get their orders up front (one
      build when nothing new turns up);
    * prepare = (candidates per label, rounds) of the coming round, with
      enough candidates to use the expansion index: the first build is
      made without orders, the expansion index of its dense labels is queued
      on the device (Engine.prepare), and the host computes the orders while
      it runs; the ordered rebuild leaves the dense labels bit-identical
      (continuous values carry no ties), so the device keeps the index;
      with overlap=False (few labels use the index: it is shorter than the
      second build it saves) the `known` orders go up front as above and the
      index is queued after the one build.

    round_call (optional): the coming round, a callable returning the
    engine's results; it then runs here and its results are returned as a
    third value (a subset rebuild's report is then read after the round:
    DEFER_REPORT).

    holder['early'] (optional): reference_orders(losses, n_below, obs_of,
    known) already running (a future: DeviceHistoryUploader.build starts it
    before its upload); a future started here is left there too.

    Returns (n_below, the labels that needed an order[, results])."""
    early = holder['early']
    n_below = n_below_of(n_valid, gamma)
    known = set(known)
    t0 = time.perf_counter()
    if prepare and (overlap or not known):
        if known and EARLY_ORDERS and early is None:
            # the previous build's order-dependent labels: their argsorts
            # start now, on the host, under the first build and the index
            early = holder['early'] = _order_thread().submit(reference_orders, losses, n_below, obs_of,
                                                             known)
        # the build queues the index itself before it returns (tpe_arm_prepare);
        # the prepare after it is then a no-op
        eng.arm_prepare(*prepare)
        nb, ties = eng.build_posterior_ordered(losses, n_valid, gamma, prior_weight, lf)
        t0 = _phase('build', t0)
        eng.prepare(*prepare)
        t0 = _phase('prepare_enqueue', t0)
        have = set()
    elif known:
        below, off, order = reference_orders(losses, n_below, obs_of, known)
        t0 = _phase('argsorts', t0)
        if prepare:
            eng.arm_prepare(*prepare)
        nb, ties = eng.build_posterior_ordered(losses, n_valid, gamma, prior_weight, lf, below, off, order)
        t0 = _phase('build', t0)
        if prepare:
            eng.prepare(*prepare)
            t0 = _phase('prepare_enqueue', t0)
        have = known
    else:
        nb, ties = eng.build_posterior_ordered(losses, n_valid, gamma, prior_weight, lf)
        t0 = _phase('build', t0)
        have = set()
    if np.any(ties[:-1] & 1):
        # a below mixture holds at most gamma_cap <= lf observations: its
        # weights are all equal, so its order can never matter
        raise AssertionError('below mixture depends on a tie order (lf < gamma_cap?)')
    need = have | set(np.flatnonzero(ties[:-1] & 2).tolist())
    res = None
    deferred = False
    if early is not None:
        orders = early.result()   # (waited for even when unused: obs_of is not shared)
        if need != have and need <= known:
            # rebuild every known label (an ordered build is right for any)
            need = set(known)
            below, off, order = orders
        else:
            early = None
    if need != have or ties[-1]:
        if early is None:
            below, off, order = reference_orders(losses, n_below, obs_of, need)
        t0 = _phase('argsorts', t0)
        if SUBSET_REBUILD and not ties[-1] and len(need) < obs_of.n_labels:
            # no tie across the split (the below set is the one just built):
            # rebuild only the labels that needed an order -- with a round
            # to follow, without waiting for its report (a rebuild of
            # quantized / categorical labels runs on the second stream; the
            # round queues the dense labels' kernels before it waits), its
            # tie check made after the round
            deferred = (DEFER_REPORT and round_call is not None and len(getattr(eng, 'devices', ())) == 1
                        and hasattr(eng, 'build_report'))
            nb, ties = eng.rebuild_labels(losses, n_valid, gamma, prior_weight, lf, off, order, need,
                                          defer=deferred)
        else:
            nb, ties = eng.build_posterior_ordered(losses, n_valid, gamma, prior_weight, lf, below, off,
                                                   order)
        t0 = _phase('rebuild', t0)
        if np.any(ties[:-1]):
            # a supplied below set can move observations between the sets,
            # creating a dependent label the first pass did not see
            need |= set(np.flatnonzero(ties[:-1] & 2).tolist())
            below, off, order = reference_orders(losses, n_below, obs_of, need)
            nb, ties = eng.build_posterior_ordered(losses, n_valid, gamma, prior_weight, lf, below, off,
                                                   order)
            assert not np.any(ties[:-1])
    if round_call is not None:
        res = round_call()
        if deferred:
            nb, ties = eng.build_report()
            if np.any(ties[:-1]):
                # (as above, found after the round: the ordered build with
                # the dependent labels, and the round again)
                need |= set(np.flatnonzero(ties[:-1] & 2).tolist())
                below, off, order = reference_orders(losses, n_below, obs_of, need)
                nb, ties = eng.build_posterior_ordered(losses, n_valid, gamma, prior_weight, lf, below, off,
                                                       order)
                assert not np.any(ties[:-1])
                res = round_call()
        _phase('round', t0)
        return nb, frozenset(need), res
    return nb, frozenset(need)


class _ObsOf(object):
    """obs_of(l) over CSR observation arrays (tpe_build_posterior's layout)."""

    def __init__(self, obs_off, obs_trial, obs_val):
        self.off, self.trial, self.val = obs_off, obs_trial, obs_val
        self.n_labels = len(obs_off) - 1

    def __call__(self, l):
        a, b = int(self.off[l]), int(self.off[l + 1])
        return self.trial[a:b], self.val[a:b]


class NonFiniteObservation(ValueError):
    """A transformed observation is NaN (e.g. the log of a non-positive value
    of a log-scale label inserted through points_to_evaluate).  The
    reference's adaptive_parzen_normal then trips its `sigma > 0` assertion
    (tpe.py:469) in the host build; the device builder cannot order NaN
    keys, so it refuses them (tpe.suggest falls back to the host builder)."""


def _check_finite(label, vals):
    if np.isnan(vals).any():
        raise NonFiniteObservation('label %r: NaN observation value' % (label,))


class DeviceHistoryUploader(object):
    """Keeps an Engine's device-resident history (tpe_history_*) in step with
    a growing trial history: only observations added since the last call are
    transformed and uploaded; anything else (new labels, another history --
    the owner is held by weak reference, so a collected history's address
    reused by a new one does not match --, a history replaced on the device
    by another call, a trial inserted before existing ones) resets it."""

    def __init__(self):
        self.key = None
        self.owner = None

    def build(self, eng, labels, view, gamma, prior_weight, lf=DEFAULT_LF, prepare=None, streams=None,
              overlap=True, round_call=None):
        """Upload what is new and build the posterior; returns (n_below,
        results): results of round_call (the coming round: see
        build_reference_order), None without one."""
        tids, losses, n_valid, cols, owner = view
        names_now = tuple(n for n, _, _ in labels)
        if (labels is not self._labels_obj or streams is not self._streams_obj or
                names_now != self._names_t):
            # (the label key of a caller that passes the same list every
            # step -- FminLoop -- is built once; the names tuple catches a
            # list changed in place -- ADVICE r5)
            self._labels_obj, self._streams_obj, self._names_t = labels, streams, names_now
            self._label_key = (tuple((n, k) for n, k, _ in labels) +
                               (tuple(streams) if streams is not None else (),))
            self._names = [n for n, _, _ in labels]
        key = (self._label_key, eng.history_generation)
        names = self._names
        obs_now = [cols[n] for n in names]
        lens = [len(o[0]) for o in obs_now]
        same_owner = self.owner is not None and self.owner() is owner
        fresh = (not same_owner or self.key != key or len(tids) < self.n_trials or
                 (self.n_trials and tids[self.n_trials - 1] != self.last_tid) or
                 any(a < c for a, c in zip(lens, self.prev_counts)))
        # invalid until the device holds exactly what prev_counts says
        self.key, self.owner = None, None
        if fresh:
            specs, cat_p, self.trs = spec_table(labels, streams)
            # per label: 0 identity, 1 np.log, 2 np.log(np.maximum(o, floor))
            self.tr_kind = np.array([0 if t is None else (1 if t is np.log else 2) for t in self.trs])
            self.tr_floor = np.array([getattr(t, 'floor', -np.inf) for t in self.trs])
            eng.history_reset(specs, cat_p)
            self.prev_counts = [0] * len(labels)
            self.pos_parts = [[] for _ in labels]    # what the device holds, per label
            self.val_parts = [[] for _ in labels]
            self.tie_labels = frozenset()
        t0 = time.perf_counter()
        counts = lens
        # the new observations of every label, transformed and placed in one
        # vectorised pass (a per-label numpy loop cost ~0.4 ms per fmin step
        # at 32 labels): np.log / np.log(np.maximum(o, floor)) elementwise,
        # as the reference's samplers transform them (tpe.py:493-576)
        n_new = [a - c for a, c in zip(lens, self.prev_counts)]
        ni_l = [o[0][c:] for o, c, m in zip(obs_now, self.prev_counts, n_new) if m]
        nv_l = [o[1][c:] for o, c, m in zip(obs_now, self.prev_counts, n_new) if m]
        if ni_l:
            ni = np.concatenate(ni_l)
            raw = np.asarray(np.concatenate(nv_l), dtype=float)
            lab = np.repeat(np.arange(len(labels)), n_new)
            kind = self.tr_kind[lab]
            vals = raw.copy()
            lg = kind > 0
            if lg.any():
                vals[lg] = np.log(np.maximum(raw[lg], self.tr_floor[lab[lg]]))
            nan = np.isnan(vals)
            if nan.any():
                raise NonFiniteObservation('label %r: NaN observation value'
                                           % (labels[int(lab[np.argmax(nan)])][0],))
            pos = np.searchsorted(tids, ni)
            pc = np.minimum(pos, len(tids) - 1)
            trial = np.where(tids[pc] == ni, pc, -1).astype(np.int32)
            o = 0
            for i, m in enumerate(n_new):
                if m:
                    self.pos_parts[i].append(trial[o:o + m])
                    self.val_parts[i].append(vals[o:o + m])
                    o += m
        # (a failed upload leaves this uploader invalid: the next call resets)
        if ni_l:
            eng.history_append(np.asarray(n_new, dtype=np.int64), trial, vals)
        self.prev_counts = counts                  # committed only after the append
        self.key = (key[0], eng.history_generation)
        self.owner = weakref.ref(owner)
        self.n_trials = len(tids)
        self.last_tid = tids[-1] if len(tids) else None
        _phase('append', t0)
        out = build_reference_order(eng, losses, n_valid, gamma, prior_weight, lf,
                                    self._obs_of(len(labels)), self.tie_labels,
                                    prepare=prepare, overlap=overlap, round_call=round_call)
        self.tie_labels = out[1]
        return out[0], (out[2] if round_call is not None else None)

    def _obs_of(self, n_labels):
        def obs_of(l):
            for parts in (self.pos_parts, self.val_parts):
                if len(parts[l]) > 1:
                    parts[l][:] = [np.concatenate(parts[l])]
            if not self.pos_parts[l]:
                return np.zeros(0, np.int32), np.zeros(0)
            return self.pos_parts[l][0], self.val_parts[l][0]
        obs_of.n_labels = n_labels
        return obs_of

    prev_counts = ()
    _labels_obj = _streams_obj = _names_t = None
    pos_parts = val_parts = ()
    tie_labels = frozenset()
    n_trials = 0
    last_tid = None
    trs = ()


def device_inputs(labels, tids, losses, obs):
    """Arguments of Engine.build_posterior (tpe_build_posterior) for a
    history: labels = [(name, kind, args)], tids/losses of the represented
    trials in tid order, obs[name] = (idxs, vals) in tid order.  Observations
    are transformed here with the reference's own numpy expressions, and
    mapped to their trial's position (-1 when the tid has no loss entry,
    which ap_filter_trials drops, tpe.py:639-646)."""
    from .engine import SPEC_DTYPE
    tids = np.asarray(tids, dtype=np.int64)
    specs = np.zeros(len(labels), dtype=SPEC_DTYPE)
    cat_p, p_len = [], 0
    off = [0]
    trial_parts, val_parts = [], []
    for i, (name, kind, args) in enumerate(labels):
        sp, tr, p = label_spec(kind, args)
        for k, v in sp.items():
            specs[i][k] = v
        if p is not None:
            specs[i]['p_off'] = p_len
            cat_p.append(p)
            p_len += len(p)
        oi, ov = obs[name]
        oi = np.asarray(oi, dtype=np.int64)
        ov = np.asarray(ov, dtype=float)
        if tr is not None and len(ov):
            ov = tr(ov)
        _check_finite(name, ov)
        if len(oi) == len(tids) and len(oi) and oi[0] == tids[0] and oi[-1] == tids[-1] \
                and np.array_equal(oi, tids):
            pos = np.arange(len(oi))                 # label active in every trial
        elif len(tids) and len(oi):
            pos = np.searchsorted(tids, oi)
            pc = np.minimum(pos, len(tids) - 1)
            pos = np.where(tids[pc] == oi, pc, -1)
        else:
            pos = np.full(len(oi), -1, dtype=np.int64)
        trial_parts.append(pos.astype(np.int32))
        val_parts.append(ov)
        off.append(off[-1] + len(oi))
    cat = np.concatenate(cat_p) if cat_p else np.zeros(0)
    return (specs, cat, np.asarray(losses, dtype=float), np.asarray(off, dtype=np.int64),
            np.concatenate(trial_parts) if trial_parts else np.zeros(0, np.int32),
            np.concatenate(val_parts) if val_parts else np.zeros(0))


def pack(posts):
    """Flatten a list of LabelPosterior into (descs, weights, mus, sigmas)."""
    descs = np.zeros(len(posts), dtype=DESC_DTYPE)
    ws, ms, ss = [], [], []
    off = 0
    for i, p in enumerate(posts):
        d = descs[i]
        if p.family == 'categorical':
            d['kind'] = L.TPE_CATEGORICAL
            parts = [(p.below, np.zeros_like(p.below), np.zeros_like(p.below)),
                     (p.above, np.zeros_like(p.above), np.zeros_like(p.above))]
        else:
            d['kind'] = L.TPE_GMM1 if p.family == 'GMM1' else L.TPE_LGMM1
            flags = 0
            if p.low is not None:
                flags |= L.TPE_HAS_LOW
                d['low'] = p.low
            if p.high is not None:
                flags |= L.TPE_HAS_HIGH
                d['high'] = p.high
            if p.q is not None:
                flags |= L.TPE_HAS_Q
                d['q'] = p.q
            d['flags'] = flags
            parts = [p.below, p.above]
        for side, (w, m, s) in zip(('below', 'above'), parts):
            d[side + '_off'] = off
            d['n_' + side] = len(w)
            ws.append(np.asarray(w, dtype=float))
            ms.append(np.asarray(m, dtype=float))
            ss.append(np.asarray(s, dtype=float))
            off += len(w)
    return descs, np.concatenate(ws), np.concatenate(ms), np.concatenate(ss)
