"""Columnar trial history for `tpe.suggest`.

The reference rebuilds, on every call, the loss of each tid (tpe.py:839-861)
and the per-label (idxs, vals) lists with a Python loop over all docs and all
labels (`miscs_to_idxs_vals`, base.py:192-207) -- O(N x L) Python work per
suggestion.  Here each doc's hyperparameter values are
ingested once into per-label arrays; a suggestion only re-reads the losses
(results change as trials finish) and masks the arrays.

Semantics kept from the reference:
  * group key = misc.get('from_tid', tid); loss None -> +inf; the doc with the
    smallest loss represents its group; a group whose first loss is NaN is
    dropped (`loss <= best` is False for NaN, tpe.py:850-853);
  * docs ordered by group key; observations of a label are the represented
    docs' misc idxs/vals in that order (the idxs stay the doc's own tid, as
    in miscs_to_idxs_vals).
"""
import math
import weakref
from itertools import repeat
from operator import itemgetter

import numpy as np

from .base import Domain

_plain_loss = Domain.loss


class _LabelColumn(object):
    __slots__ = ('tids', 'vals', 'n', 'ptids', 'pvals')

    def __init__(self):
        self.tids, self.vals = [], []
        self.n = 0
        self.ptids = np.zeros(0, dtype=np.int64)
        self.pvals = np.zeros(0, dtype=np.float64)

    def arrays(self):
        if len(self.tids) != self.n:
            self.ptids = np.concatenate([self.ptids, np.asarray(self.tids[self.n:], dtype=np.int64)])
            self.pvals = np.concatenate([self.pvals, np.asarray(self.vals[self.n:], dtype=np.float64)])
            self.n = len(self.tids)
        return self.ptids, self.pvals


class HistoryCache(object):
    def __init__(self, labels):
        self.labels = list(labels)
        self.cols = {k: _LabelColumn() for k in self.labels}
        self.seen = {}          # id(doc) -> doc (keeps ids unique while cached)
        self.n_ingested = 0
        self.last_doc = None
        self.order = []         # ingested docs in order (the fast path's view)
        self.doc_tids = []      # their tids
        self.tid_set = set()
        self.has_from = False   # any doc with misc.from_tid != tid
        self.dup_tid = False
        self._tid_arr = np.zeros(0, dtype=np.int64)

    def ingest(self, docs):
        # fast path: the docs list grew by appending (Trials.refresh keeps the
        # same doc objects in order) -- only the tail is new
        k = self.n_ingested
        if k and len(docs) >= k and docs[k - 1] is self.last_doc and id(docs[k - 1]) in self.seen:
            new = docs[k:]
        else:
            new = docs
        if new is docs:                      # not append-only: rebuild the order view
            self.order, self.doc_tids, self.tid_set = [], [], set()
            self.has_from = self.dup_tid = False
            self._tid_arr = np.zeros(0, dtype=np.int64)
        for d in new:
            m = d['misc']
            t = d['tid']
            self.order.append(d)
            self.doc_tids.append(t)
            if t in self.tid_set:
                self.dup_tid = True
            self.tid_set.add(t)
            if m.get('from_tid', t) != t:
                self.has_from = True
            if id(d) in self.seen:
                continue
            self.seen[id(d)] = d
            idxs, vals = m['idxs'], m['vals']
            for k2 in self.labels:
                ti = idxs.get(k2, [])
                if ti:
                    c = self.cols[k2]
                    c.tids.append(ti[0])
                    c.vals.append(vals[k2][0])
        self.n_ingested = len(docs)
        self.last_doc = docs[-1] if docs else None

    def gather(self, domain, trials):
        """(tids, losses, obs) where obs[label] = (idxs, vals) arrays."""
        docs = trials.trials
        self.ingest(docs)
        raw = raw_losses(domain, docs)
        if not self.has_from and not self.dup_tid and len(self.order) == len(docs):
            return self._gather_own(docs, raw)
        own = [d['tid'] for d in docs]
        keys = [d['misc'].get('from_tid', t) for d, t in zip(docs, own)]
        groups = {}
        any_from = keys != own
        for d, g, loss in zip(docs, keys, raw):
            loss = float('inf') if loss is None else float(loss)
            if g not in groups:
                if loss == loss:                       # NaN never becomes best
                    groups[g] = (loss, d)
                else:
                    groups[g] = (loss, None)
            else:
                best_loss, best = groups[g]
                if loss <= best_loss:
                    groups[g] = (loss, d)
        items = sorted((g, v) for g, v in groups.items() if v[1] is not None)
        tids = np.asarray([g for g, _ in items], dtype=np.int64)
        losses = np.asarray([v[0] for _, v in items], dtype=np.float64)
        rep = [v[1] for _, v in items]
        obs = {}
        if not any_from:
            # each doc is its own group: mask the columns to the represented
            # docs (drops errored / NaN-loss ones) and keep tid order
            every = len(rep) == len(self.seen)
            rep_tids = None if every else np.asarray([d['tid'] for d in rep], dtype=np.int64)
            for k in self.labels:
                ti, tv = self.cols[k].arrays()
                if rep_tids is not None:
                    keep = np.isin(ti, rep_tids)
                    ti, tv = ti[keep], tv[keep]
                if len(ti) > 1 and not np.all(ti[1:] > ti[:-1]):
                    o = np.argsort(ti, kind='stable')
                    ti, tv = ti[o], tv[o]
                obs[k] = (ti, tv)
        else:
            # general case: restrict to represented docs, keep group order
            for k in self.labels:
                ti, tv = [], []
                for d in rep:
                    m = d['misc']
                    x = m['idxs'].get(k, [])
                    if x:
                        ti.append(x[0])
                        tv.append(m['vals'][k][0])
                obs[k] = (np.asarray(ti, dtype=np.int64), np.asarray(tv, dtype=np.float64))
        return tids, losses, obs


    def _gather_own(self, docs, raw):
        """Every doc is its own group (no from_tid, unique tids): vectorised,
        with the tids kept incrementally."""
        n = len(docs)
        if len(self._tid_arr) != n:
            self._tid_arr = np.concatenate([self._tid_arr, np.asarray(
                self.doc_tids[len(self._tid_arr):], dtype=np.int64)])
        tids = self._tid_arr
        if None not in raw:                         # np.array would turn None into NaN
            losses = np.fromiter(raw, dtype=np.float64, count=n)
        else:                                       # pending / failed: +inf (tpe.py:844-847)
            losses = np.array([float('inf') if v is None else float(v) for v in raw],
                              dtype=np.float64)
        if n > 1 and not np.all(tids[1:] > tids[:-1]):
            o = np.argsort(tids, kind='stable')
            tids, losses = tids[o], losses[o]
        keep = losses == losses                     # a NaN loss never becomes best
        every = bool(keep.all()) and n == len(self.seen)
        if not keep.all():
            tids, losses = tids[keep], losses[keep]
        obs = {}
        for k in self.labels:
            ti, tv = self.cols[k].arrays()
            if not every:
                m = np.isin(ti, tids)
                ti, tv = ti[m], tv[m]
            if len(ti) > 1 and not np.all(ti[1:] > ti[:-1]):
                o = np.argsort(ti, kind='stable')
                ti, tv = ti[o], tv[o]
            obs[k] = (ti, tv)
        return tids, losses, obs


    def device_view(self, domain, trials):
        """The whole history as the device-resident store wants it, or None
        when the fast layout does not apply (from_tid groups, duplicate tids,
        docs not in increasing tid order): (tids of ALL docs in order, their
        losses -- None -> +inf, NaN kept, so NaN-loss docs stay out of both
        sets --, the number of non-NaN losses, the append-only per-label
        columns {label: (tids, vals)}, self)."""
        docs = trials.trials
        self.ingest(docs)
        if self.has_from or self.dup_tid or len(self.order) != len(docs):
            return None
        n = len(docs)
        if len(self._tid_arr) != n:
            self._tid_arr = np.concatenate([self._tid_arr, np.asarray(
                self.doc_tids[len(self._tid_arr):], dtype=np.int64)])
        tids = self._tid_arr
        if n > 1 and not np.all(tids[1:] > tids[:-1]):
            return None
        losses = loss_array(domain, docs)
        n_valid = int(np.count_nonzero(losses == losses))
        cols = {k: self.cols[k].arrays() for k in self.labels}
        return tids, losses, n_valid, cols, self


def raw_losses(domain, docs):
    """domain.loss(result, spec) of every doc (tpe.py:843), None kept.  The
    plain Domain.loss is result.get('loss') (base.py): read through C-level
    map()s when every result is a dict -- this loop is most of a
    device-path suggestion's host time at 10k trials."""
    if type(domain).loss is _plain_loss:
        try:
            return list(map(dict.get, map(_result_of, docs), repeat('loss')))
        except TypeError:                      # a result that is not a dict
            return [d['result'].get('loss') for d in docs]
    return [domain.loss(d['result'], d['spec']) for d in docs]


def loss_array(domain, docs):
    """float64 losses of the docs, None -> +inf (tpe.py:844-847): straight
    from the result dicts into the array when every doc has a loss (the
    steady state of fmin's serial loop), else through raw_losses.  (np.fromiter
    turns None into NaN, which would drop a pending trial instead of giving
    it +inf: any NaN sends the docs through the exact path.)"""
    if type(domain).loss is _plain_loss:
        try:
            out = np.fromiter(map(dict.get, map(_result_of, docs), repeat('loss')),
                              dtype=np.float64, count=len(docs))
            if not np.isnan(out).any():
                return out
        except TypeError:                      # a non-dict result
            pass
    raw = raw_losses(domain, docs)
    if None not in raw:
        return np.fromiter(raw, dtype=np.float64, count=len(docs))
    return np.array([float('inf') if v is None else float(v) for v in raw], dtype=np.float64)


_result_of = itemgetter('result')
_caches = weakref.WeakKeyDictionary()


def gather(domain, trials, labels):
    key = tuple(labels)
    try:
        cache = _caches.get(trials)
    except TypeError:            # not weak-referenceable: no caching
        cache = None
    if cache is None or cache.labels != list(key):
        cache = HistoryCache(key)
        try:
            _caches[trials] = cache
        except TypeError:
            pass
    return cache.gather(domain, trials)


def device_view(domain, trials, labels):
    """HistoryCache.device_view through the per-Trials cache."""
    key = tuple(labels)
    try:
        cache = _caches.get(trials)
    except TypeError:
        cache = None
    if cache is None or cache.labels != list(key):
        cache = HistoryCache(key)
        try:
            _caches[trials] = cache
        except TypeError:
            pass
    return cache.device_view(domain, trials)


def isnan(x):
    try:
        return math.isnan(x)
    except TypeError:
        return False
