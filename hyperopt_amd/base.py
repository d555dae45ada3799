"""Trial store, search domain and evaluation channel with hyperopt's public
names (`Trials`, `Domain`, `Ctrl`, the STATUS_* / JOB_STATE_* constants,
`miscs_to_idxs_vals` ...) and its trial-document schema, so histories,
pickled Trials and user code carry over.  The implementation is this
package's: a `Trials` is an append-only document log with a tid index and a
cached filtered view, validated against one schema table; `Domain` compiles
the space once into the flat label table the GPU engine uses.

Trial document (hyperopt/base.py:439-455):
    {state, tid, spec, result{status, loss, ...}, misc{tid, cmd, workdir,
     idxs{label: [tid] or []}, vals{label: [value] or []}[, from_tid]},
     exp_key, owner, version, book_time, refresh_time}
"""
import datetime
import logging
from collections.abc import MutableMapping

import numpy as np

from .exceptions import (DuplicateLabel, InvalidLoss, InvalidResultStatus,  # noqa: F401
                         InvalidTrial)
from . import labels as _labels
from .space import as_apply, rec_eval

logger = logging.getLogger(__name__)

STATUS_NEW = 'new'
STATUS_RUNNING = 'running'
STATUS_SUSPENDED = 'suspended'
STATUS_OK = 'ok'
STATUS_FAIL = 'fail'
STATUS_STRINGS = (STATUS_NEW, STATUS_RUNNING, STATUS_SUSPENDED, STATUS_OK, STATUS_FAIL)

JOB_STATE_NEW, JOB_STATE_RUNNING, JOB_STATE_DONE, JOB_STATE_ERROR = range(4)
JOB_STATES = [JOB_STATE_NEW, JOB_STATE_RUNNING, JOB_STATE_DONE, JOB_STATE_ERROR]

# the schema: keys every document / its misc must carry
TRIAL_KEYS = ['tid', 'spec', 'result', 'misc', 'state', 'owner', 'book_time',
              'refresh_time', 'exp_key']
TRIAL_MISC_KEYS = ['tid', 'cmd', 'idxs', 'vals']


def coarse_utcnow():
    """UTC now at millisecond resolution (what a BSON round trip keeps)."""
    now = datetime.datetime.utcnow()
    return now.replace(microsecond=now.microsecond - now.microsecond % 1000)


def SONify(arg):
    """Plain-Python copy of numpy scalars / arrays inside documents (the
    form the reference's BSON round trip produces)."""
    if isinstance(arg, dict):
        return {SONify(k): SONify(v) for k, v in arg.items()}
    if isinstance(arg, (list, tuple)):
        return type(arg)(map(SONify, arg))
    if isinstance(arg, np.ndarray):
        return SONify(arg.sum()) if arg.ndim == 0 else [SONify(a) for a in arg]
    if isinstance(arg, np.floating):
        return float(arg)
    if isinstance(arg, (np.integer, np.bool_)):
        return int(arg)
    return arg


# -- misc codecs: per-label (idxs, vals) <-> per-trial misc dicts -----------

def miscs_update_idxs_vals(miscs, idxs, vals, assert_all_vals_used=True, idxs_map=None):
    """Write label -> [tid...] / [value...] columns into the misc dicts of
    their trials (hyperopt/base.py:161-189).  Every misc gets an entry for
    every label (empty when the label is inactive); idxs_map renames tids
    (suggest's fake ids); a value for an unknown tid is an error unless
    assert_all_vals_used is False."""
    if set(idxs) != set(vals):
        raise AssertionError('idxs and vals name different labels')
    rename = idxs_map or {}
    target = {m['tid']: m for m in miscs}
    for m in miscs:
        m['idxs'] = {label: [] for label in idxs}
        m['vals'] = {label: [] for label in idxs}
    for label, col_tids in idxs.items():
        col_vals = vals[label]
        if len(col_tids) != len(col_vals):
            raise AssertionError('label %r: %d idxs for %d vals' % (label, len(col_tids),
                                                                   len(col_vals)))
        for raw_tid, value in zip(col_tids, col_vals):
            tid = rename.get(raw_tid, raw_tid)
            m = target.get(tid)
            if m is None:
                if assert_all_vals_used:
                    raise KeyError(tid)
                continue
            m['idxs'][label] = [tid]
            m['vals'][label] = [value]
    return miscs


def miscs_to_idxs_vals(miscs, keys=None):
    """The inverse: label -> (tids, values) columns over the misc dicts, in
    trial order (hyperopt/base.py:192-207)."""
    if keys is None:
        if not miscs:
            raise ValueError('cannot infer keys from empty miscs')
        keys = list(miscs[0]['idxs'])
    cols = {k: ([], []) for k in keys}
    for m in miscs:
        mi, mv = m['idxs'], m['vals']
        for k, (ti, tv) in cols.items():
            a, b = mi[k], mv[k]
            if len(a) != len(b):
                raise AssertionError('label %r: misc idxs/vals lengths differ' % (k,))
            ti += a
            tv += b
    return {k: c[0] for k, c in cols.items()}, {k: c[1] for k, c in cols.items()}


def spec_from_misc(misc):
    """label -> value of one trial's active labels."""
    out = {}
    for label, v in misc['vals'].items():
        if len(v) > 1:
            raise NotImplementedError('multiple values', (label, v))
        if v:
            out[label] = v[0]
    return out


def validate_trial(trial, exp_key):
    """The schema check of Trials.assert_valid_trial (hyperopt/base.py:
    439-470): InvalidTrial for a malformed document."""
    if not (hasattr(trial, 'keys') and hasattr(trial, 'values')):
        raise InvalidTrial('trial should be dict-like', trial)
    missing = [k for k in TRIAL_KEYS if k not in trial]
    if missing:
        raise InvalidTrial('trial missing key %s' % missing[0], missing[0])
    missing = [k for k in TRIAL_MISC_KEYS if k not in trial['misc']]
    if missing:
        raise InvalidTrial('trial["misc"] missing key', missing[0])
    if trial['tid'] != trial['misc']['tid']:
        raise InvalidTrial('tid mismatch between root and misc', trial)
    if trial['exp_key'] != exp_key:
        raise InvalidTrial('wrong exp_key', (trial['exp_key'], exp_key))
    return trial


class TrialAttachments(MutableMapping):
    """Per-trial view of a Trials' attachment blob store (keys are
    'ATTACH::<tid>::<name>' in the shared dict)."""

    def __init__(self, trials, trial):
        self._store, self._prefix = trials.attachments, 'ATTACH::%s::' % trial['tid']

    def __getitem__(self, name):
        return self._store[self._prefix + name]

    def __setitem__(self, name, value):
        self._store[self._prefix + name] = value

    def __delitem__(self, name):
        del self._store[self._prefix + name]

    def __iter__(self):
        n = len(self._prefix)
        return (k[n:] for k in list(self._store) if k.startswith(self._prefix))

    def __len__(self):
        return sum(1 for _ in self)


class Trials(object):
    """In-memory trial store (the reference's Trials API).

    `_dynamic_trials` is the append-only log of every inserted document;
    `trials` is the cached view of the documents of this exp_key that did
    not error, rebuilt by refresh().  Trial ids are allocated by
    new_trial_ids and never reused."""

    asynchronous = False

    def __init__(self, exp_key=None, refresh=True):
        self._dynamic_trials = []
        self._ids = set()
        self._exp_key = exp_key
        self.attachments = {}
        self._trials = []
        if refresh:
            self.refresh()

    # -- views ----------------------------------------------------------------
    def view(self, exp_key=None, refresh=True):
        """Another Trials over the same log and attachments, filtered by
        exp_key."""
        other = object.__new__(type(self))
        other.__dict__.update(self.__dict__)
        other._exp_key = exp_key
        other._trials = []
        if refresh:
            other.refresh()
        return other

    def _visible(self, doc):
        return doc['state'] != JOB_STATE_ERROR and (self._exp_key is None or
                                                    doc['exp_key'] == self._exp_key)

    def refresh(self):
        self._trials = [d for d in self._dynamic_trials if self._visible(d)]
        self._ids.update(d['tid'] for d in self._trials)

    def __iter__(self):
        return iter(self._trials)

    def __len__(self):
        return len(self._trials)

    def __getitem__(self, item):
        raise NotImplementedError('index a Trials through .trials')

    @property
    def trials(self):
        return self._trials

    def _column(self, key):
        return [d[key] for d in self._trials]

    tids = property(lambda self: self._column('tid'))
    specs = property(lambda self: self._column('spec'))
    results = property(lambda self: self._column('result'))
    miscs = property(lambda self: self._column('misc'))

    @property
    def idxs_vals(self):
        return miscs_to_idxs_vals(self.miscs)

    @property
    def idxs(self):
        return self.idxs_vals[0]

    @property
    def vals(self):
        return self.idxs_vals[1]

    def aname(self, trial, name):
        return 'ATTACH::%s::%s' % (trial['tid'], name)

    def trial_attachments(self, trial):
        return TrialAttachments(self, trial)

    # -- inserting --------------------------------------------------------------
    def assert_valid_trial(self, trial):
        return validate_trial(trial, self._exp_key)

    def _insert_trial_docs(self, docs):
        self._dynamic_trials.extend(docs)
        return [d['tid'] for d in docs]

    def insert_trial_doc(self, doc):
        return self.insert_trial_docs([doc])[0]

    def insert_trial_docs(self, docs):
        return self._insert_trial_docs([self.assert_valid_trial(SONify(d)) for d in docs])

    def new_trial_ids(self, N):
        first = len(self._ids)
        fresh = list(range(first, first + N))
        self._ids.update(fresh)
        return fresh

    def new_trial_docs(self, tids, specs, results, miscs):
        if not len(tids) == len(specs) == len(results) == len(miscs):
            raise AssertionError('tids, specs, results and miscs differ in length')
        return [{'state': JOB_STATE_NEW, 'tid': t, 'spec': sp, 'result': r, 'misc': m,
                 'exp_key': self._exp_key, 'owner': None, 'version': 0, 'book_time': None,
                 'refresh_time': None}
                for t, sp, r, m in zip(tids, specs, results, miscs)]

    def source_trial_docs(self, tids, specs, results, miscs, sources):
        """Documents derived from existing ones (Ctrl.inject_results): state,
        owner and times copied from the source, misc.from_tid set to it."""
        docs = []
        for t, sp, r, m, src in zip(tids, specs, results, miscs, sources):
            for k, v in (('tid', t), ('cmd', None), ('from_tid', src['tid'])):
                if m.setdefault(k, v) != v:
                    raise AssertionError('misc[%r] = %r, expected %r' % (k, m[k], v))
            docs.append({'version': 0, 'tid': t, 'spec': sp, 'result': r, 'misc': m,
                         'state': src['state'], 'exp_key': src['exp_key'], 'owner': src['owner'],
                         'book_time': src['book_time'], 'refresh_time': src['refresh_time']})
        return docs

    def delete_all(self):
        self._dynamic_trials = []
        self.attachments = {}
        self.refresh()

    # -- queries ------------------------------------------------------------------
    def count_by_state_synced(self, arg, trials=None):
        docs = self._trials if trials is None else trials
        if arg in JOB_STATES:
            wanted = {arg}
        elif hasattr(arg, '__iter__'):
            wanted = set(arg)
        else:
            raise TypeError(arg)
        return sum(d['state'] in wanted for d in docs)

    def count_by_state_unsynced(self, arg):
        docs = [d for d in self._dynamic_trials
                if self._exp_key is None or d['exp_key'] == self._exp_key]
        return self.count_by_state_synced(arg, trials=docs)

    def losses(self, bandit=None):
        if bandit is None:
            return [r.get('loss') for r in self.results]
        return list(map(bandit.loss, self.results, self.specs))

    def statuses(self, bandit=None):
        if bandit is None:
            return [r.get('status') for r in self.results]
        return list(map(bandit.status, self.results, self.specs))

    def average_best_error(self, bandit=None):
        """True loss of the best successful trial (the zero-variance case of
        hyperopt/base.py:509-558)."""
        ok = [r for r in self.results if r['status'] == STATUS_OK]
        if not ok:
            raise ValueError('Empty loss vector')
        if bandit is None:
            loss = np.asarray([r['loss'] for r in ok], dtype=float)
            true = [r.get('true_loss', r['loss']) for r in ok]
        else:
            loss = np.asarray([bandit.loss(r) for r in ok], dtype=float)
            true = [bandit.true_loss(r) for r in ok]
        return true[int(np.argmin(loss))]

    @property
    def best_trial(self):
        ok = [d for d in self._trials if d['result']['status'] == STATUS_OK]
        if not ok:
            from .exceptions import AllTrialsFailed
            raise AllTrialsFailed
        loss = np.asarray([float(d['result']['loss']) for d in ok])
        if np.isnan(loss).any():
            raise AssertionError('NaN loss among the successful trials')
        return ok[int(np.argmin(loss))]

    @property
    def argmin(self):
        return spec_from_misc(self.best_trial['misc'])

    def fmin(self, fn, space, algo, max_evals, rstate=None, verbose=0,
             pass_expr_memo_ctrl=None, catch_eval_exceptions=False, return_argmin=True):
        from .fmin import fmin
        return fmin(fn, space, algo, max_evals, trials=self, rstate=rstate, verbose=verbose,
                    allow_trials_fmin=False, pass_expr_memo_ctrl=pass_expr_memo_ctrl,
                    catch_eval_exceptions=catch_eval_exceptions, return_argmin=return_argmin)


def trials_from_docs(docs, validate=True, **kwargs):
    """A Trials holding the given documents."""
    out = Trials(**kwargs)
    (out.insert_trial_docs if validate else out._insert_trial_docs)(docs)
    out.refresh()
    return out


class Ctrl(object):
    """What an objective with fmin_pass_expr_memo_ctrl receives: the trial
    being evaluated, its store, logging (hyperopt/base.py:650-705)."""
    info = staticmethod(logger.info)
    warn = staticmethod(logger.warning)
    error = staticmethod(logger.error)
    debug = staticmethod(logger.debug)

    def __init__(self, trials, current_trial=None):
        self.trials = trials if trials is not None else Trials()
        self.current_trial = current_trial

    def checkpoint(self, r=None):
        if not any(d is self.current_trial for d in self.trials._trials):
            raise AssertionError('checkpoint of a trial that is not in the store')
        if r is not None:
            self.current_trial['result'] = r

    @property
    def attachments(self):
        return self.trials.trial_attachments(trial=self.current_trial)

    def inject_results(self, specs, results, miscs, new_tids=None):
        """Insert finished trials derived from the current one."""
        if self.current_trial is None:
            raise AssertionError('inject_results needs a current trial')
        if not len(specs) == len(results) == len(miscs):
            raise AssertionError('specs, results and miscs differ in length')
        tids = self.trials.new_trial_ids(len(specs)) if new_tids is None else new_tids
        docs = self.trials.source_trial_docs(tids=tids, specs=specs, results=results,
                                             miscs=miscs, sources=[self.current_trial])
        for d in docs:
            d['state'] = JOB_STATE_DONE
        return self.trials.insert_trial_docs(docs)


class Domain(object):
    """Objective + search space (the reference's Domain API).  The space is
    compiled once into the flat label table (labels.compile_space, which
    raises DuplicateLabel) that tpe.suggest hands to the GPU engine."""

    rec_eval_print_node_on_error = False

    def __init__(self, fn, expr, workdir=None, pass_expr_memo_ctrl=None, name=None,
                 loss_target=None):
        self.fn = fn
        self.pass_expr_memo_ctrl = (getattr(fn, 'fmin_pass_expr_memo_ctrl', False)
                                    if pass_expr_memo_ctrl is None else pass_expr_memo_ctrl)
        self.expr = as_apply(expr)
        self.specs = _labels.compile_space(self.expr)
        self.params = {label: s.dist for label, s in self.specs.items()}
        self.loss_target = loss_target
        self.name = name
        self.workdir = workdir
        self.cmd = ('domain_attachment', 'FMinIter_Domain')

    def memo_from_config(self, config):
        from .space import MISSING
        return {s.param: config.get(s.label, MISSING) for s in self.specs.values()}

    def evaluate(self, config, ctrl, attach_attachments=True):
        memo = self.memo_from_config(config)
        if self.pass_expr_memo_ctrl:
            out = self.fn(expr=self.expr, memo=memo, ctrl=ctrl)
        else:
            out = self.fn(rec_eval(self.expr, memo=memo))
        result = self._as_result(out)
        if attach_attachments:
            blobs = result.pop('attachments', {})
            for name, blob in blobs.items():
                ctrl.attachments[name] = blob
        return result

    @staticmethod
    def _as_result(out):
        """A number is a successful loss; a dict must carry a known status
        and, when ok, a float loss (InvalidResultStatus / InvalidLoss)."""
        if isinstance(out, (float, int, np.number)):
            return {'loss': float(out), 'status': STATUS_OK}
        result = dict(out)
        if result['status'] not in STATUS_STRINGS:
            raise InvalidResultStatus(result)
        if result['status'] == STATUS_OK:
            try:
                result['loss'] = float(result['loss'])
            except (TypeError, KeyError):
                raise InvalidLoss(result)
        return result

    def short_str(self):
        return 'Domain{%s}' % str(self.fn)

    def loss(self, result, config=None):
        return result.get('loss', None)

    def loss_variance(self, result, config=None):
        return result.get('loss_variance', 0.0)

    def true_loss(self, result, config=None):
        return result['true_loss'] if 'true_loss' in result else self.loss(result, config)

    def status(self, result, config=None):
        return result['status']

    def new_result(self):
        return {'status': STATUS_NEW}
