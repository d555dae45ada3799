"""Trial documents, `Trials`, `Domain`, `Ctrl` -- the reference's data model
(hyperopt/base.py) with the same document schema and method names, so
histories, checkpoints (pickled Trials) and user code carry over.

Trial document (base.py:439-455):
    {state, tid, spec, result{status, loss, ...}, misc{tid, cmd, workdir,
     idxs{label: [tid] or []}, vals{label: [value] or []}}, exp_key, owner,
     version, book_time, refresh_time}
"""
import datetime
import logging

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
STATUS_STRINGS = ('new', 'running', 'suspended', 'ok', 'fail')

JOB_STATE_NEW = 0
JOB_STATE_RUNNING = 1
JOB_STATE_DONE = 2
JOB_STATE_ERROR = 3
JOB_STATES = [JOB_STATE_NEW, JOB_STATE_RUNNING, JOB_STATE_DONE, JOB_STATE_ERROR]

TRIAL_KEYS = ['tid', 'spec', 'result', 'misc', 'state', 'owner', 'book_time',
              'refresh_time', 'exp_key']
TRIAL_MISC_KEYS = ['tid', 'cmd', 'idxs', 'vals']


def coarse_utcnow():
    now = datetime.datetime.utcnow()
    return now.replace(microsecond=(now.microsecond // 1000) * 1000)


def SONify(arg):
    """numpy scalars / arrays -> plain Python (what the reference's BSON
    round-trip produces, base.py:118-158)."""
    if isinstance(arg, np.floating):
        return float(arg)
    if isinstance(arg, (np.integer, np.bool_)):
        return int(arg)
    if isinstance(arg, np.ndarray):
        return SONify(arg.sum()) if arg.ndim == 0 else [SONify(a) for a in arg]
    if isinstance(arg, (list, tuple)):
        return type(arg)(SONify(a) for a in arg)
    if isinstance(arg, dict):
        return dict((SONify(k), SONify(v)) for k, v in arg.items())
    return arg


def miscs_update_idxs_vals(miscs, idxs, vals, assert_all_vals_used=True, idxs_map=None):
    """idxs/vals (label -> lists) into misc dicts (base.py:161-189)."""
    idxs_map = idxs_map or {}
    assert set(idxs.keys()) == set(vals.keys())
    by_tid = {m['tid']: m for m in miscs}
    for m in miscs:
        m['idxs'] = {k: [] for k in idxs}
        m['vals'] = {k: [] for k in idxs}
    for key in idxs:
        assert len(idxs[key]) == len(vals[key])
        for tid, val in zip(idxs[key], vals[key]):
            tid = idxs_map.get(tid, tid)
            if assert_all_vals_used or tid in by_tid:
                by_tid[tid]['idxs'][key] = [tid]
                by_tid[tid]['vals'][key] = [val]
    return miscs


def miscs_to_idxs_vals(miscs, keys=None):
    """misc dicts -> idxs/vals (label -> lists) (base.py:192-207)."""
    if keys is None:
        if not miscs:
            raise ValueError('cannot infer keys from empty miscs')
        keys = list(miscs[0]['idxs'].keys())
    idxs = {k: [] for k in keys}
    vals = {k: [] for k in keys}
    for m in miscs:
        for k in keys:
            ti, tv = m['idxs'][k], m['vals'][k]
            assert len(ti) == len(tv)
            idxs[k].extend(ti)
            vals[k].extend(tv)
    return idxs, vals


def spec_from_misc(misc):
    spec = {}
    for k, v in misc['vals'].items():
        if len(v) == 1:
            spec[k] = v[0]
        elif len(v) > 1:
            raise NotImplementedError('multiple values', (k, v))
    return spec


class Trials(object):
    """In-memory trial database (base.py:222-635)."""

    asynchronous = False

    def __init__(self, exp_key=None, refresh=True):
        self._ids = set()
        self._dynamic_trials = []
        self._exp_key = exp_key
        self.attachments = {}
        if refresh:
            self.refresh()

    def view(self, exp_key=None, refresh=True):
        rval = object.__new__(self.__class__)
        rval._exp_key = exp_key
        rval._ids = self._ids
        rval._dynamic_trials = self._dynamic_trials
        rval.attachments = self.attachments
        if refresh:
            rval.refresh()
        return rval

    def aname(self, trial, name):
        return 'ATTACH::%s::%s' % (trial['tid'], name)

    def trial_attachments(self, trial):
        trials = self

        class Attachments(object):
            def __contains__(_, name):
                return trials.aname(trial, name) in trials.attachments

            def __getitem__(_, name):
                return trials.attachments[trials.aname(trial, name)]

            def __setitem__(_, name, value):
                trials.attachments[trials.aname(trial, name)] = value

            def __delitem__(_, name):
                del trials.attachments[trials.aname(trial, name)]
        return Attachments()

    def __iter__(self):
        return iter(self._trials)

    def __len__(self):
        return len(self._trials)

    def __getitem__(self, item):
        raise NotImplementedError('')

    def refresh(self):
        if self._exp_key is None:
            self._trials = [t for t in self._dynamic_trials if t['state'] != JOB_STATE_ERROR]
        else:
            self._trials = [t for t in self._dynamic_trials
                            if t['state'] != JOB_STATE_ERROR and t['exp_key'] == self._exp_key]
        self._ids.update(t['tid'] for t in self._trials)

    @property
    def trials(self):
        return self._trials

    @property
    def tids(self):
        return [t['tid'] for t in self._trials]

    @property
    def specs(self):
        return [t['spec'] for t in self._trials]

    @property
    def results(self):
        return [t['result'] for t in self._trials]

    @property
    def miscs(self):
        return [t['misc'] for t in self._trials]

    @property
    def idxs_vals(self):
        return miscs_to_idxs_vals(self.miscs)

    @property
    def idxs(self):
        return self.idxs_vals[0]

    @property
    def vals(self):
        return self.idxs_vals[1]

    def assert_valid_trial(self, trial):
        if not (hasattr(trial, 'keys') and hasattr(trial, 'values')):
            raise InvalidTrial('trial should be dict-like', trial)
        for key in TRIAL_KEYS:
            if key not in trial:
                raise InvalidTrial('trial missing key %s' % key, key)
        for key in TRIAL_MISC_KEYS:
            if key not in trial['misc']:
                raise InvalidTrial('trial["misc"] missing key', key)
        if trial['tid'] != trial['misc']['tid']:
            raise InvalidTrial('tid mismatch between root and misc', trial)
        if trial['exp_key'] != self._exp_key:
            raise InvalidTrial('wrong exp_key', (trial['exp_key'], self._exp_key))
        return trial

    def _insert_trial_docs(self, docs):
        rval = [d['tid'] for d in docs]
        self._dynamic_trials.extend(docs)
        return rval

    def insert_trial_doc(self, doc):
        doc = self.assert_valid_trial(SONify(doc))
        return self._insert_trial_docs([doc])[0]

    def insert_trial_docs(self, docs):
        docs = [self.assert_valid_trial(SONify(d)) for d in docs]
        return self._insert_trial_docs(docs)

    def new_trial_ids(self, N):
        aa = len(self._ids)
        rval = list(range(aa, aa + N))
        self._ids.update(rval)
        return rval

    def new_trial_docs(self, tids, specs, results, miscs):
        assert len(tids) == len(specs) == len(results) == len(miscs)
        rval = []
        for tid, spec, result, misc in zip(tids, specs, results, miscs):
            rval.append(dict(state=JOB_STATE_NEW, tid=tid, spec=spec, result=result,
                             misc=misc, exp_key=self._exp_key, owner=None, version=0,
                             book_time=None, refresh_time=None))
        return rval

    def source_trial_docs(self, tids, specs, results, miscs, sources):
        rval = []
        for tid, spec, result, misc, src in zip(tids, specs, results, miscs, sources):
            doc = dict(version=0, tid=tid, spec=spec, result=result, misc=misc,
                       state=src['state'], exp_key=src['exp_key'], owner=src['owner'],
                       book_time=src['book_time'], refresh_time=src['refresh_time'])
            for k, v in (('tid', tid), ('cmd', None), ('from_tid', src['tid'])):
                assert doc['misc'].setdefault(k, v) == v
            rval.append(doc)
        return rval

    def delete_all(self):
        self._dynamic_trials = []
        self.attachments = {}
        self.refresh()

    def count_by_state_synced(self, arg, trials=None):
        trials = self._trials if trials is None else trials
        if arg in JOB_STATES:
            return sum(1 for d in trials if d['state'] == arg)
        if hasattr(arg, '__iter__'):
            states = set(arg)
            return sum(1 for d in trials if d['state'] in states)
        raise TypeError(arg)

    def count_by_state_unsynced(self, arg):
        if self._exp_key is not None:
            exp = [t for t in self._dynamic_trials if t['exp_key'] == self._exp_key]
        else:
            exp = self._dynamic_trials
        return self.count_by_state_synced(arg, trials=exp)

    def losses(self, bandit=None):
        if bandit is None:
            return [r.get('loss') for r in self.results]
        return [bandit.loss(r, s) for r, s in zip(self.results, self.specs)]

    def statuses(self, bandit=None):
        if bandit is None:
            return [r.get('status') for r in self.results]
        return [bandit.status(r, s) for r, s in zip(self.results, self.specs)]

    def average_best_error(self, bandit=None):
        """Loss of the best trial when loss variances are zero (base.py:509-558
        without the pmin_sampled branch for noisy losses)."""
        results = self.results
        ok = [r for r in results if r['status'] == STATUS_OK]
        if not ok:
            raise ValueError('Empty loss vector')
        if bandit is not None:
            loss = [bandit.loss(r) for r in ok]
            true = [bandit.true_loss(r) for r in ok]
        else:
            loss = [r['loss'] for r in ok]
            true = [r.get('true_loss', r['loss']) for r in ok]
        return true[int(np.argmin(loss))]

    @property
    def best_trial(self):
        cands = [t for t in self.trials if t['result']['status'] == STATUS_OK]
        losses = [float(t['result']['loss']) for t in cands]
        if not cands:
            from .exceptions import AllTrialsFailed
            raise AllTrialsFailed
        assert not np.any(np.isnan(losses))
        return cands[int(np.argmin(losses))]

    @property
    def argmin(self):
        vals = self.best_trial['misc']['vals']
        return {k: v[0] for k, v in vals.items() if v}

    def fmin(self, fn, space, algo, max_evals, rstate=None, verbose=0,
             pass_expr_memo_ctrl=None, catch_eval_exceptions=False, return_argmin=True):
        from .fmin import fmin
        return fmin(fn, space, algo, max_evals, trials=self, rstate=rstate, verbose=verbose,
                    allow_trials_fmin=False, pass_expr_memo_ctrl=pass_expr_memo_ctrl,
                    catch_eval_exceptions=catch_eval_exceptions, return_argmin=return_argmin)


def trials_from_docs(docs, validate=True, **kwargs):
    rval = Trials(**kwargs)
    if validate:
        rval.insert_trial_docs(docs)
    else:
        rval._insert_trial_docs(docs)
    rval.refresh()
    return rval


class Ctrl(object):
    """Channel between an evaluation and the Trials store (base.py:650-705)."""
    info = logger.info
    warn = logger.warning
    error = logger.error
    debug = logger.debug

    def __init__(self, trials, current_trial=None):
        self.trials = Trials() if trials is None else trials
        self.current_trial = current_trial

    def checkpoint(self, r=None):
        assert self.current_trial in self.trials._trials
        if r is not None:
            self.current_trial['result'] = r

    @property
    def attachments(self):
        return self.trials.trial_attachments(trial=self.current_trial)

    def inject_results(self, specs, results, miscs, new_tids=None):
        trial = self.current_trial
        assert trial is not None
        assert len(specs) == len(results) == len(miscs)
        if new_tids is None:
            new_tids = self.trials.new_trial_ids(len(specs))
        new = self.trials.source_trial_docs(tids=new_tids, specs=specs, results=results,
                                            miscs=miscs, sources=[trial])
        for t in new:
            t['state'] = JOB_STATE_DONE
        return self.trials.insert_trial_docs(new)


class Domain(object):
    """Search space + objective (base.py:708-952)."""

    rec_eval_print_node_on_error = False

    def __init__(self, fn, expr, workdir=None, pass_expr_memo_ctrl=None, name=None,
                 loss_target=None):
        self.fn = fn
        if pass_expr_memo_ctrl is None:
            self.pass_expr_memo_ctrl = getattr(fn, 'fmin_pass_expr_memo_ctrl', False)
        else:
            self.pass_expr_memo_ctrl = pass_expr_memo_ctrl
        self.expr = as_apply(expr)
        self.specs = _labels.compile_space(self.expr)    # raises DuplicateLabel
        self.params = {k: s.dist for k, s in self.specs.items()}
        self.loss_target = loss_target
        self.name = name
        self.workdir = workdir
        self.cmd = ('domain_attachment', 'FMinIter_Domain')

    def memo_from_config(self, config):
        from .space import MISSING
        memo = {}
        for s in self.specs.values():
            memo[s.param] = config.get(s.label, MISSING)
        return memo

    def evaluate(self, config, ctrl, attach_attachments=True):
        memo = self.memo_from_config(config)
        if self.pass_expr_memo_ctrl:
            rval = self.fn(expr=self.expr, memo=memo, ctrl=ctrl)
        else:
            rval = self.fn(rec_eval(self.expr, memo=memo))
        return self._result_dict(rval, ctrl, attach_attachments)

    def _result_dict(self, rval, ctrl, attach_attachments):
        if isinstance(rval, (float, int, np.number)):
            d = {'loss': float(rval), 'status': STATUS_OK}
        else:
            d = dict(rval)
            status = d['status']
            if status not in STATUS_STRINGS:
                raise InvalidResultStatus(d)
            if status == STATUS_OK:
                try:
                    d['loss'] = float(d['loss'])
                except (TypeError, KeyError):
                    raise InvalidLoss(d)
        if attach_attachments:
            for k, v in d.pop('attachments', {}).items():
                ctrl.attachments[k] = v
        return d

    def short_str(self):
        return 'Domain{%s}' % str(self.fn)

    def loss(self, result, config=None):
        return result.get('loss', None)

    def loss_variance(self, result, config=None):
        return result.get('loss_variance', 0.0)

    def true_loss(self, result, config=None):
        try:
            return result['true_loss']
        except KeyError:
            return self.loss(result, config=config)

    def status(self, result, config=None):
        return result['status']

    def new_result(self):
        return {'status': STATUS_NEW}
