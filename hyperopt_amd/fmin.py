"""`fmin`: the driver that calls the algo once per round
(hyperopt/fmin.py:249-387; the call site this package's tpe.suggest plugs
into is fmin.py:201-202).

Each round asks the algo for up to `max_queue_len - queued` new documents
(algo(new_ids, domain, trials, seed) with seed = rstate.randint(2**31 - 1),
the reference's seeding, so an rstate reproduces a run), inserts them, and
evaluates every queued document serially.  An algo that returns no documents
ends the run.  Asynchronous stores (MongoTrials) are out of scope.
"""
import functools
import logging
import os
import sys

import numpy as np

from . import base
from .base import coarse_utcnow
from .space import as_apply, rec_eval

logger = logging.getLogger(__name__)


def generate_trial(tid, space):
    """A queued document for a user-given point (points_to_evaluate)."""
    labels = list(space)
    return {'state': base.JOB_STATE_NEW, 'tid': tid, 'spec': None,
            'result': {'status': base.STATUS_NEW},
            'misc': {'tid': tid, 'cmd': ('domain_attachment', 'FMinIter_Domain'),
                     'workdir': None, 'idxs': {k: [tid] for k in labels},
                     'vals': {k: [space[k]] for k in labels}},
            'exp_key': None, 'owner': None, 'version': 0, 'book_time': None,
            'refresh_time': None}


def generate_trials_to_calculate(points):
    trials = base.Trials()
    trials.insert_trial_docs([generate_trial(t, p) for t, p in enumerate(points)])
    return trials


def fmin_pass_expr_memo_ctrl(f):
    """Mark an objective as taking (expr, memo, ctrl) instead of a point."""
    f.fmin_pass_expr_memo_ctrl = True
    return f


def partial(fn, **kwargs):
    """functools.partial that keeps the fmin_pass_expr_memo_ctrl mark."""
    out = functools.partial(fn, **kwargs)
    if hasattr(fn, 'fmin_pass_expr_memo_ctrl'):
        out.fmin_pass_expr_memo_ctrl = fn.fmin_pass_expr_memo_ctrl
    return out


def _evaluate(domain, trials, doc, catch):
    """Run the objective on one queued document and record the outcome in
    place (state DONE + result, or ERROR + misc.error)."""
    doc['book_time'] = doc['refresh_time'] = coarse_utcnow()
    ctrl = base.Ctrl(trials, current_trial=doc)
    try:
        result = domain.evaluate(base.spec_from_misc(doc['misc']), ctrl)
    except Exception as e:
        logger.info('job exception: %s' % str(e))
        doc['state'] = base.JOB_STATE_ERROR
        doc['misc']['error'] = (str(type(e)), str(e))
        doc['refresh_time'] = coarse_utcnow()
        if not catch:
            raise
        return
    doc['state'] = base.JOB_STATE_DONE
    doc['result'] = result
    doc['refresh_time'] = coarse_utcnow()


class FMinIter(object):
    """One optimisation run over a Trials store (the reference's FMinIter
    API: run / exhaust / iteration / serial_evaluate)."""

    catch_eval_exceptions = False

    def __init__(self, algo, domain, trials, rstate, asynchronous=None, max_queue_len=1,
                 poll_interval_secs=1.0, max_evals=sys.maxsize, verbose=0):
        if (trials.asynchronous if asynchronous is None else asynchronous):
            raise NotImplementedError('asynchronous trial stores (MongoTrials) are not part '
                                      'of this package')
        self.asynchronous = False
        self.algo, self.domain, self.trials, self.rstate = algo, domain, trials, rstate
        self.max_queue_len = max_queue_len
        self.poll_interval_secs = poll_interval_secs
        self.max_evals = max_evals
        self.verbose = verbose

    def _queued(self):
        return self.trials.count_by_state_unsynced(base.JOB_STATE_NEW)

    def serial_evaluate(self, N=-1):
        """Evaluate queued documents (all of them, or the first N)."""
        pending = [d for d in self.trials._dynamic_trials if d['state'] == base.JOB_STATE_NEW]
        if N >= 0:
            pending = pending[:N]
        try:
            for doc in pending:
                _evaluate(self.domain, self.trials, doc, self.catch_eval_exceptions)
        finally:
            self.trials.refresh()

    def block_until_done(self):
        self.serial_evaluate()

    def _ask(self, budget):
        """Fill the queue from the algo, at most `budget` documents; returns
        (documents queued, whether the algo stopped the run)."""
        added = 0
        while added < budget:
            room = min(self.max_queue_len - self._queued(), budget - added)
            if room <= 0:
                break
            ids = self.trials.new_trial_ids(room)
            self.trials.refresh()
            docs = self.algo(ids, self.domain, self.trials, self.rstate.randint(2 ** 31 - 1))
            if len(docs) > len(ids):
                raise AssertionError('algo returned %d documents for %d ids' % (len(docs),
                                                                               len(ids)))
            if not docs:
                return added, True
            self.trials.insert_trial_docs(docs)
            self.trials.refresh()
            added += len(docs)
        return added, False

    def run(self, N, block_until_done=True):
        """Queue and evaluate up to N new documents."""
        done = 0
        while done < N:
            added, stopped = self._ask(N - done)
            done += added
            self.serial_evaluate()
            if stopped:
                break
        if block_until_done:
            self.block_until_done()

    def __iter__(self):
        return self

    def __next__(self):
        self.run(1, block_until_done=self.asynchronous)
        if len(self.trials) >= self.max_evals:
            raise StopIteration()
        return self.trials

    def exhaust(self):
        self.run(self.max_evals - len(self.trials), block_until_done=self.asynchronous)
        self.trials.refresh()
        return self


def fmin(fn, space, algo, max_evals, trials=None, rstate=None, allow_trials_fmin=True,
         pass_expr_memo_ctrl=None, catch_eval_exceptions=False, verbose=0,
         return_argmin=True, points_to_evaluate=None, max_queue_len=1):
    """Minimize fn over space with algo (hyperopt/fmin.py:249-387: same
    arguments, same result -- the argmin labels' values -- and the same
    HYPEROPT_FMIN_SEED default seeding)."""
    if rstate is None:
        seed = os.environ.get('HYPEROPT_FMIN_SEED', '')
        rstate = np.random.RandomState(int(seed) if seed else None)
    if allow_trials_fmin and hasattr(trials, 'fmin'):
        return trials.fmin(fn, space, algo=algo, max_evals=max_evals, rstate=rstate,
                           pass_expr_memo_ctrl=pass_expr_memo_ctrl, verbose=verbose,
                           catch_eval_exceptions=catch_eval_exceptions,
                           return_argmin=return_argmin)
    if trials is None:
        if points_to_evaluate is None:
            trials = base.Trials()
        else:
            if not isinstance(points_to_evaluate, list):
                raise AssertionError('points_to_evaluate must be a list of dicts')
            trials = generate_trials_to_calculate(points_to_evaluate)
    domain = base.Domain(fn, space, pass_expr_memo_ctrl=pass_expr_memo_ctrl)
    driver = FMinIter(algo, domain, trials, rstate=rstate, max_evals=max_evals,
                      max_queue_len=max_queue_len, verbose=verbose)
    driver.catch_eval_exceptions = catch_eval_exceptions
    driver.exhaust()
    return trials.argmin if return_argmin else None


def space_eval(space, hp_assignment):
    """The point of `space` that a label -> value assignment selects
    (hyperopt/fmin.py:390-408)."""
    from . import labels as L
    space = as_apply(space)
    memo = {n: hp_assignment[L.param_label(n)] for n in L.walk(space)
            if n.name == 'hyperopt_param' and L.param_label(n) in hp_assignment}
    return rec_eval(space, memo=memo)
