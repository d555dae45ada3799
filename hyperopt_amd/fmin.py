"""`fmin` driver (hyperopt/fmin.py): ask the `algo` for new trial docs,
evaluate them serially, repeat until `max_evals`.  The algo protocol is the
reference's: algo(new_ids, domain, trials, seed) -> [trial_doc], seed drawn
as rstate.randint(2**31 - 1) per call (fmin.py:201-202)."""
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
    return {'state': base.JOB_STATE_NEW, 'tid': tid, 'spec': None,
            'result': {'status': 'new'},
            'misc': {'tid': tid, 'cmd': ('domain_attachment', 'FMinIter_Domain'),
                     'workdir': None, 'idxs': {v: [tid] for v in space},
                     'vals': {k: [v] for k, v in space.items()}},
            'exp_key': None, 'owner': None, 'version': 0, 'book_time': None,
            'refresh_time': None}


def generate_trials_to_calculate(points):
    trials = base.Trials()
    trials.insert_trial_docs([generate_trial(tid, x) for tid, x in enumerate(points)])
    return trials


def fmin_pass_expr_memo_ctrl(f):
    f.fmin_pass_expr_memo_ctrl = True
    return f


def partial(fn, **kwargs):
    rval = functools.partial(fn, **kwargs)
    if hasattr(fn, 'fmin_pass_expr_memo_ctrl'):
        rval.fmin_pass_expr_memo_ctrl = fn.fmin_pass_expr_memo_ctrl
    return rval


class FMinIter(object):
    catch_eval_exceptions = False

    def __init__(self, algo, domain, trials, rstate, asynchronous=None, max_queue_len=1,
                 poll_interval_secs=1.0, max_evals=sys.maxsize, verbose=0):
        self.algo = algo
        self.domain = domain
        self.trials = trials
        self.asynchronous = trials.asynchronous if asynchronous is None else asynchronous
        if self.asynchronous:
            raise NotImplementedError('asynchronous trial stores (MongoTrials) are not '
                                      'part of this package')
        self.poll_interval_secs = poll_interval_secs
        self.max_queue_len = max_queue_len
        self.max_evals = max_evals
        self.rstate = rstate

    def serial_evaluate(self, N=-1):
        for trial in self.trials._dynamic_trials:
            if trial['state'] != base.JOB_STATE_NEW:
                continue
            now = coarse_utcnow()
            trial['book_time'] = now
            trial['refresh_time'] = now
            spec = base.spec_from_misc(trial['misc'])
            ctrl = base.Ctrl(self.trials, current_trial=trial)
            try:
                result = self.domain.evaluate(spec, ctrl)
            except Exception as e:
                logger.info('job exception: %s' % str(e))
                trial['state'] = base.JOB_STATE_ERROR
                trial['misc']['error'] = (str(type(e)), str(e))
                trial['refresh_time'] = coarse_utcnow()
                if not self.catch_eval_exceptions:
                    self.trials.refresh()
                    raise
            else:
                trial['state'] = base.JOB_STATE_DONE
                trial['result'] = result
                trial['refresh_time'] = coarse_utcnow()
            N -= 1
            if N == 0:
                break
        self.trials.refresh()

    def block_until_done(self):
        self.serial_evaluate()

    def run(self, N, block_until_done=True):
        trials = self.trials
        n_queued = 0

        def queue_len():
            return trials.count_by_state_unsynced(base.JOB_STATE_NEW)

        stopped = False
        while n_queued < N:
            qlen = queue_len()
            while qlen < self.max_queue_len and n_queued < N:
                n_to_enqueue = min(self.max_queue_len - qlen, N - n_queued)
                new_ids = trials.new_trial_ids(n_to_enqueue)
                trials.refresh()
                new_trials = self.algo(new_ids, self.domain, trials,
                                       self.rstate.randint(2 ** 31 - 1))
                assert len(new_ids) >= len(new_trials)
                if len(new_trials):
                    trials.insert_trial_docs(new_trials)
                    trials.refresh()
                    n_queued += len(new_trials)
                    qlen = queue_len()
                else:
                    stopped = True
                    break
            self.serial_evaluate()
            if stopped:
                break
        if block_until_done:
            self.block_until_done()
            trials.refresh()

    def __iter__(self):
        return self

    def __next__(self):
        self.run(1, block_until_done=self.asynchronous)
        if len(self.trials) >= self.max_evals:
            raise StopIteration()
        return self.trials

    def exhaust(self):
        n_done = len(self.trials)
        self.run(self.max_evals - n_done, block_until_done=self.asynchronous)
        self.trials.refresh()
        return self


def fmin(fn, space, algo, max_evals, trials=None, rstate=None, allow_trials_fmin=True,
         pass_expr_memo_ctrl=None, catch_eval_exceptions=False, verbose=0,
         return_argmin=True, points_to_evaluate=None, max_queue_len=1):
    """Minimize fn over space (fmin.py:249-387, same arguments)."""
    if rstate is None:
        env = os.environ.get('HYPEROPT_FMIN_SEED', '')
        rstate = np.random.RandomState(int(env)) if env else np.random.RandomState()
    if allow_trials_fmin and hasattr(trials, 'fmin'):
        return trials.fmin(fn, space, algo=algo, max_evals=max_evals, rstate=rstate,
                           pass_expr_memo_ctrl=pass_expr_memo_ctrl, verbose=verbose,
                           catch_eval_exceptions=catch_eval_exceptions,
                           return_argmin=return_argmin)
    if trials is None:
        if points_to_evaluate is None:
            trials = base.Trials()
        else:
            assert type(points_to_evaluate) == list
            trials = generate_trials_to_calculate(points_to_evaluate)
    domain = base.Domain(fn, space, pass_expr_memo_ctrl=pass_expr_memo_ctrl)
    it = FMinIter(algo, domain, trials, max_evals=max_evals, rstate=rstate, verbose=verbose,
                  max_queue_len=max_queue_len)
    it.catch_eval_exceptions = catch_eval_exceptions
    it.exhaust()
    if return_argmin:
        return trials.argmin


def space_eval(space, hp_assignment):
    """Point of the space for a hyperparameter assignment (fmin.py:390-408)."""
    from . import labels as L
    space = as_apply(space)
    memo = {}
    for n in L.walk(space):
        if n.name == 'hyperopt_param':
            lab = L.param_label(n)
            if lab in hp_assignment:
                memo[n] = hp_assignment[lab]
    return rec_eval(space, memo=memo)
