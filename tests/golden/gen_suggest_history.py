"""Golden histories from the reference's own fmin(tpe.suggest) runs.

Run in the survey container only:
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_suggest_history.py

For each space it runs the reference fmin with tpe.suggest (some objective
calls fail, so losses are None), then calls the reference tpe.suggest once
more with `ap_filter_trials` instrumented, recording per label the inputs it
receives (observation idxs/vals, history tids/losses) and the split it
returns.  Stored: the trial documents (JSON: tid, state, result, misc) and
those per-label arrays -- data only.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(REPO, 'tools', 'refshim'), '/root/reference']

from hyperopt import Trials, fmin, hp, tpe  # noqa: E402  (reference)
from hyperopt.pyll import scope  # noqa: E402
import hyperopt.tpe as rtpe  # noqa: E402


def many_dists():
    # the 11 kinds of test_domains.py many_dists, as a dict space
    return {'a': hp.choice('a', [0, 1, 2]), 'b': hp.randint('b', 10),
            'c': hp.uniform('c', 4, 7), 'd': hp.loguniform('d', -2, 0),
            'e': hp.quniform('e', 0, 10, 3), 'f': hp.qloguniform('f', 0, 3, 2),
            'g': hp.normal('g', 4, 7), 'h': hp.lognormal('h', -2, 2),
            'i': hp.qnormal('i', 0, 10, 2), 'j': hp.qlognormal('j', 0, 2, 1),
            'k': hp.pchoice('k', [(.1, 0), (.9, 1)])}


def many_dists_loss(d):
    z = sum(float(v) for v in d.values())
    if int(d['b']) == 7:
        return {'status': 'fail'}
    return {'loss': float(np.log(1e-12 + z ** 2)), 'status': 'ok'}


def conditional():
    return {'clf': hp.choice('clf', [
        {'type': 'svm', 'C': hp.loguniform('svm_C', -5, 5),
         'kernel': hp.choice('svm_kernel', [
             {'k': 'rbf', 'gamma': hp.loguniform('svm_gamma', -8, 2)},
             {'k': 'poly', 'degree': hp.quniform('svm_degree', 2, 5, 1)}])},
        {'type': 'rf', 'n': hp.qloguniform('rf_n', np.log(10), np.log(1000), 1),
         'depth': hp.quniform('rf_depth', 1, 30, 1), 'feat': hp.uniform('rf_feat', .1, 1)},
    ]), 'lr': hp.normal('lr', 0, 1)}


def conditional_loss(d):
    c = d['clf']
    if c['type'] == 'svm':
        extra = np.log(c['C']) ** 2 / 10 + (c['kernel'].get('degree', 3) - 3) ** 2
    else:
        extra = (c['depth'] - 12) ** 2 / 50.0 + c['feat']
    return float(extra + (d['lr'] - .3) ** 2)


def capture(space, fn, n, seed, gamma=0.25):
    trials = Trials()
    fmin(fn, space, algo=tpe.suggest, max_evals=n, trials=trials,
         rstate=np.random.RandomState(seed))
    calls = []
    orig = scope._impls['ap_filter_trials']

    def hook(o_idxs, o_vals, l_idxs, l_vals, gamma, gamma_cap=rtpe.DEFAULT_LF):
        out = orig(o_idxs, o_vals, l_idxs, l_vals, gamma, gamma_cap)
        calls.append((list(o_idxs), list(o_vals), list(l_idxs), list(l_vals), out))
        return out
    scope._impls['ap_filter_trials'] = hook
    try:
        from hyperopt.base import Domain
        domain = Domain(fn, space)
        rtpe.suggest([len(trials)], domain, trials, 12345, gamma=gamma)
    finally:
        scope._impls['ap_filter_trials'] = orig
    # identify each call's label by its observation list
    from hyperopt.base import miscs_to_idxs_vals
    docs = sorted(trials.trials, key=lambda d: d['tid'])
    idxs, vals = miscs_to_idxs_vals([d['misc'] for d in docs], keys=list(domain.params))
    per_label = {}
    for label in domain.params:
        matches = [c for c in calls if c[0] == list(idxs[label]) and
                   [float(v) for v in c[1]] == [float(v) for v in vals[label]]]
        if not matches:
            continue
        c = matches[0]
        per_label[label] = dict(o_idxs=np.asarray(c[0], dtype=np.int64),
                                o_vals=np.asarray(c[1], dtype=float),
                                l_idxs=np.asarray(c[2], dtype=np.int64),
                                l_vals=np.asarray(c[3], dtype=float),
                                below=np.asarray(c[4][0], dtype=float),
                                above=np.asarray(c[4][1], dtype=float))
    jdocs = [dict(tid=d['tid'], state=d['state'], result=d['result'],
                  misc=dict(tid=d['misc']['tid'], idxs=d['misc']['idxs'],
                            vals={k: [float(x) for x in v] for k, v in d['misc']['vals'].items()}))
             for d in trials._dynamic_trials]
    return jdocs, per_label


def main():
    out = {}
    arrays = {}
    for name, space, fn, n, seed in (('many_dists', many_dists(), many_dists_loss, 60, 3),
                                     ('conditional', conditional(), conditional_loss, 60, 4)):
        docs, per_label = capture(space, fn, n, seed)
        out[name] = dict(docs=docs, labels=sorted(per_label))
        for label, rec in per_label.items():
            for k, v in rec.items():
                arrays['%s/%s/%s' % (name, label, k)] = v
        print(name, len(docs), 'docs;', len(per_label), 'labels captured')
    arrays['meta'] = np.array(json.dumps(out))
    np.savez_compressed(os.path.join(HERE, 'suggest_history.npz'), **arrays)


if __name__ == '__main__':
    main()
