"""BASELINE config 1 on the HIP path (missing #1): the reference's
own test_fmin.py:24-35 workload -- fmin(lambda x: (x - 3) ** 2,
hp.uniform('x', -5, 5), algo=tpe.suggest, max_evals=100,
rstate=np.random.RandomState(0)), n_EI_candidates = 24.

Every TPE suggestion (the 80 past the 20 startup trials) is checked: the
oracle rebuilds the posterior from the history the call saw (ap_filter_trials
+ adaptive_parzen_normal, tpe.py:404-477, 624-648), re-draws the call's 24
candidates through the sampler entry point (same Philox seed, stream and
round), scores them (GMM1_lpdf, tpe.py:110-172) and takes broadcast_best's
argmax (tpe.py:769-778): the suggested value must be that candidate, bit for
bit.  The wall time of the whole fmin is printed beside the reference's
0.141 s on one CPU core."""
import time

import numpy as np
import pytest

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu


def test_config1_quadratic_fmin_every_suggestion_is_oracle_argmax():
    import hyperopt_amd as H
    from hyperopt_amd import hp, tpe
    from hyperopt_amd.engine import get_engine

    calls = []

    def algo(new_ids, domain, trials, seed):
        docs = [d for d in trials.trials]
        out = tpe.suggest(new_ids, domain, trials, seed)
        calls.append((list(new_ids), seed, docs, out))
        return out

    def fn(x):
        return (x - 3) ** 2

    # warm the engine (context creation is a one-time cost, not fmin's)
    get_engine(0, 'f64')
    t0 = time.perf_counter()
    trials = H.Trials()
    best = H.fmin(fn, hp.uniform('x', -5, 5), algo=algo, max_evals=100, trials=trials,
                  rstate=np.random.RandomState(0))
    wall = time.perf_counter() - t0
    assert len(trials.trials) == 100
    assert abs(best['x'] - 3.0) < 0.5            # test_fmin.py:24-35's own expectation

    eng = get_engine(0, 'f64')
    n_tpe = 0
    for new_ids, seed, docs, out in calls:
        if len(docs) < 20:                        # startup: rand.suggest (tpe.py:869-871)
            continue
        n_tpe += 1
        tids = np.asarray([d['tid'] for d in docs])
        losses = np.asarray([d['result']['loss'] for d in docs], dtype=float)
        o_idxs = np.asarray([d['misc']['idxs']['x'][0] for d in docs])
        o_vals = np.asarray([d['misc']['vals']['x'][0] for d in docs], dtype=float)
        (wb, mb, sb), (wa, ma, sa) = [p[1:4] for p in O.label_posteriors(
            'uniform', dict(low=-5.0, high=5.0), o_idxs, o_vals, tids, losses, 0.25, 1.0)[:2]]
        cand = eng.GMM1(wb, mb, sb, low=-5.0, high=5.0, seed=seed, size=(24,), stream=0,
                        round=new_ids[0])
        lb = O.gmm1_lpdf(cand, wb, mb, sb, low=-5.0, high=5.0)
        la = O.gmm1_lpdf(cand, wa, ma, sa, low=-5.0, high=5.0)
        k = O.broadcast_best_index(lb, la)
        got = out[0]['misc']['vals']['x'][0]
        assert got == cand[k], (new_ids, got, cand[k], k)
    assert n_tpe == 80
    print('config 1: fmin 100 trials (80 TPE suggestions, each the oracle argmax of its 24 '
          'candidates) in %.3f s on the HIP path; reference tpe.suggest on one CPU core: 0.141 s '
          '(BASELINE.md)' % wall)
