"""Pass rates of the reference's TestOpt protocol over many seeds.

Run in the survey container only (needs /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_testopt_rates.py

For each benchmark domain of hyperopt/tests/test_tpe.py:544-656 (same
thresholds, lengths, gammas, prior weights and n_EI_candidates) the
reference's own fmin(tpe.suggest) runs from RandomState(seed) for seeds
0..N-1 under np.seterr('raise', under='ignore'); the fixture stores each
run's best loss.  tests/test_tpe_gpu.py holds the GPU engine to the
reference's pass rate on the same seeds (the draws differ: the reference
uses MT19937 through its graph interpreter, the engine Philox).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(REPO, 'tools', 'refshim'), '/root/reference']

from functools import partial  # noqa: E402

from hyperopt import Trials, fmin, tpe  # noqa: E402  (reference)
from hyperopt.tests import test_domains as TD  # noqa: E402  (reference)
from hyperopt.tests.test_tpe import TestOpt  # noqa: E402  (reference)

N_SEEDS = int(os.environ.get('N_SEEDS', '20'))
# a subset of the domains (comma-separated) into its own fixture, e.g.
#   N_SEEDS=100 DOMAINS=branin OUT=testopt_reference_branin100.json
DOMAINS = [d for d in os.environ.get('DOMAINS', '').split(',') if d]
OUT = os.environ.get('OUT', 'testopt_reference_rates.json')


def passthrough(x):
    return x


def main():
    out = {'n_seeds': N_SEEDS, 'thresholds': TestOpt.thresholds, 'best': {}}
    olderr = np.seterr('raise')
    np.seterr(under='ignore')
    try:
        for name in sorted(DOMAINS or TestOpt.thresholds):
            bandit = getattr(TD, name)()
            algo = partial(tpe.suggest,
                           gamma=TestOpt.gammas.get(name, tpe._default_gamma),
                           prior_weight=TestOpt.prior_weights.get(name, tpe._default_prior_weight),
                           n_EI_candidates=TestOpt.n_EIs.get(name, tpe._default_n_EI_candidates))
            n = TestOpt.LEN.get(name, 50)
            best = []
            for seed in range(N_SEEDS):
                trials = Trials()
                fmin(passthrough, space=bandit.expr, algo=algo, trials=trials, max_evals=n,
                     rstate=np.random.RandomState(seed), catch_eval_exceptions=False)
                best.append(float(min(trials.losses())))
            out['best'][name] = best
            rate = np.mean(np.asarray(best) < TestOpt.thresholds[name])
            print('%-14s pass rate %.2f' % (name, rate), flush=True)
    finally:
        np.seterr(**olderr)
    with open(os.path.join(HERE, OUT), 'w') as f:
        json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
