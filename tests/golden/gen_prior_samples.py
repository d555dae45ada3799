"""Prior draws of the reference's random search (rand.suggest, rand.py:15-31,
which evaluates pyll/stochastic.py:35-147 through the graph interpreter).

Run in the survey container only (needs /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_prior_samples.py

Space: every hp kind (test_domains.py many_dists' 11 kinds, as in
gen_suggest_history.py) plus a conditional choice; 4000 documents from
rand.suggest with seed 0.  Stored: per label the drawn values (NaN where the
label was inactive) -- data only.  tests/test_prior.py checks this package's
rand.suggest against them distribution-wise (the draw order differs).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(REPO, 'tools', 'refshim'), '/root/reference']

from hyperopt import Trials, hp, rand  # noqa: E402  (reference)
from hyperopt.base import Domain  # noqa: E402  (reference)

N = 4000


def space():
    return {'a': hp.choice('a', [0, 1, 2]), 'b': hp.randint('b', 10),
            'c': hp.uniform('c', 4, 7), 'd': hp.loguniform('d', -2, 0),
            'e': hp.quniform('e', 0, 10, 3), 'f': hp.qloguniform('f', 0, 3, 2),
            'g': hp.normal('g', 4, 7), 'h': hp.lognormal('h', -2, 2),
            'i': hp.qnormal('i', 0, 10, 2), 'j': hp.qlognormal('j', 0, 2, 1),
            'k': hp.pchoice('k', [(.1, 0), (.9, 1)]),
            'm': hp.choice('m', [{'u': hp.uniform('u', 0, 1)}, {'v': hp.normal('v', 0, 1)}])}


def main():
    dom = Domain(lambda d: 0.0, space())
    docs = rand.suggest(list(range(N)), dom, Trials(), 0)
    labels = sorted(docs[0]['misc']['vals'])
    out = {}
    for lab in labels:
        out[lab] = np.array([d['misc']['vals'][lab][0] if d['misc']['vals'][lab] else np.nan
                             for d in docs], dtype=float)
    np.savez_compressed(os.path.join(HERE, 'prior_samples.npz'), **out)
    print({k: (np.nanmean(v), np.isnan(v).mean()) for k, v in out.items()})


if __name__ == '__main__':
    main()
