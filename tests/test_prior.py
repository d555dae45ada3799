"""The startup sampler (rand.suggest, rand.py:15-31 / pyll/stochastic.py:
35-147) against the reference's own prior draws
(tests/golden/prior_samples.npz, gen_prior_samples.py): every hp kind and a
conditional choice, distribution by distribution.  The draw order differs
(this package draws choices first, then the selected branch), so the test is
statistical: two-sample Kolmogorov-Smirnov for continuous labels, a
chi-square test of the value counts for discrete ones, and the branch
activity rate of the conditional labels."""
import os

import numpy as np
import pytest
from scipy import stats

import hyperopt_amd as H
from hyperopt_amd import hp

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'prior_samples.npz')
DISCRETE = {'a', 'b', 'e', 'f', 'i', 'j', 'k', 'm'}


def space():
    return {'a': hp.choice('a', [0, 1, 2]), 'b': hp.randint('b', 10),
            'c': hp.uniform('c', 4, 7), 'd': hp.loguniform('d', -2, 0),
            'e': hp.quniform('e', 0, 10, 3), 'f': hp.qloguniform('f', 0, 3, 2),
            'g': hp.normal('g', 4, 7), 'h': hp.lognormal('h', -2, 2),
            'i': hp.qnormal('i', 0, 10, 2), 'j': hp.qlognormal('j', 0, 2, 1),
            'k': hp.pchoice('k', [(.1, 0), (.9, 1)]),
            'm': hp.choice('m', [{'u': hp.uniform('u', 0, 1)}, {'v': hp.normal('v', 0, 1)}])}


@pytest.fixture(scope='module')
def draws():
    ref = dict(np.load(GOLD))
    n = len(next(iter(ref.values())))
    dom = H.Domain(lambda d: 0.0, space())
    docs = H.rand.suggest(list(range(n)), dom, H.Trials(), 12345)
    ours = {lab: np.array([d['misc']['vals'][lab][0] if d['misc']['vals'][lab] else np.nan
                           for d in docs], dtype=float) for lab in ref}
    return ref, ours


@pytest.mark.parametrize('label', sorted(set('abcdefghijkmuv')))
def test_prior_distribution_matches_reference(draws, label):
    ref, ours = draws
    r, o = ref[label], ours[label]
    # activity (conditional labels): same rate
    ra, oa = np.isfinite(r).mean(), np.isfinite(o).mean()
    se = np.sqrt(ra * (1 - ra) / len(r) * 2) + 1e-12
    assert abs(ra - oa) <= 4 * se + 1e-12, (label, ra, oa)
    r, o = r[np.isfinite(r)], o[np.isfinite(o)]
    if label in DISCRETE:
        vals = np.union1d(r, o)
        table = np.array([[np.sum(r == v) for v in vals], [np.sum(o == v) for v in vals]])
        keep = table.sum(0) >= 10          # pool the sparse tail of the q* labels
        pooled = np.column_stack([table[:, keep], table[:, ~keep].sum(1)]) \
            if (~keep).any() else table[:, keep]
        pooled = pooled[:, pooled.sum(0) > 0]
        if pooled.shape[1] > 1:
            p = stats.chi2_contingency(pooled)[1]
            assert p > 1e-3, (label, p)
        # and the support: no value the reference could never draw
        if label in ('e', 'f', 'i', 'j'):
            q = {'e': 3, 'f': 2, 'i': 2, 'j': 1}[label]
            assert np.allclose(o / q, np.round(o / q))
    else:
        p = stats.ks_2samp(r, o).pvalue
        assert p > 1e-3, (label, p)
