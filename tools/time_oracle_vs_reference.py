"""The restatement-to-reference speed ratio: the C oracle
oracle/tpe_score.c (the bench's cpu_baseline) against the reference's own
GMM1_lpdf / LGMM1_lpdf (hyperopt/tpe.py:110-172, 265-307) on the same inputs
in this container, both checked to agree.

Run in the survey container only (needs /root/reference):
    PYTHONDONTWRITEBYTECODE=1 OMP_NUM_THREADS=8 python tools/time_oracle_vs_reference.py

Writes profiles/r2_oracle_vs_reference_<threads>thr.json (run once with
OMP_NUM_THREADS=1 and once with 8).  The reference is called in
chunks of <= 25k candidates (its C x K temporaries would not fit otherwise),
single-threaded (numpy ufuncs use one core); the C oracle on 1 thread and
on all threads OpenMP gives it.
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.dont_write_bytecode = True
sys.path[:0] = [REPO, os.path.join(REPO, 'tools', 'refshim'), '/root/reference']

import hyperopt.tpe as R  # noqa: E402  (reference)
from oracle import c_oracle as C  # noqa: E402
from hyperopt_amd.workloads import mixed_history  # noqa: E402


def ref_chunked(fn, x, w, m, s, **kw):
    out = [fn(x[i:i + 25000], w, m, s, **kw) for i in range(0, len(x), 25000)]
    return np.concatenate(out)


def timeit(f, reps=1):
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        r = f()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best, r


def main():
    hist = mixed_history(32, 10000, seed=0)
    posts = hist.posteriors()
    rng = np.random.RandomState(0)
    cases = []
    # one label of each family at config 3 (N = 10k history, K_a ~ 9976)
    pick = {'uniform (GMM1 bounded)': 0, 'loguniform (LGMM1 bounded)': 1,
            'quniform (GMM1 q=1)': 2, 'normal (GMM1 unbounded)': 3}
    n_cand = int(os.environ.get('N_CAND', '4096'))
    for name, li in pick.items():
        p = posts[li]
        samp = R.GMM1 if p.family == 'GMM1' else R.LGMM1
        x = samp(*p.below, low=p.low, high=p.high, q=p.q, rng=rng, size=(n_cand,))
        kw = dict(low=p.low, high=p.high, q=p.q)
        for side, mix in (('above', p.above), ('below', p.below)):
            w, m, s = mix
            rf = R.GMM1_lpdf if p.family == 'GMM1' else R.LGMM1_lpdf
            cf = C.gmm1_lpdf if p.family == 'GMM1' else C.lgmm1_lpdf
            tr, ref = timeit(lambda: ref_chunked(rf, x, w, m, s, **kw))
            tn, gotn = timeit(lambda: cf(x, w, m, s, **kw), reps=2)
            fin = np.isfinite(ref)
            rel = float(np.max(np.abs(gotn[fin] - ref[fin]) / np.maximum(1.0, np.abs(ref[fin]))))
            evals = len(x) * len(w)
            cases.append({'label': name, 'mixture': side, 'K': len(w), 'candidates': len(x),
                          'reference_s': tr, 'reference_evals_per_s': evals / tr,
                          'c_oracle_s_all_threads': tn, 'c_oracle_evals_per_s_all_threads': evals / tn,
                          'speedup_all_threads': tr / tn, 'max_rel_diff': rel})
            print('%-28s %-5s K=%5d ref %.3fs (%.3g/s)  C %.3fs (%.3g/s) x%.1f  diff %.1e'
                  % (name, side, len(w), tr, evals / tr, tn, evals / tn, tr / tn, rel), flush=True)
    out = {'note': 'reference GMM1_lpdf / LGMM1_lpdf (numpy, 1 core, <=25k-candidate chunks) vs '
                   'oracle/tpe_score.c (OpenMP, %d threads) on the same candidates of config-3 '
                   'labels, this container (8-vCPU Xeon, AVX-512)' % C.threads(),
           'threads': C.threads(), 'cases': cases}
    with open(os.path.join(REPO, 'profiles', 'r2_oracle_vs_reference_%dthr.json' % C.threads()),
              'w') as f:
        json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
