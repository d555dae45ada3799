"""Compare the resident-history build (tpe.suggest's uploader) with the
one-shot device build on the config-3 history: mixtures and round results."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401
    from hyperopt_amd import engine as E, history as Hm, posterior as P, tpe
    from hyperopt_amd.base import Domain
    from hyperopt_amd.workloads import history_trials, hp_space, mixed_history
    hist = mixed_history(32, 10000, seed=0)
    trials = history_trials(hist)
    domain = Domain(lambda d: 0.0, hp_space(hist.labels))
    eng = E.get_engine(0, 'f64')
    specs = tpe.specs_of(domain)
    labels = [(s.label, s.kind, s.args) for s in specs.values()]

    def snap():
        return [np.concatenate(eng.get_mixture(l, s)) for l in range(32) for s in (0, 1)]

    tids, losses, obs = Hm.gather(domain, trials, list(specs))
    eng.build_posterior(*tpe.device_inputs(specs, tids, losses, obs), gamma=0.25, prior_weight=1.0)
    a = snap()
    ra = eng.suggest(1234, 24, round=10001)
    up = P.DeviceHistoryUploader()
    view = Hm.device_view(domain, trials, list(specs))
    up.build(eng, labels, view, 0.25, 1.0)
    b = snap()
    rb = eng.suggest(1234, 24, round=10001)
    up.build(eng, labels, view, 0.25, 1.0)
    c = snap()
    rc = eng.suggest(1234, 24, round=10001)
    # determinism of the round and of the records across rebuilds
    cand = np.linspace(-4.9, 4.9, 333)
    def scores():
        out = []
        for l in range(32):
            kind = labels[l][1]
            if kind == 'randint':
                x = np.arange(5, dtype=float)
            elif kind == 'loguniform':
                x = np.exp(np.linspace(-4.9, 1.9, 333))
            elif kind == 'quniform':
                x = np.arange(0, 101, dtype=float)
            else:
                x = cand
            lb, la, _ = eng.score(l, x)
            out.append(np.concatenate([lb, la]))
        return out
    s1 = scores()
    r1 = eng.suggest(1234, 24, round=10001)
    r2 = eng.suggest(1234, 24, round=10001)
    print('same posterior, two rounds equal:', np.array_equal(r1['index'], r2['index']))
    up.build(eng, labels, view, 0.25, 1.0)
    s2 = scores()
    diff = [l for l in range(32) if not np.array_equal(s1[l], s2[l])]
    print('score differences after rebuild (labels):', diff)
    for l in diff[:3]:
        i = np.nonzero(s1[l] != s2[l])[0]
        print(l, labels[l][1], i[:5], s1[l][i[:3]], s2[l][i[:3]])
    for name, x in (('fresh-resident', b), ('again', c)):
        bad = [i for i, (u, v) in enumerate(zip(a, x)) if not np.array_equal(u, v)]
        print(name, 'mixtures differing:', bad[:10])
    for name, r in (('oneshot', ra), ('resident', rb), ('again', rc)):
        print(name, 'idx', r['index'][:8].tolist(), 'nan/inf lpdf:',
              int(np.sum(~np.isfinite(r['lpdf_below']))), int(np.sum(~np.isfinite(r['lpdf_above']))))
        print('   mode ms', {k: round(v[0], 3) for k, v in eng.last_mode_stats().items()})
    eng.build_posterior(*tpe.device_inputs(specs, tids, losses, obs), gamma=0.25, prior_weight=1.0)
    up.build(eng, labels, view, 0.25, 1.0)
    d = snap()
    bad = [i for i, (u, v) in enumerate(zip(a, d)) if not np.array_equal(u, v)]
    print('oneshot then resident (no append): differing', bad[:10])
    if bad:
        i = bad[0]
        print(len(a[i]), len(d[i]), np.nonzero(a[i] != d[i])[0][:10])


if __name__ == '__main__':
    main()
