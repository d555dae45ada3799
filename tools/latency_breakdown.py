"""Where the wall time of one tpe.suggest goes (config 3 history: 32 labels,
10k trials, n_EI_candidates=24), for the host and the device posterior
builders.  Stages: history gather, posterior (host numpy + pack +
set_posterior, or device_inputs + tpe_build_posterior), the fused GPU round,
trial-document creation.

    python tools/latency_breakdown.py [--labels 32] [--trials 10000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--labels', type=int, default=32)
    ap.add_argument('--trials', type=int, default=10000)
    ap.add_argument('--reps', type=int, default=10)
    args = ap.parse_args()
    import torch  # noqa: F401
    from hyperopt_amd import engine as E, history as Hm, posterior as P, tpe
    from hyperopt_amd import labels as LB
    from hyperopt_amd.base import Domain
    from hyperopt_amd.workloads import history_trials, hp_space, mixed_history
    hist = mixed_history(args.labels, args.trials, seed=0)
    trials = history_trials(hist)
    domain = Domain(lambda d: 0.0, hp_space(hist.labels))
    eng = E.get_engine(0, 'f64')
    eng.set_option('timing', 1)       # this tool reads the device timings
    for builder in ('host', 'device'):
        st = {k: [] for k in ('gather', 'posterior', 'round', 'docs', 'total', 'suggest_call')}
        for r in range(args.reps + 2):
            t0 = time.perf_counter()
            specs = tpe.specs_of(domain)
            tids, losses, obs = Hm.gather(domain, trials, list(specs))
            t1 = time.perf_counter()
            if builder == 'device':
                eng.build_posterior(*tpe.device_inputs(specs, tids, losses, obs), gamma=0.25,
                                    prior_weight=1.0)
            else:
                sp = P.Splitter(tids, losses, 0.25)
                posts = [P.label_posterior(k, s.kind, s.args, *sp.split(*obs[k]), 1.0)
                         for k, s in specs.items()]
                eng.set_posterior(*P.pack(posts))
            t2 = time.perf_counter()
            res = eng.suggest(1000 + r, 24, round=args.trials + r)[None]
            t3 = time.perf_counter()
            values = {s.label: LB.coerce(s.kind, res[0][i]['value'])
                      for i, s in enumerate(specs.values())}
            tpe._doc(args.trials + r, domain, trials, specs, values)
            t4 = time.perf_counter()
            tpe.suggest([args.trials + r], domain, trials, 1000 + r, posterior_builder=builder)
            t5 = time.perf_counter()
            if r >= 2:
                for k, v in zip(('gather', 'posterior', 'round', 'docs', 'total', 'suggest_call'),
                                (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0, t5 - t4)):
                    st[k].append(v * 1e3)
        print(json.dumps({'builder': builder, **{k: round(float(np.median(v)), 3)
                                                 for k, v in st.items()}}), flush=True)
    eng.suggest(7, 24, round=1)
    sc, rd = eng.last_timing()
    print(json.dumps({'round_device_ms': {'score': sc, 'round': rd},
                      'per_family': {k: round(v[0], 4) for k, v in eng.last_mode_stats().items()}}))


if __name__ == '__main__':
    main()
