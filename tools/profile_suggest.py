"""Host-side profile of tpe.suggest at the config-3 history (32 labels, 10k
trials, n_EI_candidates = 24): wall time per call, then cProfile's top
functions by own time and by cumulative time over the timed calls.

    python tools/profile_suggest.py [--labels 32] [--trials 10000] [--reps 30]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--labels', type=int, default=32)
    ap.add_argument('--trials', type=int, default=10000)
    ap.add_argument('--reps', type=int, default=30)
    ap.add_argument('--top', type=int, default=25)
    args = ap.parse_args()
    import torch  # noqa: F401
    from hyperopt_amd import tpe
    from hyperopt_amd.base import Domain
    from hyperopt_amd.workloads import history_trials, hp_space, mixed_history
    hist = mixed_history(args.labels, args.trials, seed=0)
    trials = history_trials(hist)
    domain = Domain(lambda d: 0.0, hp_space(hist.labels))
    for r in range(3):
        tpe.suggest([args.trials + r], domain, trials, 1000 + r)
    wall = []
    for r in range(args.reps):
        t0 = time.perf_counter()
        tpe.suggest([args.trials + r], domain, trials, 2000 + r)
        wall.append((time.perf_counter() - t0) * 1e3)
    wall.sort()
    print('suggest wall ms: median %.3f min %.3f max %.3f' % (wall[len(wall) // 2], wall[0], wall[-1]))
    pr = cProfile.Profile()
    pr.enable()
    for r in range(args.reps):
        tpe.suggest([args.trials + r], domain, trials, 3000 + r)
    pr.disable()
    for key in ('tottime', 'cumulative'):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(args.top)
        print(s.getvalue())


if __name__ == '__main__':
    main()
