"""Config 3 / 5 fmin steps through FminLoop.suggest (pipelined): wall ms of
the pieces, whether the dense round stood, and the step time.
    python tools/pipe_probe.py [config] [steps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hyperopt_amd import posterior as P
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    nl, N0 = (128, 50000) if cfg == 5 else (32, 10000)
    hist = mixed_history(nl, N0 + steps + 4, seed=0)
    eng = Engine(0, 'f64')
    loop = FminLoop(hist)
    loop.advance(eng, N0)
    acc, log = {}, []

    def wrap(obj, name, key):
        f = getattr(obj, name)

        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                dt = time.perf_counter() - t0
                acc[key] = acc.get(key, 0.0) + dt
                log.append((key, round(1e3 * dt, 3)))
        setattr(obj, name, g)
    for n in ('build_posterior_ordered', 'prepare', 'history_append', 'suggest', 'suggest_batch',
              'last_build_kept_index'):
        wrap(eng, n, n)
    wrap(P, 'reference_orders', 'orders')
    ts = []
    for i in range(steps):
        del log[:]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if cfg == 5:
            loop.suggest(eng, N0 + 1 + i, 1234, 24, rounds=list(range(4096 * i, 4096 * (i + 1))))
        else:
            loop.suggest(eng, N0 + 1 + i, 1234 + i, 1 << 24, round=i)
        ts.append(time.perf_counter() - t0)
        print('step %d %.3f ms pipelined %s kept %s: %s' % (i, 1e3 * ts[-1], loop.pipelined,
                                                           eng.last_build_kept_index(), log), flush=True)
    print('median step %.3f ms' % (1e3 * np.median(ts[1:])))
    eng.close()


if __name__ == '__main__':
    main()
