"""One label shard of the 8-way config-3 partition, alone on one GPU: wall
time of the fresh step's pieces (append + build(s) + index, round) and of
warm rounds -- what the one-GPU projection's slowest shard spends.
    python tools/shard_probe.py [shard] [steps] [config 3|5]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.parallel import label_shards
    from hyperopt_amd.workloads import FminLoop, mixed_history
    r = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    nl, N0 = (128, 50000) if cfg == 5 else (32, 10000)
    hist = mixed_history(nl, N0 + 2 * steps + 4, seed=0)
    sh = label_shards(hist.labels, 8)[r] if r >= 0 else list(range(nl))
    print('shard', r, 'labels', sh, [hist.labels[i][1] for i in sh])
    eng = Engine(0, 'f64')
    loop = FminLoop(hist, label_ids=sh if r >= 0 else None)
    # wall time per piece of the fresh step
    from hyperopt_amd import posterior as P
    acc = {}

    def wrap(obj, name, key):
        f = getattr(obj, name)

        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                acc[key] = acc.get(key, 0.0) + time.perf_counter() - t0
        setattr(obj, name, g)
    wrap(eng, 'build_posterior_ordered', 'build')
    wrap(eng, 'prepare', 'prepare')
    wrap(eng, 'history_append', 'append')
    wrap(P, 'reference_orders', 'orders')
    loop.advance(eng, N0)
    C, NR = (24, 4096) if cfg == 5 else (1 << 24, 1)

    def rnd(i, seed):
        if cfg == 5:
            return eng.suggest_batch(seed=seed, rounds=list(range(i * NR, (i + 1) * NR)), n_candidates=C)
        return eng.suggest(seed=seed, n_candidates=C, round=i)
    ta, ts = [], []
    for i in range(steps + 2):
        if i == 2:
            acc.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop.advance(eng, N0 + 1 + i, n_candidates=C, n_rounds=NR)
        t1 = time.perf_counter()
        rnd(i, 1234 + i)
        t2 = time.perf_counter()
        if i >= 2:
            ta.append(t1 - t0)
            ts.append(t2 - t1)
    tw = []
    for i in range(steps):
        t0 = time.perf_counter()
        rnd(i, 99 + i)
        tw.append(time.perf_counter() - t0)
    print('advance %.3f ms  round %.3f ms  warm %.3f ms  (medians; index %.3f ms, build %.3f ms)'
          % (1e3 * np.median(ta), 1e3 * np.median(ts), 1e3 * np.median(tw),
             eng.last_prepare_ms(), eng.last_build_ms()))
    print('advance pieces (ms per step):', {k: round(1e3 * v / steps, 3) for k, v in acc.items()})
    print('modes', eng.last_mode_stats(), 'tie labels', sorted(loop.uploader.tie_labels))
    eng.close()


if __name__ == '__main__':
    main()
