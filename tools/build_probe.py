"""Which label kinds make the device build's per-label kernels long: for
each kind of the config-3/5 cycle, a 26-label history of that kind alone
(N = 50k, config 5's size) built on the device, REPS times, 0.2 s apart
from the next kind (under rocprofv3 --kernel-trace the launches then fall
into one cluster per kind, in CYCLE order).

    python tools/build_probe.py [reps] [n_trials]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
    import torch
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import CYCLE, History, bowl, prior_draw
    eng = Engine(0)
    out = {}
    for kind, args in CYCLE:
        rng = np.random.RandomState(0)
        labels = [('x%03d' % i, kind, args) for i in range(26)]
        tids = np.arange(n, dtype=np.int64)
        loss = 0.1 * rng.normal(size=n)
        obs = {}
        for name, k, a in labels:
            v = prior_draw(k, a, rng, n)
            loss = loss + bowl(k, v)
            obs[name] = (tids, v)
        hist = History(labels, tids, loss, obs)
        inputs = hist.device_inputs()
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.build_posterior(*inputs, gamma=0.25, prior_weight=1.0)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        out[kind] = {'wall_ms_median': round(float(np.median(ts)), 3), 'last_build_ms': eng.last_build_ms()}
        time.sleep(0.2)
    eng.close()
    print(json.dumps(out))


if __name__ == '__main__':
    main()
