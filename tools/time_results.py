"""Where a config-5 round's host time goes: the batched round (4096 new_ids
x 128 labels x 24 candidates) returned to a numpy array (tpe_suggest_batch)
against the same round left in device memory (tpe_suggest_batch_device),
and the cost of the 25 MB result array itself.

    python tools/time_results.py [reps] [host]   (host: the host-array round only, for a trace)
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def med(f, reps):
    import torch
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(float(np.median(ts)), 3)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    import torch
    from hyperopt_amd.engine import RESULT_DTYPE, Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    hist = mixed_history(128, 50001, seed=0)
    eng = Engine(0)
    eng.set_option('value_only', 1)
    eng.set_option('aux_families', 1)
    FminLoop(hist).advance(eng, 50000, n_candidates=24, n_rounds=4096)
    ids = list(range(4096))
    L = eng._labels()
    nbytes = 4096 * L * RESULT_DTYPE.itemsize
    dbuf = torch.empty(nbytes, dtype=torch.uint8, device='cuda')
    eng.suggest_batch(7, ids, 24)
    eng.suggest_batch_device(7, ids, 24, dbuf)
    if sys.argv[2:3] == ['host']:
        print(json.dumps({'host_results_ms': med(lambda: eng.suggest_batch(7, ids, 24), reps)}))
        eng.close()
        return
    out = {}
    for seed, first in ((7, 0), (1234, 4096), (1234, 8192)):
        ii = list(range(first, first + 4096))
        out['seed%d_ids%d_ms' % (seed, first)] = med(lambda: eng.suggest_batch(seed, ii, 24), 3)
        out['seed%d_ids%d_screened_rescored' % (seed, first)] = eng.last_screen()
    out.update({
        'host_results_ms': med(lambda: eng.suggest_batch(7, ids, 24), reps),
        'device_results_ms': med(lambda: eng.suggest_batch_device(7, ids, 24, dbuf), reps),
        'np_zeros_ms': med(lambda: np.zeros(4096 * L, dtype=RESULT_DTYPE), reps),
        'np_empty_touch_ms': med(lambda: np.empty(4096 * L, dtype=RESULT_DTYPE).view(np.uint8).fill(1), reps),
        'result_bytes': nbytes,
    })
    eng.close()
    print(json.dumps(out))


if __name__ == '__main__':
    main()
