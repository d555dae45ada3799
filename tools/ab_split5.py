"""The expansion index's window split at config 5 (128 labels, N = 50k,
rounds of 4096 x 24), alternated in one process: each fmin step appends a
trial and rebuilds the posterior, whose index is then timed
(tpe_last_prepare: device ms, the wall of the queued index).

    python tools/ab_split5.py [reps] [splits, e.g. 1:2:3]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    splits = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else '1:2:3').split(':')]
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    n0 = 50000
    hist = mixed_history(128, n0 + 1 + len(splits) * (reps + 1), seed=0)
    eng = Engine(0)
    eng.set_option('value_only', 1)
    eng.set_option('aux_families', 1)
    loop = FminLoop(hist)
    loop.advance(eng, n0)
    n = n0
    out = {}
    for i, v in enumerate(splits * (reps + 1)):
        eng.set_option('bx_split', v)
        n += 1
        loop.advance(eng, n, n_candidates=24, n_rounds=4096)
        ms = eng.last_prepare_ms()
        if i >= len(splits):   # (the first pass warms every variant up)
            out.setdefault(v, []).append(ms)
    eng.close()
    print(json.dumps({str(v): {'index_ms_median': round(float(np.median(x)), 4), 'n': len(x),
                               'all': [round(t, 3) for t in x]} for v, x in out.items()}))


if __name__ == '__main__':
    main()
