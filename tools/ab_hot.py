"""A/B of engine options on one box, in one process (the boxes of the pool
differ by up to ~1.7x on the same code, so variants are only compared within
a call): config-3 warm rounds (2^24 candidates x 32 labels) with the hot-bin
prefilter's draw kernels (TPE_OPT_HOT32 0 / 1), and the expansion index's
build with the window split (TPE_OPT_BX_SPLIT 1 / auto), alternating.

    python tools/ab_hot.py [reps]        (AB_SPLITS=1,2,4,8: the bx_split values to alternate)
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    import torch
    from hyperopt_amd import posterior as P
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(32, 10000, seed=0)
    packed = P.pack(hist.posteriors())
    eng = Engine(0)
    eng.set_posterior(*packed)
    C = 1 << 24
    out = {'hot32': {}, 'bx_split': {}}
    for v in (0, 1, 2):   # warm-up of every variant
        eng.set_option('hot32', min(v, 1))
        eng.suggest(1, C, round=0)
    for v in [0, 1] * reps:
        eng.set_option('hot32', v)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.suggest(7, C, round=v)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        _, _, ms = eng.last_screen(with_ms=True)
        out['hot32'].setdefault(v, []).append((wall, ms))
    eng.set_option('hot32', 1)
    splits = [int(x) for x in os.environ.get('AB_SPLITS', '1,0').split(',')]
    for v in splits * reps:
        eng.set_option('bx_split', v)
        eng.set_posterior(*packed)           # a new posterior: the index is rebuilt
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.prepare(C)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        out['bx_split'].setdefault(v, []).append((wall, eng.last_prepare_ms()))
    eng.close()
    summ = {}
    for k, d in out.items():
        summ[k] = {str(v): {'wall_ms_median': round(float(np.median([a for a, _ in x])), 4),
                            'device_ms_median': round(float(np.median([b for _, b in x])), 4),
                            'n': len(x)} for v, x in d.items()}
    print(json.dumps(summ))


if __name__ == '__main__':
    main()
