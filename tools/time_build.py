"""Posterior build time, host (numpy posterior.py + pack + tpe_set_posterior's
host fold and upload) vs device (tpe_build_posterior), at the BASELINE
configurations' history sizes.

    python tools/time_build.py [--reps 5]
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
    ap.add_argument('--reps', type=int, default=5)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    from hyperopt_amd import posterior as P
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import conditional_history, hartmann_history, mixed_history
    eng = Engine(0, 'f64')
    cases = [('config2', hartmann_history(2000, seed=0)),
             ('config3', mixed_history(32, 10000, seed=0)),
             ('config4', conditional_history(5000, seed=0)),
             ('config5', mixed_history(128, 50000, seed=0))]
    out = {}
    for name, hist in cases:
        host, dev, dev_k, prep = [], [], [], []
        for r in range(args.reps + 1):
            t0 = time.perf_counter()
            posts = hist.posteriors()
            eng.set_posterior(*P.pack(posts))
            t1 = time.perf_counter()
            inp = hist.device_inputs()
            t2 = time.perf_counter()
            eng.build_posterior(*inp, gamma=0.25, prior_weight=1.0)
            t3 = time.perf_counter()
            if r:
                host.append(t1 - t0)
                prep.append(t2 - t1)
                dev.append(t3 - t2)
                dev_k.append(eng.last_build_ms())
        out[name] = dict(labels=len(hist.labels), trials=len(hist.tids),
                         host_ms=round(1e3 * float(np.median(host)), 3),
                         device_inputs_ms=round(1e3 * float(np.median(prep)), 3),
                         device_call_ms=round(1e3 * float(np.median(dev)), 3),
                         device_kernels_ms=round(float(np.median(dev_k)), 3))
        print(json.dumps({name: out[name]}), flush=True)
    eng.close()


if __name__ == '__main__':
    main()
