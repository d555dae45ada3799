"""Device posterior build per label kind: 4-label single-kind histories of
10k trials, each built --reps times; host CLOCK_MONOTONIC windows per kind
go to gpurun_out/build_kinds.json so a rocprofv3 --kernel-trace of this
script can be split by kind (tools/build_kinds.py --report <trace dir>).

    rocprofv3 --kernel-trace -d <dir> -o run --output-format csv -- python tools/build_kinds.py
    python tools/build_kinds.py --report <dir>
"""
import argparse
import csv
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out',
                   'build_kinds.json')


def run(reps, trials):
    import torch  # noqa: F401
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import CYCLE, History, prior_draw
    import numpy as np
    eng = Engine(0, 'f64')
    windows = {}
    for kind, args in CYCLE:
        rng = np.random.RandomState(0)
        labels = [('%s%d' % (kind, i), kind, args) for i in range(4)]
        tids = np.arange(trials, dtype=np.int64)
        losses = rng.normal(size=trials)
        obs = {name: (tids, prior_draw(k, a, rng, trials)) for name, k, a in labels}
        hist = History(labels, tids, losses, obs)
        inp = hist.device_inputs()
        eng.build_posterior(*inp, gamma=0.25, prior_weight=1.0)
        t0 = time.monotonic_ns()
        ms = []
        for _ in range(reps):
            eng.build_posterior(*inp, gamma=0.25, prior_weight=1.0)
            ms.append(eng.last_build_ms())
        windows[kind] = (t0, time.monotonic_ns())
        print(kind, 'device build ms (median)', sorted(ms)[len(ms) // 2], flush=True)
        time.sleep(0.05)
    eng.close()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    json.dump(windows, open(OUT, 'w'))


def report(d):
    windows = json.load(open(OUT))
    rows = []
    for f in glob.glob(d + '/**/*kernel_trace.csv', recursive=True):
        rows += list(csv.DictReader(open(f)))
    for kind, (t0, t1) in windows.items():
        acc = {}
        for r in rows:
            s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            if t0 <= s <= t1:
                name = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '')
                name = name.split('(')[0][:40]
                acc.setdefault(name, []).append((e - s) / 1e3)
        print(kind, {k: round(sorted(v)[len(v) // 2], 1) for k, v in acc.items()})


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--trials', type=int, default=10000)
    ap.add_argument('--report')
    a = ap.parse_args()
    if a.report:
        report(a.report)
    else:
        run(a.reps, a.trials)
