"""Config 2's candidate-shard fresh step against the whole one: fmin steps
(append a trial, rebuild, index, round) with C = 2^20 candidates per label,
then with C/8 at the whole round's map choices (whole_n = C, what a
candidate-shard rank runs), then C/8 alone -- ms per step each.

    python tools/probe_cshard.py [steps]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    import torch
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, hartmann_history
    C = 1 << 20
    hist = hartmann_history(2000 + 4 * steps + 8, seed=0)
    eng = Engine(0)
    eng.set_option('value_only', 1)
    eng.set_option('aux_families', 1)
    loop = FminLoop(hist)
    n = 2000
    loop.advance(eng, n)
    out = {}
    for name, nc, whole in (('whole', C, 0), ('shard_whole_n', C // 8, C), ('shard_alone', C // 8, 0),
                            ('whole_again', C, 0)):
        eng.set_option('whole_n', whole)
        ts = []
        for i in range(steps + 2):
            n += 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            loop.advance(eng, n, n_candidates=nc, n_rounds=1,
                         round_call=lambda: eng.suggest(1234 + n, nc, round=n))
            torch.cuda.synchronize()
            if i >= 2:
                ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        out[name] = round(ts[len(ts) // 2], 3)
    eng.close()
    print(json.dumps(out))


if __name__ == '__main__':
    main()
