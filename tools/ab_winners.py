"""Winners of fixed rounds (configs 3 and 2, fmin-step posteriors) saved to
an .npz, to compare two builds bit for bit (e.g. the product library vs a
variant of an older commit: HYPEROPT_AMD_VARIANT=tools/var_<name>.so) --
a kernel change that must not move a single draw.

    python tools/ab_winners.py out.npz
    python tools/ab_winners.py --compare a.npz b.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out):
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, hartmann_history, mixed_history
    res = {}
    eng = Engine(0, 'f64')
    for name, hist, n0, C in (('c3', mixed_history(32, 10003, seed=0), 10000, 1 << 24),
                              ('c2', hartmann_history(2003, seed=0), 2000, 1 << 20)):
        loop = FminLoop(hist)
        for i in range(3):
            loop.advance(eng, n0 + i + 1, n_candidates=C)
            res['%s_%d' % (name, i)] = np.ascontiguousarray(eng.suggest(1234 + i, C, round=i)).view(np.uint8)
            res['%s_%d_hot' % (name, i)] = np.array(eng.last_hot(), dtype=np.int64)
    eng.close()
    np.savez(out, **res)
    print('saved', out, len(res))


def compare(a, b):
    A, B = np.load(a), np.load(b)
    same = True
    for k in sorted(A.files):
        if k.endswith('_hot'):
            print(k, A[k].tolist(), B[k].tolist())
            continue
        eq = A[k].tobytes() == B[k].tobytes()
        same = same and eq
        print(k, 'identical' if eq else 'DIFFERENT')
    print('ALL IDENTICAL' if same else 'MISMATCH')
    return 0 if same else 1


if __name__ == '__main__':
    if sys.argv[1] == '--compare':
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    run(sys.argv[1])
