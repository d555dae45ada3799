import numpy as np
from hyperopt_amd import posterior as P
from hyperopt_amd.engine import Engine, merge_results
from hyperopt_amd.workloads import hartmann_history
hist = hartmann_history(2000, seed=0)
posts = hist.posteriors()
eng = Engine(0, 'f64')
eng.set_posterior(*P.pack(posts))
for C in (1 << 14, 1 << 18, 1 << 20):
    full = eng.suggest(77, C, round=5)
    for shards in (2, 8):
        parts = [eng.suggest(77, C // shards, round=5, cand_offset=k * (C // shards)) for k in range(shards)]
        print(C, shards, 'full', full['index'][:3], full['score'][:3])
        for k, p in enumerate(parts):
            print('  part', k, p['index'][:3], p['score'][:3], p['status'][:3], p['label'][:3])
        m = merge_results(np.stack(parts))
        print('  merged', m['index'][:3], m['score'][:3], m['status'][:3])
eng.close()
