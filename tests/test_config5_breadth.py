"""Config 5 at breadth on the product path:
BASELINE config 5 -- 128 labels (103 continuous, 25 choice), a 50k-trial
history, 4096 new_ids x 24 EI candidates per round -- with the posterior
fmin's loop builds (FminLoop: device build with numpy's tie order, the
expansion index queued beside the argsorts) and the engine tpe.suggest runs
(value-only rounds, the quantized and categorical families on the second
stream).  For 32 rounds x all 128 labels (4096 cells), the 24 candidates
are re-drawn through the sampler entry points and scored by the C
restatement of the reference's GMM1_lpdf / LGMM1_lpdf / categorical_lpdf
(oracle/tpe_score.c, OpenMP); broadcast_best's argmax (tpe.py:769-778) must
be the round's index and value in every cell."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_config5_value_only_rounds_match_oracle_argmax():
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    from oracle import c_oracle, near_ties
    if not c_oracle.available():
        pytest.skip('C oracle not built (make -C oracle)')
    hist = mixed_history(128, 50001, seed=0)
    eng = Engine(0, 'f64')
    try:
        eng.set_option('value_only', 1)
        eng.set_option('aux_families', 1)
        loop = FminLoop(hist)
        loop.advance(eng, 50000)
        ids = list(range(20000, 20000 + 4096))
        seed = 4242
        # the fmin step: one appended trial, the rebuild and its index, the round
        _, res = loop.advance(eng, 50001, n_candidates=24, n_rounds=len(ids),
                              round_call=lambda: eng.suggest_batch(seed, ids, 24))
        assert res.shape == (4096, 128)
        decided = int(np.sum(np.isnan(res['lpdf_below'])))
        posts = near_ties.posteriors_of(eng, hist.labels)
        rows = np.random.RandomState(5).choice(len(ids), 32, replace=False)
        cells = near_ties.batched_agreement(eng, posts, res, seed, ids, 24, rows)
    finally:
        eng.close()
    bad = [c for c in cells if not c['agree']]
    print('config 5: %d cells, %d agree; %d of %d cells decided by the screen alone (value-only)'
          % (len(cells), len(cells) - len(bad), decided, res.size))
    assert len(cells) == 32 * 128
    assert not bad, bad[:5]
