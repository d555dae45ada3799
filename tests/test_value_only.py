"""Value-only batched rounds (TPE_OPT_VALUE_ONLY): the
reference's suggestion document carries only the chosen values
(tpe.py:906-916), so a packed-map round whose screen selected ONE candidate
clearing every other's upper bound by 1e-9 (relative) reports its index and
value without computing its fp64 lpdfs.  The index and value must be the
exact round's bytewise (configs 3 and 5); the lpdfs of the decided cells are
NaN and every other cell's result is the exact round's.  Also the device-
planned re-score's overflow path (a round listing more candidates than the
buffers hold runs again with larger ones): same bytes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def eng():
    from hyperopt_amd.engine import Engine
    e = Engine(0, 'f64')
    yield e
    e.close()


def _both(eng, fn):
    eng.set_option('value_only', 0)
    exact = fn()
    eng.set_option('value_only', 1)
    try:
        vo = fn()
    finally:
        eng.set_option('value_only', 0)
    return exact, vo


def _check(exact, vo):
    assert np.array_equal(exact['index'], vo['index'])
    assert exact['value'].tobytes() == vo['value'].tobytes()
    decided = np.isnan(vo['lpdf_below']) & ~np.isnan(exact['lpdf_below'])
    # a decided cell says so (TPE_STATUS_VALUE_ONLY); every other one is ok
    assert np.all(vo['status'][decided] == 1) and np.all(vo['status'][~decided] == 0)
    assert np.all(exact['status'] == 0)
    # the cells the screen did not decide alone are the exact round's, bit for bit
    same = ~decided
    assert np.ascontiguousarray(exact[same]).tobytes() == np.ascontiguousarray(vo[same]).tobytes()
    return int(decided.sum())


def test_value_only_config5(eng):
    """Config 5 at its BASELINE size (128 labels, N = 50k, 4096 new_ids x
    24): most (round, dense label) cells are decided by the screen."""
    from hyperopt_amd.workloads import FminLoop, mixed_history
    hist = mixed_history(128, 50000, seed=0)
    FminLoop(hist).advance(eng, 50000, n_candidates=24, n_rounds=4096)
    ids = list(range(9000, 9000 + 4096))
    exact, vo = _both(eng, lambda: eng.suggest_batch(77, ids, 24))
    n = _check(exact, vo)
    dense = sum(1 for _, k, _ in hist.labels if k in ('uniform', 'loguniform', 'normal'))
    print('value-only config 5: %d of %d dense cells decided by the screen' % (n, dense * len(ids)))
    assert n > 0.5 * dense * len(ids)


def test_value_only_leaves_tile_rounds_exact(eng):
    """Config 3 (tile map, 2^20 candidates): value-only changes nothing --
    the near-tie re-score stays (the tile map's winners are merged across
    shards by score)."""
    from hyperopt_amd.workloads import FminLoop, mixed_history
    hist = mixed_history(32, 10000, seed=0)
    FminLoop(hist).advance(eng, 10000, n_candidates=1 << 20)
    exact, vo = _both(eng, lambda: eng.suggest(5, 1 << 20, round=3))
    assert np.ascontiguousarray(exact).tobytes() == np.ascontiguousarray(vo).tobytes()


@pytest.mark.parametrize('value_only', [0, 1])
def test_packed_rescore_overflow_runs_again(eng, value_only):
    """A packed round whose selection exceeds the re-score buffers (capacity
    forced to 1) runs again with buffers for all of them: the same bytes as
    with room to spare."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(64, 20000, seed=1)
    eng.set_posterior(*P.pack(hist.posteriors()))
    ids = list(range(7000, 7512))
    eng.set_option('value_only', value_only)
    try:
        eng.set_option('rescore_cap', 1 << 20)
        a = eng.suggest_batch(31, ids, 24)
        eng.set_option('rescore_cap', 1)
        b = eng.suggest_batch(31, ids, 24)
        c = eng.suggest_batch(31, ids, 24)   # (the grown buffers, no second run)
    finally:
        eng.set_option('value_only', 0)
    assert np.ascontiguousarray(a).tobytes() == np.ascontiguousarray(b).tobytes()
    assert np.ascontiguousarray(a).tobytes() == np.ascontiguousarray(c).tobytes()


def test_exact_round_after_an_empty_value_only_plan(eng):
    """A value-only round whose screen decides every cell plans no re-score
    and skips the zero windows (k_zero_windows exits on the empty plan); an
    exact round on the same posterior afterwards must build them: its bytes
    equal those of an exact round on a fresh posterior."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(64, 20000, seed=2)
    posts = P.pack(hist.posteriors())
    ids = list(range(300, 812))
    eng.set_posterior(*posts)
    eng.set_option('value_only', 1)
    try:
        vo = eng.suggest_batch(13, ids, 24)
        rescored = eng.last_screen()[1]
    finally:
        eng.set_option('value_only', 0)
    assert rescored == 0, rescored            # the plan was empty: no zero windows built
    after = eng.suggest_batch(13, ids, 24)
    eng.set_posterior(*posts)              # a fresh posterior: windows built in its first round
    fresh = eng.suggest_batch(13, ids, 24)
    assert np.ascontiguousarray(after).tobytes() == np.ascontiguousarray(fresh).tobytes()
    assert np.isnan(vo['lpdf_below']).any()   # (the value-only round decided cells alone)


def test_merge_refuses_value_only_records(eng):
    """Candidate shards merge by score (broadcast_best): a value-only record
    has none, so both merges refuse it instead of ranking its NaN (ADVICE
    r4), and parallel.DeviceExchange turns value-only off for candidate
    shards."""
    import torch
    from hyperopt_amd import posterior as P
    from hyperopt_amd.engine import EngineError, merge_results
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(64, 20000, seed=2)
    eng.set_posterior(*P.pack(hist.posteriors()))
    ids = list(range(300, 812))
    eng.set_option('value_only', 1)
    try:
        vo = eng.suggest_batch(13, ids, 24)
    finally:
        eng.set_option('value_only', 0)
    exact = eng.suggest_batch(13, ids, 24)
    assert (vo['status'] == 1).any()
    with pytest.raises(EngineError):
        merge_results(np.stack([vo.ravel(), exact.ravel()]))
    parts = torch.from_numpy(np.ascontiguousarray(np.stack([exact.ravel(), vo.ravel()])).view(np.uint8)
                             .reshape(-1)).cuda()
    out = torch.empty(exact.size * exact.dtype.itemsize, dtype=torch.uint8, device='cuda')
    with pytest.raises(EngineError, match='value-only'):
        eng.merge_results_device(parts, 2, exact.size, out)
    # two exact parts merge as before
    ok = torch.from_numpy(np.ascontiguousarray(np.stack([exact.ravel(), exact.ravel()])).view(np.uint8)
                          .reshape(-1)).cuda()
    eng.merge_results_device(ok, 2, exact.size, out)
    assert out.cpu().numpy().tobytes() == np.ascontiguousarray(exact.ravel()).tobytes()
