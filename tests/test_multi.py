"""Multi-device contexts (tpe_ctx_create_multi, hyperopt_amd/csrc/tpe_multi.hip):
a round split over several device contexts -- here several contexts on the
one GPU of the test box, each with its own stream and host thread -- returns
the single-device winners bit for bit, for candidate shards (large C, with
the fp32 screen, quantized grid tables and categorical labels), round shards
(batched new_ids: split-K and chunked packed maps) and uneven splits; and
fmin(..., algo=partial(tpe.suggest, devices=[0, 0])) proposes the documents
devices=[0] proposes (hyperopt/fmin.py:201-202)."""
import functools

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ('index', 'value', 'score', 'lpdf_below', 'lpdf_above', 'label')


def _same(a, b):
    for f in FIELDS:
        assert np.array_equal(a[f], b[f], equal_nan=f not in ('index', 'label')), f


@pytest.fixture(scope='module')
def engines():
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(32, 10000, seed=0)
    one, two, three = Engine(0), Engine([0, 0]), Engine([0, 0, 0])
    for e in (one, two, three):
        e.build_posterior(*hist.device_inputs(), gamma=0.25, prior_weight=1.0)
    yield one, two, three
    for e in (one, two, three):
        e.close()


def test_devices_reported(engines):
    import ctypes
    one, two, three = engines
    arr = (ctypes.c_int32 * 4)()
    assert one.lib.tpe_ctx_devices(three.h, arr, 4) == 3
    assert list(arr)[:3] == [0, 0, 0]
    assert one.lib.tpe_ctx_devices(one.h, arr, 4) == 1


@pytest.mark.parametrize('C', [1 << 20, 3000, 1500, (1 << 16) + 5])
def test_candidate_shards_identical(engines, C):
    one, two, three = engines
    ref = one.suggest(77, C, round=4)
    for e in (two, three):
        got = e.suggest(77, C, round=4)
        _same(got, ref)
        assert e.last_evals() >= one.last_evals() - 0   # table evals run per device
    s1 = one.last_screen()
    assert s1[0] >= 0


@pytest.mark.parametrize('rounds,C', [(64, 24), (512, 24), (37, 100), (6, 4096)])
def test_round_shards_identical(engines, rounds, C):
    one, two, three = engines
    ids = list(range(1000, 1000 + rounds))
    ref = one.suggest_batch(9, ids, C)
    for e in (two, three):
        _same(e.suggest_batch(9, ids, C), ref)


def test_fmin_devices_same_documents():
    from hyperopt_amd import Trials, fmin, hp, tpe
    space = {'a': hp.uniform('a', -5, 5), 'b': hp.loguniform('b', -3, 2),
             'c': hp.quniform('c', 0, 20, 1), 'd': hp.choice('d', [0, 1, 2])}

    def fn(p):
        return (p['a'] - 1) ** 2 + (np.log(p['b']) + 1) ** 2 + (p['c'] - 7) ** 2 / 10 + p['d']

    vals = []
    for devs in ([0], [0, 0]):
        trials = Trials()
        fmin(fn, space, algo=functools.partial(tpe.suggest, devices=devs, n_EI_candidates=4096),
             max_evals=40, trials=trials, rstate=np.random.RandomState(3))
        vals.append([t['misc']['vals'] for t in trials.trials])
    assert vals[0] == vals[1]


@pytest.mark.parametrize('cfg', ['config3', 'config5'])
def test_label_shards_fmin_loop_identical(cfg):
    """a multi-device context over the resident history
    partitions the LABELS (TPE_OPT_LABEL_SHARDS: each device appends, builds,
    indexes and runs whole rounds of its labels only) and returns the
    one-device results bytewise -- fmin's loop (append, device build with
    numpy's tie orders, expansion index, round) at config 3's shape (32
    labels, 2^20 candidates per label) and config 5's (128 labels, batched
    rounds of 24 candidates), over 2 and 3 devices; the replicated
    candidate split (label_shards = 0) too."""
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    if cfg == 'config3':
        L, n0, C, R = 32, 10000, 1 << 20, 1
    else:
        L, n0, C, R = 128, 20000, 24, 512
    hist = mixed_history(L, n0 + 4, seed=0)
    engs = [Engine(0), Engine([0, 0]), Engine([0, 0, 0]), Engine([0, 0])]
    engs[3].set_option('label_shards', 0)
    loops = [FminLoop(hist) for _ in engs]
    try:
        for e, lp in zip(engs, loops):
            lp.advance(e, n0)
        for i in range(2):
            res = []
            for e, lp in zip(engs, loops):
                lp.advance(e, n0 + 1 + i, n_candidates=C, n_rounds=R)
                if R == 1:
                    res.append(e.suggest(seed=11 + i, n_candidates=C, round=i))
                else:
                    res.append(e.suggest_batch(seed=11 + i, rounds=list(range(R * i, R * i + R)), n_candidates=C))
            for r in res[1:]:
                _same(r, res[0])
            for li in (0, 1, 2, 3, 4, L - 1):   # the sharded contexts' mixtures come from their devices
                for side in (0, 1):
                    a, b = engs[0].get_mixture(li, side), engs[1].get_mixture(li, side)
                    assert all(np.array_equal(x, y) for x, y in zip(a, b))
        lib = engs[0].lib
        for e, nd in ((engs[1], 2), (engs[2], 3)):
            devs = [lib.tpe_label_device(e.h, li) for li in range(L)]
            assert sorted(set(devs)) == list(range(nd))   # every device holds labels
        assert lib.tpe_label_device(engs[3].h, 0) == -1   # replicated
        assert lib.tpe_label_device(engs[0].h, 0) == -1
    finally:
        for e in engs:
            e.close()


def test_fmin_devices_label_shards_same_documents():
    """fmin(..., partial(tpe.suggest, devices=[0, 0], posterior_builder='device'))
    -- the resident history, label-sharded over the two contexts -- proposes
    the documents devices=[0] proposes."""
    from hyperopt_amd import Trials, fmin, hp, tpe
    space = {'a': hp.uniform('a', -5, 5), 'b': hp.loguniform('b', -3, 2),
             'c': hp.quniform('c', 0, 20, 1), 'd': hp.choice('d', [0, 1, 2])}

    def fn(p):
        return (p['a'] - 1) ** 2 + (np.log(p['b']) + 1) ** 2 + (p['c'] - 7) ** 2 / 10 + p['d']

    vals = []
    for devs in ([0], [0, 0]):
        trials = Trials()
        fmin(fn, space, algo=functools.partial(tpe.suggest, devices=devs, n_EI_candidates=4096,
                                               posterior_builder='device'),
             max_evals=40, trials=trials, rstate=np.random.RandomState(3))
        vals.append([t['misc']['vals'] for t in trials.trials])
    assert vals[0] == vals[1]
