"""fmin's loop on the device (workloads.FminLoop, bench.py's default step):
every step appends a trial to the resident history, rebuilds the posterior
with numpy's tie order (posterior.build_reference_order) while the
expansion index of the first, order-free build runs (Engine.prepare), and
the ordered rebuild keeps that index because the dense labels come out
bit-identical (tpe_build.hip: bx_keep_check).  The rounds must equal, bit
for bit, those of an engine that builds each history from scratch with the
index built inside its round -- i.e. the kept index is the one the round
would have built (reference: tpe.suggest rebuilds everything per call,
hyperopt/tpe.py:834,900)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_fmin_loop_rounds_equal_fresh_engine():
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    hist = mixed_history(32, 10000 + 6, seed=0)
    C = 1 << 20
    eng = Engine(0, 'f64')
    loop = FminLoop(hist)
    loop.advance(eng, 10000)
    for i in range(4):
        n = 10001 + i
        loop.advance(eng, n, n_candidates=C)
        got = eng.suggest(seed=77 + i, n_candidates=C, round=i)
        ref_eng = Engine(0, 'f64')
        FminLoop(hist).advance(ref_eng, n)          # one upload, no prepare: index built in the round
        want = ref_eng.suggest(seed=77 + i, n_candidates=C, round=i)
        # the device mixtures of the two engines are identical too
        for li in (0, 2, 3):
            for side in (0, 1):
                a, b = eng.get_mixture(li, side), ref_eng.get_mixture(li, side)
                assert all(np.array_equal(x, y) for x, y in zip(a, b))
        ref_eng.close()
        assert np.ascontiguousarray(got).view(np.uint8).tobytes() == \
            np.ascontiguousarray(want).view(np.uint8).tobytes(), i
        # quantized labels needed numpy's order; the loop supplied it
        assert {2, 7, 12, 17, 22, 27} <= set(loop.uploader.tie_labels)
    eng.close()


def test_pipelined_step_equals_one_round():
    """FminLoop.suggest pipelines the step (the dense labels' round on the
    order-free build while a background thread computes numpy's tie orders,
    the quantized and categorical labels' round on the ordered rebuild):
    every label's winner, value and lpdfs equal one full round on the
    ordered posterior, for single rounds (2^20 candidates) and batched ones
    (512 new_ids x 24)."""
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    hist = mixed_history(32, 10000 + 8, seed=0)
    eng = Engine(0, 'f64')
    loop = FminLoop(hist)
    loop.advance(eng, 10000)
    for i in range(4):
        n = 10001 + i
        if i % 2 == 0:
            got = loop.suggest(eng, n, 77 + i, 1 << 20, round=i)
        else:
            got = loop.suggest(eng, n, 77 + i, 24, rounds=list(range(512 * i, 512 * (i + 1))))
        assert loop.pipelined, i
        want = (eng.suggest(77 + i, 1 << 20, round=i) if i % 2 == 0
                else eng.suggest_batch(77 + i, list(range(512 * i, 512 * (i + 1))), 24))
        assert np.ascontiguousarray(got).tobytes() == np.ascontiguousarray(want).tobytes(), i
    eng.close()


def test_tpe_suggest_pipelined_documents_equal_host_build():
    """tpe.suggest with a large n_EI_candidates on a space of 8 dense, 2
    quantized and 2 categorical labels past DEVICE_BUILD_MIN_OBS: the
    pipelined device path proposes the documents of the host build."""
    import hyperopt_amd as H
    from hyperopt_amd import hp, tpe
    rng = np.random.RandomState(5)
    space = {('u%d' % i): hp.uniform('u%d' % i, -3, 3) for i in range(6)}
    space.update({'n0': hp.normal('n0', 0, 2), 'l0': hp.loguniform('l0', -3, 1),
                  'q0': hp.quniform('q0', 0, 10, 1), 'q1': hp.quniform('q1', 0, 20, 2),
                  'c0': hp.choice('c0', [0, 1, 2]), 'c1': hp.randint('c1', 4)})
    trials = H.Trials()
    H.fmin(lambda d: float(np.sum([v for v in d.values()])) + rng.normal(), space, algo=H.rand.suggest,
           max_evals=1500, trials=trials, rstate=np.random.RandomState(1))
    dom = H.Domain(lambda d: 0, space)
    for seed in (3, 4):
        a = tpe.suggest([5000], dom, trials, seed, n_EI_candidates=1 << 16)[0]['misc']['vals']
        b = tpe.suggest([5000], dom, trials, seed, n_EI_candidates=1 << 16,
                        posterior_builder='host')[0]['misc']['vals']
        assert a == b
