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


@pytest.mark.parametrize('C, n_rounds, labels', [(1 << 20, 1, 32), (24, 512, 64)])
def test_round_call_step_equals_sequential(C, n_rounds, labels):
    """round_call (tpe.suggest's and bench.py's step): the ordered subset
    rebuild's report deferred into the round (DEFER_REPORT: the dense labels'
    kernels queued first, the quantized / categorical families after the
    rebuild on the second stream) -- bytewise the results of the sequential
    step (ordered rebuild, then the whole round), tile rounds (config 3) and
    batched packed rounds (config 5) alike."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    hist = mixed_history(labels, 10000 + 4, seed=3)
    a, b = Engine(0, 'f64'), Engine(0, 'f64')
    la, lb = FminLoop(hist), FminLoop(hist)
    la.advance(a, 10000)
    lb.advance(b, 10000)
    P.PHASES = {}
    try:
        for i in range(3):
            n = 10001 + i
            rounds = list(range(100 * i, 100 * i + n_rounds))

            def rnd(e=a):
                if n_rounds == 1:
                    return e.suggest(seed=5 + i, n_candidates=C, round=rounds[0])
                return e.suggest_batch(seed=5 + i, rounds=rounds, n_candidates=C)
            _, got = la.advance(a, n, n_candidates=C, n_rounds=n_rounds, round_call=rnd)
            lb.advance(b, n, n_candidates=C, n_rounds=n_rounds)
            want = rnd(b)
            assert np.ascontiguousarray(got).view(np.uint8).tobytes() == \
                np.ascontiguousarray(want).view(np.uint8).tobytes(), i
            # the statistics of both halves survive: the dense screen's and
            # the quantized families' of the last round that ran them
            assert a.last_screen() == b.last_screen()
            ms_a, ms_b = a.last_mode_stats(), b.last_mode_stats()
            assert {k: v[1] for k, v in ms_a.items()} == {k: v[1] for k, v in ms_b.items()}
    finally:
        P.PHASES = None
        a.close()
        b.close()


def test_armed_prepare_is_queued_by_the_build():
    """tpe_arm_prepare (what FminLoop / tpe.suggest do before a build that a
    large round follows): the build itself queues the expansion index
    before it returns, the round on it equals a fresh engine's bytewise, and
    the arm is consumed -- the next build queues nothing."""
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    hist = mixed_history(8, 3000 + 3, seed=1)
    C = 1 << 16
    eng = Engine(0, 'f64')
    eng.set_option('timing', 1)
    loop = FminLoop(hist)
    loop.advance(eng, 3000)
    eng.last_prepare_ms()
    eng.arm_prepare(C)
    loop.advance(eng, 3001)           # the caller asks for no index: the armed build queues it
    ms = eng.last_prepare_ms()
    assert ms > 0
    got = eng.suggest(seed=3, n_candidates=C, round=0)
    ref = Engine(0, 'f64')
    FminLoop(hist).advance(ref, 3001)
    want = ref.suggest(seed=3, n_candidates=C, round=0)
    ref.close()
    assert np.ascontiguousarray(got).view(np.uint8).tobytes() == \
        np.ascontiguousarray(want).view(np.uint8).tobytes()
    loop.advance(eng, 3002)           # consumed: this build queues no index
    assert eng.last_prepare_ms() == ms
    eng.arm_prepare(C)
    eng.arm_prepare(0)                # disarmed
    loop.advance(eng, 3003)
    assert eng.last_prepare_ms() == ms
    eng.close()
