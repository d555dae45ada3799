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
