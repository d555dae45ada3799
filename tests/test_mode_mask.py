"""TPE_OPT_MODE_MASK: a round limited to some label families leaves the
other labels' entries unspecified, and the launched labels' results equal
those of the whole round bytewise (the families' launches are independent:
each label's candidates come from its own Philox stream).  Both the tile map
(2^16 candidates) and the packed map (batched rounds of 24)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FAMILIES = {'dense': 1 | 2, 'quantized': 4 | 8, 'categorical': 16}


@pytest.fixture(scope='module')
def eng():
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    e = Engine(0, 'f64')
    FminLoop(mixed_history(15, 3000, seed=4)).advance(e, 3000)
    yield e
    e.close()


def _modes(eng):
    from hyperopt_amd.workloads import mixed_space
    kinds = [k for _, k, _ in mixed_space(15)]
    return np.array(['quantized' if k.startswith('q') else 'categorical' if k == 'randint' else 'dense'
                     for k in kinds])


@pytest.mark.parametrize('C, rounds', [(1 << 16, [3]), (24, list(range(40, 104)))])
def test_masked_families_equal_the_whole_round(eng, C, rounds):
    modes = _modes(eng)
    whole = eng.suggest_batch(9, rounds, C)
    try:
        for fam, mask in FAMILIES.items():
            eng.set_option('mode_mask', mask)
            part = eng.suggest_batch(9, rounds, C)
            cols = np.flatnonzero(modes == fam)
            assert len(cols)
            assert np.ascontiguousarray(part[:, cols]).tobytes() == \
                np.ascontiguousarray(whole[:, cols]).tobytes(), fam
    finally:
        eng.set_option('mode_mask', 31)


def test_mode_mask_range(eng):
    from hyperopt_amd.engine import EngineError
    for bad in (0, 32, -1):
        with pytest.raises(EngineError):
            eng.set_option('mode_mask', bad)
    eng.set_option('mode_mask', 31)


@pytest.mark.parametrize('C, rounds', [(1 << 16, [5]), (24, list(range(7, 71)))])
def test_side_families_on_the_second_stream(eng, C, rounds):
    """TPE_OPT_AUX_FAMILIES: the quantized and categorical labels' kernels
    run on the context's second stream beside the dense draw -- the results
    equal those of the one-stream round bytewise.  (Their early exit's draw
    counts, a statistic, depend on how the streams interleave: not compared.)"""
    try:
        one = eng.suggest_batch(11, rounds, C)
        eng.set_option('aux_families', 1)
        two = eng.suggest_batch(11, rounds, C)
    finally:
        eng.set_option('aux_families', 0)
    assert np.ascontiguousarray(one).tobytes() == np.ascontiguousarray(two).tobytes()
