"""The reference's tie order on the device-built posterior.

adaptive_parzen_normal orders the observations with `np.argsort(mus)`
(tpe.py:433) and ap_filter_trials the losses with `np.argsort(l_vals)`
(tpe.py:637): numpy's unstable sort, whose placement of equal keys no device
sort reproduces.  On a quantized label (or any label with repeated values)
the order of equal mus decides which linear-forgetting weight sits in which
slot: which weight meets a run end's sigma (the gap to the neighbouring grid
value) instead of the clipped minimum of the run's inner slots, and the order
of the normalising np.sum.  On a coarse grid (quniform(0, 10, 1): gap 1,
clipped minimum 0.1) the mixtures differ as functions.

The device builder flags every mixture that depends on a tie order (k_parzen)
and every tie of losses across the split (k_split); the host computes numpy's
own np.argsort for exactly those and the device builds again with it
(posterior.build_reference_order, tpe_build_posterior_resident_ordered).

Bar: the device mixtures are BIT-IDENTICAL to the host build (posterior.py,
numpy in the reference's call order) on coarse quantized labels -- quniform,
qloguniform, qnormal -- at >= 16384 observations, with a tie of losses at the
split; and tpe.suggest with posterior_builder='auto' (device build past 16384
observations) proposes the documents posterior_builder='host' proposes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

COARSE = [
    ('qu10', 'quniform', dict(low=0.0, high=10.0, q=1.0)),
    ('qlu', 'qloguniform', dict(low=0.0, high=float(np.log(40.0)), q=1.0)),
    ('qn', 'qnormal', dict(mu=0.0, sigma=2.0, q=0.5)),
    ('qu100', 'quniform', dict(low=0.0, high=100.0, q=1.0)),
    ('u', 'uniform', dict(low=-5.0, high=5.0)),
    ('ri', 'randint', dict(upper=4)),
]


def coarse_history(n_trials=6000, seed=0, split_tie=True):
    """6 labels x 6000 trials = 36k observations (>= DEVICE_BUILD_MIN_OBS);
    losses with a tie straddling the n_below boundary (n_below = 20: 15
    trials at -6, 10 at -5)."""
    from hyperopt_amd.workloads import History, prior_draw
    rng = np.random.RandomState(seed)
    tids = np.arange(n_trials, dtype=np.int64)
    obs, loss = {}, 0.1 * rng.normal(size=n_trials)
    for name, kind, args in COARSE:
        v = prior_draw(kind, args, rng, n_trials)
        obs[name] = (tids, v)
        loss = loss + 0.01 * (v - v.mean()) ** 2 / (v.var() + 1.0)
    if split_tie:
        pick = rng.permutation(n_trials)[:25]
        loss[pick[:15]] = -6.0
        loss[pick[15:]] = -5.0
    return History(COARSE, tids, loss, obs)


def _assert_same(eng, hist, posts):
    for li, p in enumerate(posts):
        sides = ((0, p.below), (1, p.above))
        for side, want in sides:
            w, m, s = eng.get_mixture(li, side)
            if p.family == 'categorical':
                assert np.array_equal(w, want), (p.label, side)
                continue
            hw, hm, hs = want
            assert np.array_equal(m, hm), (p.label, side, 'mus')
            assert np.array_equal(s, hs), (p.label, side, 'sigmas')
            assert np.array_equal(w, hw), (p.label, side, 'weights', float(np.max(np.abs(w - hw))))


def test_coarse_quantized_mixtures_bit_identical_to_host():
    from hyperopt_amd import posterior as P
    from hyperopt_amd.engine import Engine
    hist = coarse_history()
    inputs = hist.device_inputs()
    posts = hist.posteriors()                      # host build: the reference's np.argsort
    eng = Engine(0)
    try:
        # without the reference's order the device flags the tied mixtures
        # and the split tie -- and its position-order mixtures differ
        eng.history_reset(inputs[0], inputs[1])
        eng.history_append(np.diff(inputs[3]), inputs[4], inputs[5])
        nb, ties = eng.build_posterior_ordered(hist.losses, len(hist.losses), 0.25, 1.0)
        assert nb == 20 and ties[-1] == 1, ties
        flagged = {COARSE[l][0] for l in np.flatnonzero(ties[:-1] & 2)}
        assert {'qu10', 'qlu', 'qn', 'qu100'} <= flagged, flagged
        assert not flagged & {'u', 'ri'}
        w_pos = eng.get_mixture(0, 1)[0]
        assert not np.array_equal(w_pos, posts[0].above[0])   # the test can tell orders apart
        # the product path: the reference's order where it matters
        nb = eng.build_posterior(*inputs, gamma=0.25, prior_weight=1.0)
        assert nb == 20
        assert {COARSE[l][0] for l in eng.tie_labels} == flagged
        _assert_same(eng, hist, posts)
        # the resident history, built incrementally, keeps the order too
        from hyperopt_amd.history import device_view
        from hyperopt_amd.base import Domain
        from hyperopt_amd.workloads import history_trials, hp_space
        trials = history_trials(hist)
        dom = Domain(lambda d: 0.0, hp_space(hist.labels))
        up = P.DeviceHistoryUploader()
        view = device_view(dom, trials, [n for n, _, _ in COARSE])
        up.build(eng, COARSE, view, 0.25, 1.0)
        _assert_same(eng, hist, posts)
        # and on identical candidates the winners and lpdfs equal those of the
        # host-built posterior
        res_dev = [eng.suggest(seed, C, round=r) for C, r, seed in ((24, 3, 5), (1 << 18, 4, 6))]
        eng.set_posterior(*P.pack(posts))
        res_host = [eng.suggest(seed, C, round=r) for C, r, seed in ((24, 3, 5), (1 << 18, 4, 6))]
        for a, b in zip(res_dev, res_host):
            assert np.array_equal(a['index'], b['index'])
            assert np.array_equal(a['value'], b['value'])
            np.testing.assert_allclose(a['lpdf_below'], b['lpdf_below'], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(a['lpdf_above'], b['lpdf_above'], rtol=1e-12, atol=1e-12)
    finally:
        eng.close()


def test_auto_and_host_builders_suggest_identical_documents():
    """tpe.suggest on the coarse history: 'auto' takes the device builder
    (36k observations), 'host' the numpy one; same documents for several
    seeds, and again after trials are appended (the resident history grows
    incrementally, the known tie-dependent labels keep their order)."""
    from hyperopt_amd import tpe
    from hyperopt_amd.base import Domain
    from hyperopt_amd.engine import get_engine
    from hyperopt_amd.workloads import history_trials, hp_space
    hist = coarse_history(seed=1)
    trials = history_trials(hist)
    dom = Domain(lambda d: 0.0, hp_space(hist.labels))
    n = len(hist.tids)
    for step in range(4):
        new_id = n + step
        a = tpe.suggest([new_id], dom, trials, 100 + step, posterior_builder='auto')
        b = tpe.suggest([new_id], dom, trials, 100 + step, posterior_builder='host')
        assert a[0]['misc']['vals'] == b[0]['misc']['vals'], step
        # finish the suggested trial with a loss that ties the split boundary
        doc = a[0]
        doc['state'] = 2
        doc['result'] = {'status': 'ok', 'loss': -5.0 if step % 2 else float(step)}
        trials.insert_trial_docs(a)
        trials.refresh()
    up = get_engine(0, 'f64')._history_uploader
    assert up.tie_labels, 'the device path did not run'


def test_label_subset_rebuild_equals_full_rebuild():
    """tpe_rebuild_labels (posterior.build_reference_order's second build
    when no loss tie straddles the split): rebuilding only the labels whose
    mixtures needed numpy's order gives the mixtures, records and round
    results of the full ordered rebuild, and the host build's mixtures; a
    rebuild after an append, or with different arguments, is refused."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.engine import Engine, EngineError
    hist = coarse_history(6000, seed=3, split_tie=False)
    specs, cat, losses, off, tr, val = hist.device_inputs()
    n_valid = int(np.count_nonzero(losses == losses))
    n_below = P.n_below_of(n_valid, 0.25, 25)
    out = []
    for subset in (False, True):
        eng = Engine(0, 'f64')
        eng.history_reset(specs, cat)
        eng.history_append(np.diff(off), tr, val)
        nb, ties = eng.build_posterior_ordered(losses, n_valid, 0.25, 1.0, 25)
        assert not ties[-1]
        need = set(np.flatnonzero(ties[:-1] & 2).tolist())
        assert need and len(need) < len(hist.labels)
        below, o_off, order = P.reference_orders(losses, n_below, P._ObsOf(off, tr, val), need)
        if subset:
            nb2, ties2 = eng.rebuild_labels(losses, n_valid, 0.25, 1.0, 25, o_off, order, need)
            with pytest.raises(EngineError):   # different arguments
                eng.rebuild_labels(losses, n_valid, 0.3, 1.0, 25, o_off, order, need)
            changed = losses.copy()            # one loss changed, same length
            changed[int(np.flatnonzero(changed == changed)[0])] += 1.0
            with pytest.raises(EngineError):
                eng.rebuild_labels(changed, n_valid, 0.25, 1.0, 25, o_off, order, need)
        else:
            nb2, ties2 = eng.build_posterior_ordered(losses, n_valid, 0.25, 1.0, 25, below, o_off, order)
        assert nb2 == nb and not np.any(ties2)
        _assert_same(eng, hist, hist.posteriors())
        mix = [eng.get_mixture(li, side) for li in range(len(hist.labels)) for side in (0, 1)]
        res = eng.suggest(5, 1 << 16, round=2)
        out.append((mix, np.ascontiguousarray(res).tobytes()))
        if subset:   # after an append the kept state is stale: refused
            eng.history_append(np.zeros(len(hist.labels), dtype=np.int64), np.zeros(0, np.int32), np.zeros(0))
            with pytest.raises(EngineError):
                eng.rebuild_labels(losses, n_valid, 0.25, 1.0, 25, o_off, order, need)
        eng.close()
    (m0, r0), (m1, r1) = out
    assert r0 == r1
    for a, b in zip(m0, m1):
        assert all(np.array_equal(x, y) for x, y in zip(a, b))


@pytest.mark.parametrize('aux,first', [(1, 'round'), (0, 'round'), (1, 'mixture'), (1, 'batch')])
def test_deferred_rebuild_report(aux, first):
    """A subset rebuild of quantized labels whose report is deferred
    (TPE_OPT_DEFER_REPORT, Engine.rebuild_labels(defer=True)): it returns
    zero ties, the next call on the context applies the report -- a round
    after queuing the dense labels' kernels (aux families on), or any other
    call first -- and the round, the mixtures and build_report()'s ties are
    those of the rebuild that waited."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(32, 4000, seed=2)
    specs, cat, losses, off, tr, val = hist.device_inputs()
    n_valid = int(np.count_nonzero(losses == losses))
    n_below = P.n_below_of(n_valid, 0.25, 25)
    out = []
    for defer in (False, True):
        eng = Engine(0, 'f64')
        eng.set_option('aux_families', aux)
        eng.history_reset(specs, cat)
        eng.history_append(np.diff(off), tr, val)
        eng.arm_prepare(1 << 16, 1)
        nb, ties = eng.build_posterior_ordered(losses, n_valid, 0.25, 1.0, 25)
        need = set(np.flatnonzero(ties[:-1] & 2).tolist())
        assert need and all(hist.labels[l][1].startswith('q') for l in need)
        _, o_off, order = P.reference_orders(losses, n_below, P._ObsOf(off, tr, val), need)
        nb2, ties2 = eng.rebuild_labels(losses, n_valid, 0.25, 1.0, 25, o_off, order, need, defer=defer)
        if defer:
            assert not np.any(ties2)
        if first == 'mixture':
            mix = [eng.get_mixture(li, side) for li in sorted(need) for side in (0, 1)]
            res = eng.suggest(5, 1 << 16, round=2)
        elif first == 'batch':
            res = eng.suggest_batch(5, list(range(64)), 24)
            mix = [eng.get_mixture(li, side) for li in sorted(need) for side in (0, 1)]
        else:
            res = eng.suggest(5, 1 << 16, round=2)
            mix = [eng.get_mixture(li, side) for li in sorted(need) for side in (0, 1)]
        nb3, ties3 = eng.build_report()
        assert nb3 == nb2 == nb and not np.any(ties3)
        res2 = eng.suggest(6, 1 << 16, round=3)   # (a second round: nothing left pending)
        out.append((mix, np.ascontiguousarray(res).tobytes(), np.ascontiguousarray(res2).tobytes()))
        eng.close()
    (m0, r0, s0), (m1, r1, s1) = out
    assert r0 == r1 and s0 == s1
    for a, b in zip(m0, m1):
        assert all(np.array_equal(x, y) for x, y in zip(a, b))


@pytest.mark.parametrize('n_trials,tie', [(40000, False), (40000, True), (70000, True), (200000, False)])
def test_split_over_slices(n_trials, tie):
    """Histories past 16k trials take k_split in slices of 16 Ki losses
    (each slice's n_below + 1 smallest (loss, position) pairs, merged by
    one workgroup): the below set is the reference's when no tie straddles
    the n_below boundary (the mixtures equal the host build's), and a tie
    there is reported (ties[-1]) -- the product then supplies numpy's below
    set and again matches the host build."""
    from hyperopt_amd.engine import Engine
    hist = coarse_history(n_trials, seed=7, split_tie=False)
    if tie:   # 15 trials at -6, 20 at -5: n_below = 25 takes 10 of the 20
        rng = np.random.RandomState(1)
        pick = rng.permutation(n_trials)[:35]
        hist.losses[pick[:15]] = -6.0
        hist.losses[pick[15:]] = -5.0
    inputs = hist.device_inputs()
    eng = Engine(0)
    try:
        eng.history_reset(inputs[0], inputs[1])
        eng.history_append(np.diff(inputs[3]), inputs[4], inputs[5])
        nb, ties = eng.build_posterior_ordered(hist.losses, len(hist.losses), 0.25, 1.0)
        assert nb == 25 and ties[-1] == (1 if tie else 0), (nb, ties[-1])
        nb = eng.build_posterior(*inputs, gamma=0.25, prior_weight=1.0)
        assert nb == 25
        _assert_same(eng, hist, hist.posteriors())
    finally:
        eng.close()
