"""Device posterior builder (tpe_build_posterior, hyperopt_amd/csrc/tpe_build.hip)
against the CPU oracle's restatement of ap_filter_trials + adaptive_parzen_normal
+ the categorical pseudocount posteriors (tpe.py:385-477, 581-648).

Bar: the built (weights, mus, sigmas) are BIT-IDENTICAL to the oracle's in
the reference's own tie order (np.argsort's, sort_kind=None): the device
flags the mixtures that depend on the order of tied observations / losses and
the host supplies numpy's order for those (posterior.build_reference_order).
The position-order build (one tpe_build_posterior call, tie_order='position')
is bit-identical to the stable-order oracle (sort_kind='stable').  The folded
records are checked through a full suggestion round against the same
mixtures uploaded with tpe_set_posterior (host fold)."""
import numpy as np
import pytest

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu

ALL_KINDS = [
    ('u', 'uniform', dict(low=-5.0, high=5.0)),
    ('qu', 'quniform', dict(low=0.0, high=20.0, q=1.0)),
    ('lu', 'loguniform', dict(low=-5.0, high=2.0)),
    ('qlu', 'qloguniform', dict(low=0.0, high=4.0, q=1.0)),
    ('n', 'normal', dict(mu=0.0, sigma=3.0)),
    ('qn', 'qnormal', dict(mu=0.0, sigma=3.0, q=0.5)),
    ('ln', 'lognormal', dict(mu=0.0, sigma=1.0)),
    ('qln', 'qlognormal', dict(mu=1.0, sigma=1.0, q=1.0)),
    ('ri', 'randint', dict(upper=7)),
    ('pc', 'categorical', dict(upper=4, p=[0.1, 0.2, 0.3, 0.4])),
]


def make_history(labels, n_trials, seed, active_frac=1.0, loss_round=None, orphan=0):
    """Synthetic history: prior draws, each label active in a random subset,
    losses optionally rounded (ties), `orphan` observations whose tid has no
    loss entry (the reference drops them)."""
    from hyperopt_amd.workloads import History, prior_draw
    rng = np.random.RandomState(seed)
    tids = np.arange(n_trials, dtype=np.int64) * 3 + 5          # sparse, sorted tids
    losses = rng.normal(size=n_trials)
    if loss_round is not None:
        losses = np.round(losses, loss_round)
    obs = {}
    for name, kind, args in labels:
        act = tids[rng.uniform(size=n_trials) < active_frac] if active_frac < 1 else tids
        v = prior_draw(kind, args, rng, len(act))
        if orphan:
            extra = np.arange(orphan, dtype=np.int64) * 3 + 6        # never a trial tid
            act = np.concatenate([act, extra])
            v = np.concatenate([v, prior_draw(kind, args, rng, orphan)])
            o = np.argsort(act, kind='stable')
            act, v = act[o], v[o]
        obs[name] = (act, v)
    return History(labels, tids, losses, obs)


def oracle_mixtures(hist, gamma=0.25, pw=1.0, sort_kind=None):
    out = []
    for name, kind, args in hist.labels:
        oi, ov = hist.obs[name]
        r = O.label_posteriors(kind, args, oi, ov, hist.tids, hist.losses, gamma, pw,
                               sort_kind=sort_kind)
        if r[0] == 'CAT':
            out.append(((r[1],), (r[2],)))
        else:
            out.append((r[0][1:4], r[1][1:4]))
    return out


@pytest.fixture(scope='module')
def eng():
    from hyperopt_amd.engine import Engine
    e = Engine(0, 'f64')
    yield e
    e.close()


def _build(eng, hist, gamma=0.25, pw=1.0, tie_order='reference'):
    return eng.build_posterior(*hist.device_inputs(), gamma=gamma, prior_weight=pw, tie_order=tie_order)


def _check_bit_exact(eng, hist, want):
    for li, (name, kind, _) in enumerate(hist.labels):
        for side in (0, 1):
            w, m, s = eng.get_mixture(li, side)
            ref = want[li][side]
            if kind in ('randint', 'categorical'):
                assert np.array_equal(w, ref[0]), (name, side, w, ref[0])
            else:
                rw, rm, rs = ref
                assert len(w) == len(rw), (name, side, len(w), len(rw))
                assert np.array_equal(m, rm), (name, side, 'mus')
                assert np.array_equal(s, rs), (name, side, 'sigmas')
                assert np.array_equal(w, rw), (name, side, 'weights',
                                               np.max(np.abs(w - rw)))


@pytest.mark.parametrize('n_trials', [1, 2, 3, 25, 26, 27, 200, 3000])
def test_build_all_kinds_bit_exact(eng, n_trials):
    hist = make_history(ALL_KINDS, n_trials, seed=n_trials)
    nb = _build(eng, hist)
    assert nb == min(int(np.ceil(0.25 * np.sqrt(n_trials))), 25)
    _check_bit_exact(eng, hist, oracle_mixtures(hist))


@pytest.mark.parametrize('n_trials', [4095, 4097, 9000])
def test_build_categorical_bin_counts(eng, n_trials):
    """Categorical bincounts on both device paths -- ordered compaction by bin
    (upper <= 32, chunks of 4096) and wave-per-bin walks (upper > 32, chunks
    of 8192) -- across chunk boundaries, with empty bins: bit-exact."""
    labels = [('r2', 'randint', dict(upper=2)), ('r32', 'randint', dict(upper=32)),
              ('r33', 'randint', dict(upper=33)), ('r200', 'randint', dict(upper=200)),
              ('pc', 'categorical', dict(upper=6, p=[0.5, 0.0, 0.2, 0.1, 0.1, 0.1]))]
    hist = make_history(labels, n_trials, seed=n_trials, active_frac=0.9)
    _build(eng, hist)
    _check_bit_exact(eng, hist, oracle_mixtures(hist))


def test_build_conditional_ties_orphans(eng):
    """Labels active in subsets, tied losses, observations of trials without
    a loss entry (dropped from both sets, tpe.py:639-646)."""
    hist = make_history(ALL_KINDS, 1500, seed=7, active_frac=0.4, loss_round=1, orphan=17)
    _build(eng, hist)
    _check_bit_exact(eng, hist, oracle_mixtures(hist))
    assert eng.tie_labels                      # tied quantized labels took numpy's order


@pytest.mark.parametrize('n_trials', [200, 3000])
def test_build_position_order_is_stable_order(eng, n_trials):
    """tie_order='position' (tpe_build_posterior alone): ties by position,
    bit-identical to the stable-order oracle."""
    hist = make_history(ALL_KINDS, n_trials, seed=n_trials, loss_round=1)
    _build(eng, hist, tie_order='position')
    _check_bit_exact(eng, hist, oracle_mixtures(hist, sort_kind='stable'))


def test_build_matches_default_order_when_tie_free(eng):
    """Continuous kinds and distinct losses: the stable order IS numpy's
    order, so the build equals the reference's default-order mixtures."""
    labels = [l for l in ALL_KINDS if l[1] in ('uniform', 'loguniform', 'normal', 'lognormal')]
    hist = make_history(labels, 5000, seed=3)
    _build(eng, hist)
    _check_bit_exact(eng, hist, oracle_mixtures(hist, sort_kind=None))


@pytest.mark.parametrize('gamma,pw', [(0.25, 1.0), (0.5, 0.3), (0.1, 4.0)])
def test_build_gamma_prior_weight(eng, gamma, pw):
    hist = make_history(ALL_KINDS, 700, seed=11, active_frac=0.7)
    _build(eng, hist, gamma, pw)
    _check_bit_exact(eng, hist, oracle_mixtures(hist, gamma, pw))


def test_build_config3_and_round_matches_host_fold(eng):
    """Config-3 history (32 labels, 10k trials): bit-exact mixtures, then one
    fused round on the device-folded records against the same mixtures folded
    on the host (tpe_set_posterior): same winners, lpdfs within 1e-12."""
    from hyperopt_amd.engine import Engine
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(32, 10000, seed=0)
    _build(eng, hist)
    want = oracle_mixtures(hist)
    _check_bit_exact(eng, hist, want)
    res_dev = eng.suggest(seed=99, n_candidates=1 << 16, round=3)
    posts = []
    for li, (name, kind, args) in enumerate(hist.labels):
        b, a = (eng.get_mixture(li, 0), eng.get_mixture(li, 1))
        if kind in ('randint', 'categorical'):
            posts.append(P.LabelPosterior(name, 'categorical', b[0], a[0], upper=len(b[0])))
        else:
            spec, _, _ = P.label_spec(kind, args)
            fam = 'GMM1' if spec['kind'] == 0 else 'LGMM1'
            posts.append(P.LabelPosterior(name, fam, b, a, low=args.get('low'),
                                          high=args.get('high'), q=args.get('q')))
    e2 = Engine(0, 'f64')
    try:
        e2.set_posterior(*P.pack(posts))
        res_host = e2.suggest(seed=99, n_candidates=1 << 16, round=3)
    finally:
        e2.close()
    assert np.array_equal(res_dev['index'], res_host['index'])
    assert np.array_equal(res_dev['value'], res_host['value'])
    for f in ('lpdf_below', 'lpdf_above'):
        np.testing.assert_allclose(res_dev[f], res_host[f], rtol=1e-12, atol=1e-12)


def test_build_config5_scale_bit_exact(eng):
    """Config-5-sized history: 128 labels of config 3's
    kind pattern, N = 50k trials, losses rounded to one decimal so that ties
    straddle the split -- the sliced k_split (past 16k trials: slices of 16 Ki
    losses, k_split_merge) and every label's mixtures bit-identical to the
    oracle's (numpy's tie orders supplied where the device reports them)."""
    kinds = [('uniform', dict(low=-5.0, high=5.0)), ('loguniform', dict(low=-5.0, high=2.0)),
             ('quniform', dict(low=0.0, high=100.0, q=1.0)), ('normal', dict(mu=0.0, sigma=3.0)),
             ('randint', dict(upper=5))]
    labels = [('x%d' % i, kinds[i % 5][0], kinds[i % 5][1]) for i in range(128)]
    hist = make_history(labels, 50000, seed=5, active_frac=0.8, loss_round=1)
    nb = _build(eng, hist)
    assert nb == 25
    srt = np.sort(hist.losses)
    assert srt[nb - 1] == srt[nb]                # a loss tie straddles the split
    _check_bit_exact(eng, hist, oracle_mixtures(hist))
    assert eng.tie_labels                        # numpy's orders were needed and supplied


def test_build_errors(eng):
    from hyperopt_amd.engine import SPEC_DTYPE
    hist = make_history(ALL_KINDS[:1], 50, seed=1)
    specs, cat, losses, off, tr, val = hist.device_inputs()
    bad = specs.copy()
    bad[0]['low'], bad[0]['high'] = 1.0, 1.0
    with pytest.raises(ValueError, match='low >= high'):
        eng.build_posterior(bad, cat, losses, off, tr, val, 0.25, 1.0)
    bad = np.zeros(1, dtype=SPEC_DTYPE)
    bad[0]['kind'] = 9
    with pytest.raises(Exception):
        eng.build_posterior(bad, cat, losses, off, tr, val, 0.25, 1.0)


def test_resident_history_incremental(eng):
    """Device-resident history: observations appended in several batches
    (sorted per batch, merged into each label's value order) give, after
    every append, the same mixtures as the oracle on the history so far --
    with tied losses and values, conditional labels, pending trials (+inf)
    and NaN-loss trials (outside the history: their observations join
    neither set, as the reference drops such docs).  The 400 -> 1999 batch
    (~9.6k staged observations) takes the chip-wide two-sort path of the
    append (>= 4096), the others the per-label segmented sort."""
    from hyperopt_amd import posterior as P
    hist = make_history(ALL_KINDS, 2400, seed=21, active_frac=0.6, loss_round=1)
    losses = hist.losses.copy()
    losses[7] = np.inf
    losses[100] = np.nan
    losses[1500] = np.nan
    specs, cat_p, trs = P.spec_table(hist.labels)
    eng.history_reset(specs, cat_p)
    counts = [0] * len(hist.labels)
    held = [[np.zeros(0, np.int32), np.zeros(0)] for _ in hist.labels]

    def obs_of(l):
        return held[l][0], held[l][1]
    obs_of.n_labels = len(hist.labels)
    for cut in (30, 31, 400, 1999, 2400):
        n_new, tr_parts, val_parts = [], [], []
        for i, (name, kind, args) in enumerate(hist.labels):
            oi, ov = hist.obs[name]
            keep = oi < hist.tids[cut - 1] + 1
            oi, ov = oi[keep], ov[keep]
            ni, nv = oi[counts[i]:], ov[counts[i]:]
            if trs[i] is not None and len(nv):
                nv = trs[i](nv)
            tr_parts.append(np.searchsorted(hist.tids, ni).astype(np.int32))
            val_parts.append(np.asarray(nv, dtype=float))
            held[i] = [np.concatenate([held[i][0], tr_parts[-1]]), np.concatenate([held[i][1], val_parts[-1]])]
            n_new.append(len(ni))
            counts[i] = len(oi)
        eng.history_append(np.asarray(n_new), np.concatenate(tr_parts), np.concatenate(val_parts))
        lsub = losses[:cut]
        n_valid = int(np.count_nonzero(lsub == lsub))
        ok = lsub == lsub
        from hyperopt_amd.workloads import History
        sub = History(hist.labels, hist.tids[:cut][ok], lsub[ok],
                      {n: hist.obs[n] for n, _, _ in hist.labels})
        # position order, then the reference's order (the product path)
        eng.build_posterior_resident(lsub, n_valid, 0.25, 1.0)
        _check_bit_exact(eng, sub, oracle_mixtures(sub, sort_kind='stable'))
        P.build_reference_order(eng, lsub, n_valid, 0.25, 1.0, 25, obs_of)
        _check_bit_exact(eng, sub, oracle_mixtures(sub))


def test_rebuilds_are_deterministic(eng):
    """Rebuilding the same posterior (one-shot and resident, several times)
    gives identical records: the scores of a fixed candidate grid and a
    round's winners and lpdfs are bit-identical and finite (guards the
    block-level reductions of the builder against races)."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(12, 10000, seed=4)
    grid = {'uniform': np.linspace(-4.9, 4.9, 257), 'normal': np.linspace(-9, 9, 257),
            'loguniform': np.exp(np.linspace(-4.9, 1.9, 257)),
            'quniform': np.arange(0, 101, dtype=float), 'randint': np.arange(5, dtype=float)}
    ref = None
    specs, cat, losses, off, tr, val = hist.device_inputs()
    for it in range(5):
        if it % 2 == 0:
            _build(eng, hist)
        else:   # the resident history again, with the orders the last build needed
            P.build_reference_order(eng, losses, len(losses), 0.25, 1.0, 25, P._ObsOf(off, tr, val),
                                    eng.tie_labels)
        out = []
        for li, (name, kind, _) in enumerate(hist.labels):
            lb, la, _ = eng.score(li, grid[kind])
            assert np.all(np.isfinite(lb)) and np.all(np.isfinite(la)), (it, name)
            out.append(np.concatenate([lb, la]))
        r = eng.suggest(5, 24, round=77)
        out.append(r['lpdf_below'])
        out.append(r['lpdf_above'])
        out.append(r['index'].astype(float))
        if ref is None:
            ref = out
        else:
            for a, b in zip(ref, out):
                assert np.array_equal(a, b), it
