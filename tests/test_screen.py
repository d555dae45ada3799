"""The fp32 screen of the fp64 round (tpe_engine.hip k_screen / k_select /
k_rescore): every dense candidate is scored in packed fp32 with a rigorous
error bound, and only the candidates whose bound interval reaches the
round's largest lower bound are re-scored in fp64.

* the bound holds: |score32 - score64| <= bound for every candidate of a
  config-3 posterior (sampled, far-tail and boundary candidates), where
  score64 is the plain fp64 path (tpe_score);
* the screened round is the fp64 round: winners, values, scores and lpdfs
  are bit-identical with the screen on and off (configs 2, 3 and 4, host and
  device posteriors, a posterior whose candidates all fail certification).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dense_labels(posts):
    return [i for i, p in enumerate(posts) if p.family != 'categorical' and p.q is None]


@pytest.fixture(scope='module')
def eng():
    from hyperopt_amd.engine import Engine
    e = Engine(0, 'f64')
    yield e
    e.close()


@pytest.mark.parametrize('expand,window,win_t', [(1, 1, 16), (0, 1, 40), (0, 1, 16), (0, 1, 8),
                                                  (0, 0, 16)])
def test_screen_bound_holds(eng, expand, window, win_t):
    """expand=1: the probe goes through the expansion screen (fp64 score
    from the bin's Taylor polynomial + list, bound ~1e-12).
    window=1: the probe goes through the windowed screen (candidates
    sorted into tiles of neighbours, components outside a tile's window left
    out and covered by the bound's skip term); at win_t = 16 (the default)
    and 8 the terms left out reach 2^-16 / 2^-8 of the largest, where the
    per-bin skipped-mass bound carries real weight (at 8 it is the rigour,
    not the certification rate, that is checked)."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(32, 10000, seed=0)
    posts = hist.posteriors()
    eng.set_posterior(*P.pack(posts))
    worst, cert, emax = 0.0, [], 0.0
    for li in _dense_labels(posts):
        p = posts[li]
        samp = eng.GMM1 if p.family == 'GMM1' else eng.LGMM1
        x = samp(*p.below, low=p.low, high=p.high, q=None, seed=11, size=(20000,), stream=li)
        # plus far tails and the bounds themselves
        if p.family == 'GMM1':
            lo, hi = (p.low, p.high) if p.low is not None else (-30.0, 30.0)
            extra = np.concatenate([np.linspace(lo, hi, 2001), [lo, hi, 0.0, 1e-9]])
        else:
            extra = np.exp(np.linspace(p.low, p.high, 2001))
        x = np.concatenate([x, extra])
        eng.set_option('expand', expand)
        eng.set_option('window', window)
        eng.set_option('win_t', win_t)
        try:
            s32, err = eng.screen_probe(li, x)
        finally:
            eng.set_option('expand', 1)
            eng.set_option('window', 1)
            eng.set_option('win_t', 16)
        lb, la, _ = eng.score(li, x)
        s64 = lb - la
        ok = np.isfinite(err) & np.isfinite(s64)
        cert.append(ok.mean())
        emax = max(emax, float(np.median(err[ok])))
        assert np.all(np.abs(s32[ok] - s64[ok]) <= err[ok]), li
        worst = max(worst, float(np.max(np.abs(s32[ok] - s64[ok]) / err[ok])))
    # the bound is rigorous, and (but for T = 8, where the skipped mass is a
    # real share of the fp32 error) not tight
    assert worst < (1.0 if win_t < 16 else 0.5), worst
    if win_t >= 16:
        assert min(cert) > 0.9, cert
    if expand:   # fp64-accurate: the bound is ~1e-12, not ~1e-6
        assert emax < 1e-9, emax
    print('screen bound (expand %d, window %d, T %d): worst |s - s64| / bound = %.3g, '
          'certified %.4f..%.4f' % (expand, window, win_t, worst, min(cert), max(cert)))


def _suggest_both(eng, C, rnd, seed):
    eng.set_option('screen', 1)
    a = eng.suggest(seed, C, round=rnd)
    screened, rescored = eng.last_screen()
    _suggest_both.hot = eng.last_hot()        # (of the screened round: the next one resets it)
    eng.set_option('screen', 0)
    b = eng.suggest(seed, C, round=rnd)
    assert eng.last_screen() == (0, 0)
    eng.set_option('screen', 1)
    return a, b, screened, rescored


def _assert_same(a, b):
    for f in ('index', 'value', 'score', 'lpdf_below', 'lpdf_above', 'label'):
        assert np.array_equal(a[f], b[f], equal_nan=f != 'index' and f != 'label'), f


def test_screened_round_is_the_fp64_round_at_2_24(eng):
    """The bench's own size: config 3 as fmin's loop builds it (device build
    with numpy's tie order), 2^24 candidates per label -- the hot-bin
    prefilter, the expansion index, the early exits and the near-tie fp64
    re-scores against the plain fp64 round, bytewise, on two seeds."""
    from hyperopt_amd.workloads import FminLoop, mixed_history
    hist = mixed_history(32, 10001, seed=0)
    loop = FminLoop(hist)
    loop.advance(eng, 10000)
    loop.advance(eng, 10001, n_candidates=1 << 24)
    for rnd, seed in ((3, 1237), (4, 1238)):
        a, b, screened, rescored = _suggest_both(eng, 1 << 24, rnd, seed)
        assert np.ascontiguousarray(a).tobytes() == np.ascontiguousarray(b).tobytes()
        assert screened == 20 * (1 << 24) and 0 < rescored < screened // 1000
        assert _suggest_both.hot[0] > 0            # the hot-bin prefilter ran


@pytest.mark.parametrize('config', ['config2', 'config3', 'config3_device', 'config4_device',
                                    'hartmann_n30'])
def test_screened_round_is_the_fp64_round(eng, config):
    """C = 2^20 and 2^16 go through the windowed screen, 3000 and 5000
    through the plain one; hartmann_n30 (30 trials: wide components, few
    narrow ones) exercises the wide list."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import conditional_history, hartmann_history, mixed_history
    if config == 'config2':
        hist = hartmann_history(2000, seed=0)
    elif config == 'hartmann_n30':
        hist = hartmann_history(30, seed=3)
    elif config.startswith('config4'):
        hist = conditional_history(5000, seed=0)
    else:
        hist = mixed_history(32, 10000, seed=0)
    if config.endswith('device'):
        eng.build_posterior(*hist.device_inputs(), gamma=0.25, prior_weight=1.0)
    else:
        eng.set_posterior(*P.pack(hist.posteriors()))
    fracs = []
    for rnd, (C, seed) in enumerate([(1 << 20, 5), (3000, 6), (1 << 16, 7), (5000, 8)]):
        a, b, screened, rescored = _suggest_both(eng, C, rnd, seed)
        _assert_same(a, b)
        assert screened > 0 and 0 < rescored <= screened
        fracs.append(rescored / screened)
    print('%s: re-scored fraction per round %s' % (config, ['%.4f' % f for f in fracs]))


def test_screen_uncertified_candidates(eng):
    """A posterior whose above mixture sits thousands of sigmas away from
    every candidate: the fp32 sums underflow, nothing is certified, every
    candidate is re-scored and the round is still the fp64 round."""
    from hyperopt_amd import posterior as P
    lp = [P.LabelPosterior('far', 'GMM1',
                           (np.array([1.0]), np.array([0.0]), np.array([0.01])),
                           (np.array([0.5, 0.5]), np.array([-50.0, 50.0]), np.array([0.01, 0.01])),
                           low=None, high=None, q=None),
          P.LabelPosterior('near', 'GMM1',
                           (np.array([0.5, 0.5]), np.array([0.0, 1.0]), np.array([0.3, 0.2])),
                           (np.array([1.0]), np.array([0.5]), np.array([2.0])),
                           low=-3.0, high=3.0, q=None)]
    eng.set_posterior(*P.pack(lp))
    a, b, screened, rescored = _suggest_both(eng, 1 << 14, 3, 21)
    _assert_same(a, b)
    # label 0: all 2^14 re-scored; label 1: a few
    assert rescored >= (1 << 14) and rescored < screened


@pytest.mark.parametrize('rounds,C,chunks', [(512, 24, 0), (4096, 24, 0), (300, 24, 1),
                                             (64, 100, 0), (40, 700, 3)])
def test_screened_packed_rounds_are_the_fp64_rounds(eng, rounds, C, chunks):
    """Batched rounds with small C (the packed map; config 5's shape) --
    chunked or not -- screened and unscreened give identical winners and
    lpdfs."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(128, 50000, seed=0) if rounds >= 4096 else mixed_history(64, 20000, seed=1)
    eng.set_posterior(*P.pack(hist.posteriors()))
    eng.set_option('chunks', chunks)
    try:
        ids = list(range(7000, 7000 + rounds))
        eng.set_option('screen', 1)
        a = eng.suggest_batch(31, ids, C)
        screened, rescored = eng.last_screen()
        eng.set_option('screen', 0)
        b = eng.suggest_batch(31, ids, C)
        eng.set_option('screen', 1)
    finally:
        eng.set_option('chunks', 0)
    _assert_same(a, b)
    assert screened > 0 and rescored < screened
    print('packed %d x %d (chunks %d): re-scored %.4f' % (rounds, C, chunks, rescored / screened))


def test_packed_rescore_zero_windows_same_bits(eng):
    """Config 5 (128 labels, N = 50k, 4096 rounds x 24): the packed
    re-score summing only the above components whose fp64 terms can be
    nonzero at the wave's candidates (TPE_OPT_ZERO_WIN, k_zero_windows)
    gives the bytes of the full sums -- and of the unscreened round."""
    from hyperopt_amd.workloads import FminLoop, mixed_history
    hist = mixed_history(128, 50000, seed=0)
    FminLoop(hist).advance(eng, 50000)
    ids = list(range(9000, 9000 + 4096))
    out = {}
    for zw, screen in ((1, 1), (0, 1), (1, 0)):
        eng.set_option('zero_win', zw)
        eng.set_option('screen', screen)
        out[(zw, screen)] = np.ascontiguousarray(eng.suggest_batch(77, ids, 24)).tobytes()
    eng.set_option('zero_win', 1)
    eng.set_option('screen', 1)
    assert out[(1, 1)] == out[(0, 1)] == out[(1, 0)]


@pytest.mark.parametrize('value_only', [0, 1])
@pytest.mark.parametrize('rounds,chunks', [(128, 0), (96, 3), (600, 0)])
def test_packed_rescore_sliced_same_bits(eng, value_only, rounds, chunks):
    """The packed map's re-score of a few listed candidates split by
    summation slices (TPE_OPT_PK_SLICED: one wave per 64 candidates and
    slice, the chunk sums added in the chunked map's order) gives the bytes
    of the one-thread-per-candidate re-score (and, with lpdfs, of the
    unscreened round); value_only 0 re-scores every cell's winner (a few thousand candidates:
    sliced at 128 and 96 rounds, chunked at 600 by default)."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(64, 20000, seed=1)
    eng.set_posterior(*P.pack(hist.posteriors()))
    ids = list(range(3000, 3000 + rounds))
    out, counts = {}, {}
    eng.set_option('value_only', value_only)
    eng.set_option('chunks', chunks)
    try:
        # sliced before the posterior's zero windows exist, chunked (builds
        # them), sliced inside them, unscreened
        for pk, screen in ((8192, 1), (0, 1), (65536, 1), (8192, 0)):
            eng.set_option('pk_sliced', pk)
            eng.set_option('screen', screen)
            out[(pk, screen)] = np.ascontiguousarray(eng.suggest_batch(41, ids, 24)).tobytes()
            counts[(pk, screen)] = eng.last_screen()
    finally:
        eng.set_option('pk_sliced', 8192)
        eng.set_option('screen', 1)
        eng.set_option('chunks', 0)
        eng.set_option('value_only', 0)
    assert out[(0, 1)] == out[(8192, 1)] == out[(65536, 1)]
    if not value_only:   # (value-only cells the screen decided carry no lpdfs)
        assert out[(8192, 1)] == out[(8192, 0)]
    rescored = counts[(65536, 1)][1]
    assert rescored > 0 or (value_only and rounds == 600)   # (none left there)
    if not value_only:
        assert rescored >= rounds   # (every cell's winner)
    print('packed %d rounds, value_only %d: re-scored %d' % (rounds, value_only, rescored))


def test_windowed_screen_skips_terms(eng):
    """Config 3's posterior, 2^20 candidates: the windowed screen sums a
    fraction of the terms the plain screen sums, and both give the fp64
    round's winners bit for bit."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(32, 10000, seed=0)
    eng.build_posterior(*hist.device_inputs(), gamma=0.25, prior_weight=1.0)
    C = 1 << 20
    eng.set_option('expand', 0)
    try:
        eng.set_option('window', 1)
        a = eng.suggest(9, C, round=2)
        terms_w = eng.last_screen_terms()
        eng.set_option('window', 0)
        b = eng.suggest(9, C, round=2)
        terms_p = eng.last_screen_terms()
        eng.set_option('window', 1)
        eng.set_option('screen', 0)
        c = eng.suggest(9, C, round=2)
        eng.set_option('screen', 1)
    finally:
        eng.set_option('expand', 1)
    _assert_same(a, c)
    _assert_same(b, c)
    frac = terms_w / terms_p
    print('windowed screen: %.4f of the plain screen\'s terms' % frac)
    assert 0 < frac < 0.35


@pytest.mark.parametrize('groups', [0, 3, 5])
def test_windowed_screen_batched_rounds(eng, groups):
    """Several tile-map rounds in one call (grid.z): keys carry the round,
    so each round's candidates are sorted and selected on their own.
    groups > 0: the labels in that many groups, each keyed and sorted on the
    second stream while the previous group is screened (two buffer slots,
    so 3 and 5 groups reuse them)."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(24, 6000, seed=4)
    eng.set_posterior(*P.pack(hist.posteriors()))
    ids = [11, 12, 13]
    eng.set_option('win_groups', groups)
    try:
        a = eng.suggest_batch(5, ids, 1 << 15)
        screened, rescored = eng.last_screen()
        eng.set_option('screen', 0)
        b = eng.suggest_batch(5, ids, 1 << 15)
        eng.set_option('screen', 1)
    finally:
        eng.set_option('win_groups', 0)
    _assert_same(a, b)
    assert 0 < rescored < screened


@pytest.mark.parametrize('config', ['config3', 'config3_device', 'config2', 'config4_device'])
def test_expansion_screen_rescores_near_ties_only(eng, config):
    """The expansion screen's bound is ~1e-12: at 2^20 candidates per label
    only the near-ties of each label's best score are re-scored (a handful
    per label, against ~0.2 % with the fp32 screens), it sums a few dozen
    direct terms per candidate, and the round is the fp64 round bit for bit
    -- as is the windowed screen's round on the same candidates."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import conditional_history, hartmann_history, mixed_history
    if config == 'config2':
        hist = hartmann_history(2000, seed=0)
    elif config.startswith('config4'):
        hist = conditional_history(5000, seed=0)
    else:
        hist = mixed_history(32, 10000, seed=0)
    if config.endswith('device'):
        eng.build_posterior(*hist.device_inputs(), gamma=0.25, prior_weight=1.0)
    else:
        eng.set_posterior(*P.pack(hist.posteriors()))
    C = 1 << 20
    a = eng.suggest(13, C, round=4)
    screened, rescored = eng.last_screen()
    terms = eng.last_screen_terms()
    eng.set_option('expand', 0)
    try:
        w = eng.suggest(13, C, round=4)
        _, rescored_w = eng.last_screen()
    finally:
        eng.set_option('expand', 1)
    eng.set_option('screen', 0)
    b = eng.suggest(13, C, round=4)
    eng.set_option('screen', 1)
    _assert_same(a, b)
    _assert_same(w, b)
    n_dense = screened // C
    assert n_dense > 0
    print('%s: expansion screen re-scored %d of %d (windowed: %d), %.1f direct terms per '
          'candidate' % (config, rescored, screened, rescored_w, terms / screened))
    assert rescored <= 64 * n_dense, rescored
    assert rescored < rescored_w


@pytest.mark.parametrize('config', ['config3_device', 'config2', 'config4_device', 'config3_batched'])
def test_hot_prefilter_same_winners(eng, config):
    """Hot-bin prefilter (tpe_device.h "hot-bin prefilter"): every candidate
    is drawn and bounded by its sub-bin's score interval, only the ones that
    can still win go through the expansion screen.  The round is the fp64
    round bit for bit -- with the prefilter, without it, with the forced
    fallback (hot = 2: nothing listed, every candidate screened), and with
    the screen off -- and the prefilter lists a small part of the candidates."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import conditional_history, hartmann_history, mixed_history
    if config == 'config2':
        hist = hartmann_history(2000, seed=0)
    elif config.startswith('config4'):
        hist = conditional_history(5000, seed=0)
    else:
        hist = mixed_history(32, 10000, seed=0)
    if config.endswith('device'):
        eng.build_posterior(*hist.device_inputs(), gamma=0.25, prior_weight=1.0)
    else:
        eng.set_posterior(*P.pack(hist.posteriors()))
    C = 1 << 20
    run = (lambda: eng.suggest_batch(17, [5, 6, 7], C // 4)) if config.endswith('batched') else \
        (lambda: eng.suggest(17, C, round=5))
    a = run()
    listed, fb = eng.last_hot()
    screened, rescored = eng.last_screen()
    assert eng.last_screen_mode() == 3
    try:
        eng.set_option('hot', 0)
        b = run()
        assert eng.last_hot() == (-1, 0)
        eng.set_option('hot', 2)
        c = run()
        listed_c, fb_c = eng.last_hot()
    finally:
        eng.set_option('hot', 1)
    # lists far too short for the listed candidates: the round overflows
    # them and screens every candidate instead
    try:
        eng.set_option('hot_div', 1 << 20)
        e = run()
        _, fb_e = eng.last_hot()
    finally:
        eng.set_option('hot_div', 16)
    eng.set_option('screen', 0)
    d = run()
    eng.set_option('screen', 1)
    _assert_same(a, d)
    _assert_same(b, d)
    _assert_same(c, d)
    _assert_same(e, d)
    assert fb == 0 and fb_c == 1
    assert fb_e & 2 or listed <= 4096 * 32 * 3   # (batched: short rounds list fewer than a minimal list)
    print('%s: hot prefilter listed %d of %d (%.4f), re-scored %d' %
          (config, listed, screened, listed / screened, rescored))
    assert 0 < listed < 0.25 * screened


def test_hot_bounds_hold(eng):
    """The hot-bin prefilter's table: lower <= score64 <= upper over each
    candidate's sub-bin (sampled candidates, a grid over the whole range,
    far tails), score64 from the plain fp64 path (tpe_score); the intervals
    are narrow near each label's best score (the prefilter lists few)."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(32, 10000, seed=0)
    posts = hist.posteriors()
    eng.set_posterior(*P.pack(posts))
    for li in _dense_labels(posts):
        p = posts[li]
        samp = eng.GMM1 if p.family == 'GMM1' else eng.LGMM1
        x = samp(*p.below, low=p.low, high=p.high, q=None, seed=12, size=(50000,), stream=li)
        if p.family == 'GMM1':
            lo, hi = (p.low, p.high) if p.low is not None else (-30.0, 30.0)
            extra = np.concatenate([np.linspace(lo, hi, 20001), [lo, hi, 0.0, 1e-9]])
        else:
            extra = np.exp(np.linspace(p.low, p.high, 20001))
        x = np.concatenate([x, extra])
        u, l, m = eng.hot_probe(li, x)
        lb, la, _ = eng.score(li, x)
        s64 = lb - la
        fin = np.isfinite(s64)
        assert np.all(l[fin] <= s64[fin]) and np.all(s64[fin] <= u[fin]), li
        ns = 50000
        tau = np.max(l[:ns])
        hot = np.mean(u[:ns] >= tau)
        w = u[:ns] - l[:ns]
        tau0 = np.max(np.where(m[:ns] >= 64.0 / (1 << 20), l[:ns], -np.inf))
        print('label %d (%s): tau %.6f tau0(2^20) %.6f best %.6f, hot %.5f, median width %.3g, '
              'mass at best %.3g, mean mass %.3g' %
              (li, p.family, tau, tau0, np.max(s64[:ns]), hot, np.median(w[np.isfinite(w)]),
               m[np.argmax(s64[:ns])], np.mean(m[:ns])))
        assert hot < 0.02, (li, hot)


@pytest.mark.parametrize('split', [3, 8, 0])
def test_index_window_split_same_round(eng, split):
    """k_bx_table's split window (TPE_OPT_BX_SPLIT: the bins' component
    window summed by several workgroups, the parts added by k_bx_table_fin):
    the Taylor rows round differently, the winners do not -- the round equals
    the unsplit index's bytewise, and the sub-bin bounds built on the split
    rows still bracket the fp64 score."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(32, 10000, seed=0)
    packed = P.pack(hist.posteriors())
    posts = hist.posteriors()
    C = 1 << 20
    try:
        eng.set_option('bx_split', 1)
        eng.set_posterior(*packed)
        a = eng.suggest(23, C, round=4)
        eng.set_option('bx_split', split)
        eng.set_posterior(*packed)
        b = eng.suggest(23, C, round=4)
        for li in (0, 1, 3):
            p = posts[li]
            samp = eng.GMM1 if p.family == 'GMM1' else eng.LGMM1
            x = samp(*p.below, low=p.low, high=p.high, q=None, seed=3, size=(20000,), stream=li)
            u, l, _ = eng.hot_probe(li, x)
            lb, la, _ = eng.score(li, x)
            s64 = lb - la
            fin = np.isfinite(s64)
            assert np.all(l[fin] <= s64[fin]) and np.all(s64[fin] <= u[fin]), li
    finally:
        eng.set_option('bx_split', 0)
    _assert_same(a, b)


@pytest.mark.parametrize('cut', [48, 96, 128])
def test_index_cut_same_round(eng, cut):
    """The expansion index's window cut T (TPE_OPT_BX_T; auto: 64): fewer or more components in a bin's
    window and its bound's skipped mass na 2^-T -- the winners do not move,
    and the sub-bin bounds of the forced-T index still bracket the fp64
    score."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import mixed_history
    hist = mixed_history(32, 10000, seed=0)
    packed = P.pack(hist.posteriors())
    posts = hist.posteriors()
    C = 1 << 20
    try:
        eng.set_option('bx_t', 0)
        eng.set_posterior(*packed)
        a = eng.suggest(29, C, round=6)
        eng.set_option('bx_t', cut)
        eng.set_posterior(*packed)
        b = eng.suggest(29, C, round=6)
        for li in (0, 1, 3):
            p = posts[li]
            samp = eng.GMM1 if p.family == 'GMM1' else eng.LGMM1
            x = samp(*p.below, low=p.low, high=p.high, q=None, seed=4, size=(20000,), stream=li)
            u, l, _ = eng.hot_probe(li, x)
            lb, la, _ = eng.score(li, x)
            s64 = lb - la
            fin = np.isfinite(s64)
            assert np.all(l[fin] <= s64[fin]) and np.all(s64[fin] <= u[fin]), li
    finally:
        eng.set_option('bx_t', 0)
    _assert_same(a, b)
