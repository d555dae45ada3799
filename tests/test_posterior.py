"""The product's host descriptor builder (hyperopt_amd/posterior.py) must
reproduce the reference's split and Parzen mixtures bit-for-bit on the
golden vectors (CPU only)."""
import numpy as np
import pytest

from hyperopt_amd import posterior as P
from tests import golden_io


@pytest.mark.parametrize('fixture', ['labels_small.npz', 'labels_medium.npz'])
def test_posterior_bit_exact(fixture):
    n = 0
    for meta, rec in golden_io.cases(fixture):
        bt, at = P.split_history(rec['l_idxs'], rec['l_vals'], meta['gamma'])
        below, above = P.split_label(rec['o_idxs'], rec['o_vals'], bt, at)
        assert np.array_equal(np.asarray(below, float), rec['below'])
        assert np.array_equal(np.asarray(above, float), rec['above'])
        post = P.label_posterior('x', meta['kind'], meta['args'], below, above,
                                 meta['prior_weight'])
        if post.family == 'categorical':
            assert np.array_equal(post.below, rec['p_below'])
            assert np.array_equal(post.above, rec['p_above'])
        else:
            assert post.family == meta['sampler']
            for tag, trip in (('b', post.below), ('a', post.above)):
                w, m, s = trip
                assert np.array_equal(w, rec['w_' + tag]), (meta['kind'], meta['n_hist'])
                assert np.array_equal(m, rec['mu_' + tag])
                assert np.array_equal(s, rec['sigma_' + tag])
            kw = meta['lpdf_kwargs']
            assert post.low == kw.get('low') and post.high == kw.get('high')
            assert post.q == kw.get('q')
        n += 1
    assert n > 0


def test_pack_layout():
    from hyperopt_amd import _lib as L
    posts = [P.LabelPosterior('a', 'GMM1', ([.5, .5], [0., 1.], [1., 1.]),
                              ([1.], [0.], [2.]), low=-1.0, high=2.0),
             P.LabelPosterior('b', 'categorical', np.array([.2, .8]), np.array([.5, .5]),
                              upper=2),
             P.LabelPosterior('c', 'LGMM1', ([1.], [0.], [1.]), ([1.], [0.], [1.]), q=2.0)]
    d, w, m, s = P.pack(posts)
    assert list(d['kind']) == [L.TPE_GMM1, L.TPE_CATEGORICAL, L.TPE_LGMM1]
    assert list(d['flags']) == [3, 0, 4]
    assert list(d['below_off']) == [0, 3, 7] and list(d['above_off']) == [2, 5, 8]
    assert list(d['n_below']) == [2, 2, 1] and len(w) == 9
    assert np.array_equal(w[3:7], [.2, .8, .5, .5])


@pytest.mark.parametrize('fixture', ['labels_small.npz', 'labels_medium.npz'])
def test_splitter_equals_split_label(fixture):
    """The binary-search Splitter used by tpe.suggest gives the reference's
    split (same as the np.isin form pinned above)."""
    for meta, rec in golden_io.cases(fixture):
        sp = P.Splitter(rec['l_idxs'], rec['l_vals'], meta['gamma'])
        b, a = sp.split(rec['o_idxs'], rec['o_vals'])
        assert np.array_equal(np.asarray(b, float), rec['below'])
        assert np.array_equal(np.asarray(a, float), rec['above'])


def test_spec_table_streams_and_label_subsets():
    """A label subset (a label-sharded rank) keeps each label's Philox
    stream: spec_table sets TPE_HAS_STREAM and the space index; without
    streams the flag is clear (the device uses the position).  FminLoop's
    view of a subset holds only its labels' observations."""
    from hyperopt_amd import _lib as L
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import FminLoop, mixed_history
    hist = mixed_history(10, 50, seed=1)
    specs, _, _ = P.spec_table(hist.labels)
    assert not np.any(specs['flags'] & L.TPE_HAS_STREAM)
    ids = [1, 4, 7]
    specs, _, _ = P.spec_table([hist.labels[i] for i in ids], streams=ids)
    assert np.all(specs['flags'] & L.TPE_HAS_STREAM)
    assert list(specs['stream']) == ids
    loop = FminLoop(hist, label_ids=ids)
    assert loop.streams == ids and [n for n, _, _ in loop.labels] == [hist.labels[i][0] for i in ids]
    tids, losses, n_valid, obs, owner = loop.view(30)
    assert set(obs) == {hist.labels[i][0] for i in ids} and len(tids) == 30 and owner is loop
    assert all(len(obs[n][0]) == 30 for n in obs)


class _RecordingEngine(object):
    """Captures what DeviceHistoryUploader uploads (no device)."""
    history_generation = 0

    def __init__(self):
        self.appends = []

    def history_reset(self, specs, cat_p):
        self.appends.append(None)

    def history_append(self, n_new, trial, vals):
        self.appends.append((np.array(n_new), np.array(trial), np.array(vals)))


def test_uploader_vectorised_append_matches_per_label_transforms(monkeypatch):
    """The uploader transforms and places the new observations of every
    label in one pass: per label the values equal the reference's own
    transform of that label's new observations (np.log, np.log(np.maximum(o,
    floor)) for q-log kinds, identity), positions are the trials' rows, and
    a NaN names its label."""
    from hyperopt_amd import posterior as P
    from hyperopt_amd.workloads import FminLoop, conditional_history, mixed_history
    monkeypatch.setattr(P, 'build_reference_order', lambda *a, **k: (0, frozenset()))
    for hist in (mixed_history(12, 700, seed=0), conditional_history(600, seed=1)):
        eng = _RecordingEngine()
        up, loop = P.DeviceHistoryUploader(), FminLoop(hist)
        steps = [(0, 500), (500, 501), (501, 540)]
        for _, n in steps:
            up.build(eng, hist.labels, loop.view(n), 0.25, 1.0)
        _, _, trs = P.spec_table(hist.labels)
        got = [a for a in eng.appends if a is not None]
        assert len(got) == len(steps)
        for (n_new, trial, vals), (n0, n1) in zip(got, steps):
            o = 0
            for i, (name, _, _) in enumerate(hist.labels):
                oi, ov = hist.obs[name]
                sel = (oi >= n0) & (oi < n1)
                want = ov[sel] if trs[i] is None else trs[i](ov[sel])
                m = int(sel.sum())
                assert n_new[i] == m
                assert np.array_equal(vals[o:o + m], np.asarray(want, dtype=float))
                assert np.array_equal(trial[o:o + m], np.flatnonzero(np.isin(hist.tids[:n1], oi[sel])))
                o += m
    # a NaN after the transform (log of a negative value) names its label
    hist = mixed_history(6, 50, seed=2)
    name = hist.labels[1][0]                       # loguniform
    oi, ov = hist.obs[name]
    hist.obs[name] = (oi, np.where(oi == 40, -1.0, ov))
    up, loop, eng = P.DeviceHistoryUploader(), FminLoop(hist), _RecordingEngine()
    up.build(eng, hist.labels, loop.view(30), 0.25, 1.0)
    with pytest.raises(P.NonFiniteObservation, match=name):
        up.build(eng, hist.labels, loop.view(45), 0.25, 1.0)


@pytest.mark.parametrize('n_trials', [300, 40000])
def test_reference_orders_matches_per_label_argsort(n_trials):
    """posterior.reference_orders (the tie orders the device build takes:
    gathers, argsorts and int32 stores in the sort pool past _POOL_MIN
    observations) equals a plain per-label np.argsort of the above
    observations in observation order (tpe.py:433), for labels observed in
    every trial and for conditional labels (some trials without the label,
    a trial position of -1, NaN losses)."""
    rng = np.random.RandomState(5)
    T = n_trials
    losses = np.round(rng.normal(size=T), 1)
    losses[rng.rand(T) < 0.05] = np.nan
    offs, trials, vals = [0], [], []
    for l in range(6):
        if l % 2 == 0:   # in every trial, quantized (many ties)
            tr = np.arange(T, dtype=np.int32)
        else:            # conditional, with a trial of no position
            tr = np.sort(rng.choice(T, size=T // 3, replace=False)).astype(np.int32)
            tr[0] = -1
        v = np.round(rng.uniform(0, 20, size=len(tr)))
        trials.append(tr)
        vals.append(v)
        offs.append(offs[-1] + len(tr))
    off = np.asarray(offs, dtype=np.int64)
    tr_all, val_all = np.concatenate(trials), np.concatenate(vals)
    obs_of = P._ObsOf(off, tr_all, val_all)
    n_valid = int(np.count_nonzero(losses == losses))
    n_below = P.n_below_of(n_valid, 0.25, 25)
    labels = {0, 1, 3, 4}
    below, o_off, order = P.reference_orders(losses, n_below, obs_of, labels)
    above = (losses == losses) & (below == 0)
    assert int(below.sum()) == n_below
    for l in range(6):
        got = order[o_off[l]:o_off[l + 1]]
        if l not in labels:
            assert len(got) == 0
            continue
        tr, v = trials[l], vals[l]
        ok = (tr >= 0) & (tr < T)
        keep = np.zeros(len(tr), dtype=bool)
        keep[ok] = above[tr[ok]]
        want = np.argsort(v[keep])
        assert got.dtype == np.int32 and np.array_equal(got, want), l
