"""Batched suggestions, defined against sequential reference calls
(tpe.py:823-916 returns one document per call; pending trials enter later
calls as +inf losses, tpe.py:844-847; fmin queues up to max_queue_len,
fmin.py:193-202), plus the startup phase and the device-resident history's
bookkeeping (generation + owner identity, NaN observations)."""
import copy

import numpy as np
import pytest

import hyperopt_amd as H
from hyperopt_amd import hp, tpe

SPACE = {'a': hp.uniform('a', -3, 3), 'b': hp.loguniform('b', -2, 2),
         'c': hp.choice('c', [{'q': hp.quniform('q', 0, 10, 1)}, {'n': hp.normal('n', 0, 1)}])}


def _loss(d):
    return d['a'] ** 2 + np.log(d['b']) ** 2 + d['c'].get('q', 0.0) / 10 + d['c'].get('n', 0.0)


def _history(n, seed, algo=None):
    trials = H.Trials()
    H.fmin(_loss, SPACE, algo=algo or H.rand.suggest, max_evals=n, trials=trials,
           rstate=np.random.RandomState(seed))
    return trials


def _vals(docs):
    return [(d['tid'], d['misc']['vals']) for d in docs]


def test_startup_answers_every_new_id():
    """Fewer docs than n_startup_jobs: rand.suggest(new_ids) answers, one
    document per new_id (tpe.py:869-871) -- no GPU needed."""
    trials = _history(5, 1)
    dom = H.Domain(_loss, SPACE)
    docs = tpe.suggest([10, 11, 12], dom, trials, 42)
    assert [d['tid'] for d in docs] == [10, 11, 12]
    assert _vals(docs) == _vals(H.rand.suggest([10, 11, 12], dom, trials, 42))


def test_device_inputs_reject_nan_observation():
    from hyperopt_amd import posterior as P
    labels = [('b', 'loguniform', dict(low=-2.0, high=2.0))]
    tids = np.arange(3)
    obs = {'b': (tids, np.array([1.0, -1.0, 2.0]))}   # log(-1) = NaN
    with np.errstate(invalid='ignore'):
        with pytest.raises(P.NonFiniteObservation):
            P.device_inputs(labels, tids, np.zeros(3), obs)


@pytest.mark.gpu
def test_batch_true_is_independent_calls_on_the_same_trials():
    trials = _history(300, 2)
    dom = H.Domain(_loss, SPACE)
    ids = [1000, 1001, 1002, 1003, 1004]
    batch = tpe.suggest(ids, dom, trials, 77, batch=True)
    single = [tpe.suggest([i], dom, trials, 77)[0] for i in ids]
    assert _vals(batch) == _vals(single)


@pytest.mark.gpu
@pytest.mark.parametrize('builder', ['host', 'device'])
def test_batch_pending_is_sequential_calls_with_pending_docs(builder):
    trials = _history(300, 3)
    dom = H.Domain(_loss, SPACE)
    ids = [2000, 2001, 2002, 2003]
    batch = tpe.suggest(ids, dom, trials, 5, batch='pending', posterior_builder=builder)
    seq_trials = copy.deepcopy(trials)
    seq = []
    for i in ids:
        d = tpe.suggest([i], dom, seq_trials, 5, posterior_builder=builder)
        seq_trials.insert_trial_docs(d)          # pending: state new, no loss
        seq_trials.refresh()
        seq.extend(d)
    assert _vals(batch) == _vals(seq)
    # the first call sees no pending doc: it equals the batch=True one
    excl = tpe.suggest(ids, dom, trials, 5, batch=True, posterior_builder=builder)
    assert _vals(excl)[0] == _vals(batch)[0]
    # later calls see the earlier suggestions: with the first one inserted
    # (pending, loss +inf) every label it set has one more above component
    with_first = copy.deepcopy(trials)
    with_first.insert_trial_docs(batch[:1])
    with_first.refresh()
    _, _, p0 = tpe.build_posteriors(dom, trials)
    _, _, p1 = tpe.build_posteriors(dom, with_first)
    set_labels = [k for k, v in batch[0]['misc']['vals'].items() if v]
    for a, b in zip(p0, p1):
        if a.label in set_labels and a.family != 'categorical':
            assert len(b.above[0]) == len(a.above[0]) + 1, a.label


def test_batch_pending_startup_phase_draws_distinct_documents():
    """a 'pending' batch that starts in the startup phase gets the
    reference's rand.suggest(new_ids) documents (one RandomState(seed) over
    the ids: distinct draws), the documents batch=True returns -- not one
    identically seeded rand.suggest per id.  No GPU needed: every call stays
    in the startup phase."""
    trials = _history(5, 6)
    dom = H.Domain(_loss, SPACE)
    ids = [40, 41, 42, 43]
    pend = tpe.suggest(ids, dom, trials, 8, batch='pending')
    both = tpe.suggest(ids, dom, trials, 8, batch=True)
    assert _vals(pend) == _vals(both)
    a_vals = [d['misc']['vals']['a'][0] for d in pend]
    assert len(set(a_vals)) == len(a_vals)


@pytest.mark.gpu
def test_batch_pending_crossing_the_startup_phase():
    """a 'pending' batch that starts 2 documents short of
    n_startup_jobs: the first 2 ids are ONE rand.suggest(new_ids[:2]) call,
    the others sequential TPE calls that see every earlier suggestion of the
    batch as a pending trial."""
    trials = _history(18, 7)
    dom = H.Domain(_loss, SPACE)
    ids = [3000, 3001, 3002, 3003, 3004]
    pend = tpe.suggest(ids, dom, trials, 11, batch='pending')
    assert [d['tid'] for d in pend] == ids
    assert _vals(pend[:2]) == _vals(H.rand.suggest(ids[:2], dom, trials, 11))
    seq_trials = copy.deepcopy(trials)
    seq_trials.insert_trial_docs(copy.deepcopy(pend[:2]))
    seq_trials.refresh()
    seq = []
    for i in ids[2:]:
        d = tpe.suggest([i], dom, seq_trials, 11)
        seq_trials.insert_trial_docs(d)
        seq_trials.refresh()
        seq.extend(d)
    assert _vals(pend[2:]) == _vals(seq)


@pytest.mark.gpu
def test_tpe_from_scratch_without_startup():
    """n_startup_jobs=0 on an empty history: TPE on the prior-only
    posterior (tpe.py:877-880), not random search."""
    dom = H.Domain(_loss, SPACE)
    docs = tpe.suggest([0], dom, H.Trials(), 9, n_startup_jobs=0)
    assert len(docs) == 1 and docs[0]['tid'] == 0
    assert -3 <= docs[0]['misc']['vals']['a'][0] < 3


@pytest.mark.gpu
def test_uploader_tracks_owner_and_generation():
    """The per-thread engine's resident history alternates between two
    Trials objects, is replaced by a direct build_posterior call, and sees a
    Trials object dropped and another one created in its place; every
    suggestion equals a from-scratch device build of the same history."""
    import gc
    from hyperopt_amd import engine as E
    from hyperopt_amd import history
    dom = H.Domain(_loss, SPACE)
    specs = tpe.specs_of(dom)
    ref_eng = E.Engine(0)

    def reference(trials, new_id, seed):
        tids, losses, obs = history.gather(dom, trials, list(specs))
        ref_eng.build_posterior(*tpe.device_inputs(specs, tids, losses, obs), gamma=0.25,
                                prior_weight=1.0)
        res = ref_eng.suggest(seed, 24, round=new_id)
        return [float(r['value']) for r in res]

    def device(trials, new_id, seed):
        d = tpe.suggest([new_id], dom, trials, seed, posterior_builder='device')[0]
        return d['misc']['vals']

    def expect(trials, new_id, seed):
        vals = device(trials, new_id, seed)
        ref = reference(trials, new_id, seed)
        for i, lab in enumerate(specs):
            if vals[lab]:
                assert float(vals[lab][0]) == ref[i], (lab, vals[lab], ref[i])

    A, B = _history(200, 4), _history(250, 5)
    expect(A, 500, 1)
    expect(B, 501, 2)
    expect(A, 502, 3)
    eng = E.get_engine(0, 'f64')
    tids, losses, obs = history.gather(dom, B, list(specs))
    eng.build_posterior(*tpe.device_inputs(specs, tids, losses, obs), gamma=0.25, prior_weight=1.0)
    expect(A, 503, 4)                       # must re-upload A
    for k in range(3):                      # dropped Trials, new ones in their place
        C = _history(120 + k, 10 + k)
        expect(C, 600 + k, 5 + k)
        del C
        gc.collect()
    ref_eng.close()


def test_loss_array_pending_is_inf_and_nan_kept():
    """The fast loss read (history.loss_array): None -> +inf (a pending or
    failed trial joins the above set, tpe.py:844-847), NaN stays NaN (the doc
    is dropped), non-dict results go through domain.loss."""
    from hyperopt_amd import history
    dom = H.Domain(_loss, SPACE)
    docs = [{'result': {'loss': 1.5}}, {'result': {'status': 'new'}},
            {'result': {'loss': float('nan')}}, {'result': {'loss': 2}}]
    out = history.loss_array(dom, docs)
    assert out[0] == 1.5 and out[1] == np.inf and np.isnan(out[2]) and out[3] == 2.0
    ok = [{'result': {'loss': 0.25}}, {'result': {'loss': -1.0}}]
    assert list(history.loss_array(dom, ok)) == [0.25, -1.0]


@pytest.mark.gpu
def test_pending_batch_keeps_the_main_resident_history():
    """a batch='pending' view runs on its own context, so
    the real trials' device-resident history is not replaced (and uploaded
    whole again by the next regular call)."""
    from hyperopt_amd import engine as E
    trials = _history(300, 3)
    dom = H.Domain(_loss, SPACE)
    tpe.suggest([1999], dom, trials, 5, posterior_builder='device')
    main = E.get_engine(0, 'f64')
    gen, key = main.history_generation, main._history_uploader.key
    tpe.suggest([2000, 2001, 2002], dom, trials, 5, batch='pending', posterior_builder='device')
    assert main.history_generation == gen and main._history_uploader.key == key
    assert E.get_engine(0, 'f64', 'pending') is not main
