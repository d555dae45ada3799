"""Synthetic trial histories for the BASELINE.json configurations (SURVEY.md
§8(d)).  Values come from each hyperparameter's prior, drawn with
np.random.RandomState(seed); losses are a separable bowl plus noise.  Used by
bench.py and the tests; no data files, no network."""
import numpy as np

from . import posterior as P

PREPARE_MIN = 8192   # candidate slots of a round from which it uses the expansion index
# index labels from which the first build goes without the tie orders and
# the index runs beside the host's argsorts and the ordered subset rebuild;
# below it the known labels' argsorts come first and ONE ordered build
# follows (r5q, config 3: a 4-label shard's step 1.19 -> 1.10 ms without the
# overlap, the whole 32-label step 2.57 -> 2.88 ms: the index is long enough
# to hide the argsorts only with many dense labels) -- until the subset
# rebuild's report was deferred into the round (posterior.DEFER_REPORT): the
# overlap then wins for shards too (config 3's 4-label shards 0.95-1.03 ->
# 0.85-0.97 ms, r5bh)
OVERLAP_MIN_DENSE = 1
DENSE_KINDS = ('uniform', 'loguniform', 'normal', 'lognormal')

# config-3 kind cycle: kind = i mod 5
CYCLE = (('uniform', dict(low=-5.0, high=5.0)),
         ('loguniform', dict(low=-5.0, high=2.0)),
         ('quniform', dict(low=0.0, high=100.0, q=1.0)),
         ('normal', dict(mu=0.0, sigma=3.0)),
         ('randint', dict(upper=5)))


def prior_draw(kind, args, rng, n):
    if kind == 'uniform':
        return rng.uniform(args['low'], args['high'], n)
    if kind == 'quniform':
        return np.round(rng.uniform(args['low'], args['high'], n) / args['q']) * args['q']
    if kind == 'loguniform':
        return np.exp(rng.uniform(args['low'], args['high'], n))
    if kind == 'qloguniform':
        return np.round(np.exp(rng.uniform(args['low'], args['high'], n)) / args['q']) * args['q']
    if kind == 'normal':
        return rng.normal(args['mu'], args['sigma'], n)
    if kind == 'qnormal':
        return np.round(rng.normal(args['mu'], args['sigma'], n) / args['q']) * args['q']
    if kind == 'lognormal':
        return np.exp(rng.normal(args['mu'], args['sigma'], n))
    if kind == 'qlognormal':
        return np.round(np.exp(rng.normal(args['mu'], args['sigma'], n)) / args['q']) * args['q']
    if kind in ('randint', 'categorical'):
        return rng.randint(args['upper'], size=n).astype(float)
    raise ValueError(kind)


def bowl(kind, x):
    if kind == 'uniform':
        return (x - 1.0) ** 2
    if kind == 'loguniform':
        return (np.log(x) + 1.0) ** 2
    if kind == 'quniform':
        return ((x - 30.0) / 10.0) ** 2
    if kind == 'normal':
        return (x - 0.5) ** 2
    if kind == 'randint':
        return (x != 2).astype(float)
    return np.zeros_like(x)


def hartmann6(x):
    """Standard Hartmann-6 (config 2 objective)."""
    alpha = np.array([1.0, 1.2, 3.0, 3.2])
    A = np.array([[10, 3, 17, 3.5, 1.7, 8], [.05, 10, 17, .1, 8, 14],
                  [3, 3.5, 1.7, 10, 17, 8], [17, 8, .05, 10, .1, 14]])
    Pm = 1e-4 * np.array([[1312, 1696, 5569, 124, 8283, 5886], [2329, 4135, 8307, 3736, 1004, 9991],
                          [2348, 1451, 3522, 2883, 3047, 6650], [4047, 8828, 8732, 5743, 1091, 381]])
    inner = ((x[:, None, :] - Pm[None]) ** 2 * A[None]).sum(-1)
    return -(alpha[None] * np.exp(-inner)).sum(-1)


class History(object):
    """Flat history: labels, per-label active (tids, vals), per-trial losses."""

    def __init__(self, labels, tids, losses, obs):
        self.labels = labels          # [(name, kind, args)]
        self.tids = tids              # (N,) int64, sorted
        self.losses = losses          # (N,) float64
        self.obs = obs                # name -> (idxs, vals)

    def posteriors(self, gamma=0.25, prior_weight=1.0):
        splitter = P.Splitter(self.tids, self.losses, gamma)
        posts = []
        for name, kind, args in self.labels:
            oi, ov = self.obs[name]
            b, a = splitter.split(oi, ov)
            posts.append(P.label_posterior(name, kind, args, b, a, prior_weight))
        return posts


    def device_inputs(self):
        """Arguments of Engine.build_posterior for this history (after gamma,
        prior_weight: see posterior.device_inputs)."""
        return P.device_inputs(self.labels, self.tids, self.losses, self.obs)

    def prefix(self, n):
        """The history of the first n trials (tids 0..n-1)."""
        obs = {}
        for name, (oi, ov) in self.obs.items():
            k = int(np.searchsorted(oi, n))
            obs[name] = (oi[:k], ov[:k])
        return History(self.labels, self.tids[:n], self.losses[:n], obs)


class FminLoop(object):
    """The device side of fmin's serial loop over a synthetic history: each
    `advance` appends the next trials (their losses and observations) and
    rebuilds the posterior the way tpe.suggest does past
    DEVICE_BUILD_MIN_OBS -- the device-resident history takes only the new
    observations (DeviceHistoryUploader), the device builder splits, sorts,
    fits the Parzen mixtures and folds the records, with numpy's np.argsort
    tie order for the labels whose mixtures depend on it
    (posterior.build_reference_order).  The view tuple is the one
    history.device_view hands tpe.suggest.

    label_ids: the subset of the space's labels this loop holds (a
    label-sharded rank, parallel.label_shards); each keeps its Philox stream
    (its index in the whole space), so its candidates and winner are the
    whole space's."""

    def __init__(self, hist, gamma=0.25, prior_weight=1.0, label_ids=None):
        self.hist = hist
        self.gamma, self.prior_weight = gamma, prior_weight
        self.label_ids = (list(range(len(hist.labels))) if label_ids is None
                          else [int(i) for i in label_ids])
        self.labels = [hist.labels[i] for i in self.label_ids]
        self.streams = None if label_ids is None else self.label_ids
        self.names = [n for n, _, _ in self.labels]
        # labels observed in every trial: their view is a prefix slice
        self.full = [np.array_equal(hist.obs[n][0], hist.tids) for n in self.names]
        self.n_dense = sum(1 for _, k, _ in self.labels if k in DENSE_KINDS)
        self.uploader = P.DeviceHistoryUploader()
        self.n = 0

    def view(self, n):
        obs = {}
        hobs = self.hist.obs
        kt = int(np.searchsorted(self.hist.tids, n))   # (a label in every trial: the same prefix)
        for name, full in zip(self.names, self.full):
            oi, ov = hobs[name]
            k = kt if full else int(np.searchsorted(oi, n))
            obs[name] = (oi[:k], ov[:k])
        losses = self.hist.losses[:n]
        return (self.hist.tids[:n], losses, int(np.count_nonzero(losses == losses)), obs, self)

    def advance(self, eng, n, n_candidates=0, n_rounds=1, round_call=None):
        """History of the first n trials on the device, posterior rebuilt
        (its expansion index queued meanwhile when the coming round(s) of
        n_candidates per label will use it, as tpe.suggest does); returns
        (n_below, results of round_call -- the step's round, run as
        tpe.suggest runs it: see posterior.build_reference_order -- or None)."""
        if n > len(self.hist.tids):
            raise ValueError('the synthetic history holds %d trials' % len(self.hist.tids))
        self.n = n
        return self.uploader.build(eng, self.labels, self.view(n), self.gamma, self.prior_weight,
                                   prepare=((n_candidates, n_rounds)
                                            if n_candidates * n_rounds >= PREPARE_MIN else None),
                                   streams=self.streams, overlap=self.n_dense >= OVERLAP_MIN_DENSE,
                                   round_call=round_call)


def mixed_space(n_labels):
    return [('x%03d' % i,) + CYCLE[i % 5] for i in range(n_labels)]


def mixed_history(n_labels=32, n_trials=10000, seed=0):
    """Configs 3 and 5: kind = i mod 5; loss = sum of bowls + 0.1 N(0,1)."""
    rng = np.random.RandomState(seed)
    labels = mixed_space(n_labels)
    tids = np.arange(n_trials, dtype=np.int64)
    loss = 0.1 * rng.normal(size=n_trials)
    obs = {}
    for name, kind, args in labels:
        v = prior_draw(kind, args, rng, n_trials)
        loss = loss + bowl(kind, v)
        obs[name] = (tids, v)
    return History(labels, tids, loss, obs)


def hartmann_history(n_trials=2000, seed=0):
    """Config 2: Hartmann-6 over hp.uniform('x{i}', 0, 1)."""
    rng = np.random.RandomState(seed)
    x = rng.uniform(0, 1, size=(n_trials, 6))
    tids = np.arange(n_trials, dtype=np.int64)
    labels = [('x%d' % i, 'uniform', dict(low=0.0, high=1.0)) for i in range(6)]
    obs = {labels[i][0]: (tids, x[:, i]) for i in range(6)}
    return History(labels, tids, hartmann6(x), obs)


def conditional_history(n_trials=5000, seed=0):
    """Config 4: hp.choice('clf', [svm{...}, rf{...}, gbm{...}]) -- children are
    active only in the trials that chose their branch."""
    rng = np.random.RandomState(seed)
    ln = np.log
    branches = [
        [('svm_C', 'loguniform', dict(low=-5.0, high=5.0)),
         ('svm_gamma', 'loguniform', dict(low=-8.0, high=2.0)),
         ('svm_kernel', 'randint', dict(upper=3)),
         ('svm_degree', 'quniform', dict(low=2.0, high=5.0, q=1.0))],
        [('rf_n', 'qloguniform', dict(low=float(ln(10)), high=float(ln(1000)), q=1.0)),
         ('rf_depth', 'quniform', dict(low=1.0, high=30.0, q=1.0)),
         ('rf_max_feat', 'uniform', dict(low=0.1, high=1.0)),
         ('rf_crit', 'randint', dict(upper=2))],
        [('gbm_lr', 'loguniform', dict(low=float(ln(1e-3)), high=0.0)),
         ('gbm_n', 'qloguniform', dict(low=float(ln(10)), high=float(ln(1000)), q=1.0)),
         ('gbm_subsample', 'uniform', dict(low=0.5, high=1.0)),
         ('gbm_depth', 'quniform', dict(low=1.0, high=10.0, q=1.0))],
    ]
    labels = [('clf', 'randint', dict(upper=3))] + [l for b in branches for l in b]
    tids = np.arange(n_trials, dtype=np.int64)
    clf = rng.randint(3, size=n_trials)
    loss = 0.1 * rng.normal(size=n_trials) + 0.3 * clf
    obs = {'clf': (tids, clf.astype(float))}
    for bi, br in enumerate(branches):
        act = tids[clf == bi]
        for name, kind, args in br:
            v = prior_draw(kind, args, rng, len(act))
            if kind in ('uniform', 'loguniform', 'quniform', 'qloguniform'):
                lv = np.log(v) if 'log' in kind else v
                lo, hi = args['low'], args['high']
                contrib = ((lv - lo) / (hi - lo) - 0.3) ** 2
            else:
                contrib = (v != 1).astype(float) * 0.2
            loss[clf == bi] += contrib
            obs[name] = (act, v)
    return History(labels, tids, loss, obs)


def hp_space(labels):
    """The hp.* space of a synthetic label list (randint -> hp.choice)."""
    from . import hp
    space = {}
    for name, kind, args in labels:
        if kind == 'randint':
            space[name] = hp.choice(name, list(range(int(args['upper']))))
        else:
            space[name] = getattr(hp, kind)(name, *[args[k] for k in
                                                    (('low', 'high', 'q') if 'low' in args
                                                     else ('mu', 'sigma', 'q')) if k in args])
    return space


def history_trials(hist):
    """A Trials object holding the synthetic history as finished trial docs."""
    from .base import JOB_STATE_DONE, STATUS_OK, Trials
    trials = Trials()
    names = [n for n, _, _ in hist.labels]
    cols = {}
    for n in names:
        oi, ov = hist.obs[n]
        cols[n] = dict(zip(oi.tolist(), ov.tolist()))
    kinds = {n: k for n, k, _ in hist.labels}
    docs = []
    for tid, loss in zip(hist.tids.tolist(), hist.losses.tolist()):
        idxs, vals = {}, {}
        for n in names:
            v = cols[n].get(tid)
            if v is None:
                idxs[n], vals[n] = [], []
            else:
                idxs[n] = [tid]
                vals[n] = [int(v) if kinds[n] in ('randint', 'categorical') else float(v)]
        docs.append(dict(state=JOB_STATE_DONE, tid=tid, spec=None,
                         result={'status': STATUS_OK, 'loss': float(loss)},
                         misc=dict(tid=tid, cmd=('domain_attachment', 'FMinIter_Domain'),
                                   workdir=None, idxs=idxs, vals=vals),
                         exp_key=None, owner=None, version=0, book_time=None,
                         refresh_time=None))
    trials._insert_trial_docs(docs)
    trials.refresh()
    return trials
