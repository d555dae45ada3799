"""Tree-structured Parzen Estimator: drop-in `tpe.suggest` running on MI355X.

    from hyperopt_amd import fmin, hp, tpe, Trials
    fmin(fn, space, algo=tpe.suggest, max_evals=100, trials=Trials())

`suggest` keeps the reference's signature, defaults and returned document
(hyperopt/tpe.py:823-916).  Per call:
  1. history: tids, losses (None -> +inf, min per from_tid group) and per-label
     observations, from a columnar cache (history.py);
  2. fewer than n_startup_jobs docs -> random search (rand.suggest);
  3. posteriors: split by loss rank + adaptive Parzen mixtures / categorical
     pseudocounts per label, bit-identical to the reference (posterior.py);
  4. one fused GPU round over ALL labels (engine.Engine.suggest): sample
     n_EI_candidates per label from l(x) (Philox, stream = label, counter =
     candidate index, round = new_id), lpdf under l and g, broadcast_best;
  5. labels under an un-chosen hp.choice branch are dropped (the reference
     routes every candidate id to the winning branch, vectorize.py:25-43;
     labels are independent given the history, so evaluating every branch
     and keeping the selected one is the same distribution).

Extra keyword arguments (not in the reference): `precision` ('f64'; 'f32'
is accepted and runs the same exact path -- see `suggest`), `device` (HIP ordinal), `devices` (a list of ordinals: one
multi-device context splits every round over those GPUs, same documents as
one GPU; tpe_ctx_create_multi), `batch` (True: one independent
suggestion per new_id instead of only new_ids[0]), `posterior_builder`:
'host' (numpy, posterior.py -- the reference's own np.argsort tie order),
'device' (the GPU build: split, sort, Parzen and fold in HIP kernels on the
device-resident history; the device flags every mixture whose value depends
on the order of tied losses or observations, and for exactly those the host
supplies numpy's np.argsort orders and the device builds again --
posterior.build_reference_order -- so the mixtures are the host build's bit
for bit) or 'auto' (device once the history holds DEVICE_BUILD_MIN_OBS
observations over all labels, where the host build starts to dominate the
suggestion).
"""
import logging
import time

import numpy as np

from . import engine as _engine
from . import history as _history
from . import labels as _labels
from . import posterior as _post
from . import rand
from .base import miscs_update_idxs_vals

logger = logging.getLogger(__name__)

EPS = 1e-12
DEFAULT_LF = 25
_default_prior_weight = 1.0
_default_n_EI_candidates = 24
_default_gamma = 0.25
_default_n_startup_jobs = 20
_default_linear_forgetting = DEFAULT_LF
DEVICE_BUILD_MIN_OBS = 16384

# host-side restatements, exported under the reference's names
ap_filter_trials_split = _post.split_history
adaptive_parzen_normal = _post.adaptive_parzen_normal
linear_forgetting_weights = _post.linear_forgetting_weights


def ap_filter_trials(o_idxs, o_vals, l_idxs, l_vals, gamma, gamma_cap=DEFAULT_LF):
    """tpe.py:624-648."""
    bt, at = _post.split_history(l_idxs, l_vals, gamma, gamma_cap)
    return _post.split_label(o_idxs, o_vals, bt, at)


def specs_of(domain):
    specs = getattr(domain, 'specs', None)
    if isinstance(specs, dict) and specs and isinstance(next(iter(specs.values())),
                                                        _labels.LabelSpec):
        return specs
    cached = getattr(domain, '_hyperopt_amd_specs', None)
    if cached is None:
        cached = _labels.compile_space(domain.expr)
        try:
            domain._hyperopt_amd_specs = cached
        except AttributeError:
            pass
    return cached


def build_posteriors(domain, trials, prior_weight=_default_prior_weight,
                     gamma=_default_gamma):
    """(specs, n_docs, posteriors) for the current history."""
    specs = specs_of(domain)
    tids, losses, obs = _history.gather(domain, trials, list(specs))
    if len(tids) == 0:
        return specs, 0, None
    splitter = _post.Splitter(tids, losses, gamma)
    posts = []
    for label, s in specs.items():
        oi, ov = obs[label]
        b, a = splitter.split(oi, ov)
        posts.append(_post.label_posterior(label, s.kind, s.args, b, a, prior_weight))
    return specs, len(tids), posts


def device_inputs(specs, tids, losses, obs):
    """Arguments of Engine.build_posterior for a gathered history."""
    labels = [(s.label, s.kind, s.args) for s in specs.values()]
    return _post.device_inputs(labels, tids, losses, obs)


def _doc(new_id, domain, trials, specs, values):
    flat = getattr(domain, '_hyperopt_amd_flat', None)
    if flat is None:
        flat = _labels.always_active(domain.expr)
        try:
            domain._hyperopt_amd_flat = flat
        except AttributeError:
            pass
    active = specs if flat else _labels.active_labels(domain.expr, values)
    idxs = {k: ([new_id] if k in active else []) for k in specs}
    vals = {k: ([values[k]] if k in active else []) for k in specs}
    misc = dict(tid=new_id, cmd=domain.cmd, workdir=domain.workdir)
    miscs_update_idxs_vals([misc], idxs, vals)
    return trials.new_trial_docs([new_id], [None], [domain.new_result()], [misc])


class _PendingView(object):
    """The trials a sequential caller would see after inserting a batch's
    earlier suggestions: the real documents plus those, still pending (state
    new, result {'status': 'new'}: loss None -> +inf, tpe.py:844-847)."""

    def __init__(self, trials):
        self._base = trials
        self.trials = list(trials.trials)

    def new_trial_docs(self, *args, **kwargs):
        return self._base.new_trial_docs(*args, **kwargs)

    def __len__(self):
        return len(self.trials)


PREPARE_MIN = 8192   # candidate slots of a round from which it uses the expansion index


def _resident_posterior(eng, domain, trials, specs, view, gathered, gamma, prior_weight,
                        builder, n_candidates=0, n_rounds=1, round_call=None):
    """Put the posterior of the current history on the engine, from the
    device-resident history's `view` or the general gather (tids, losses,
    obs); returns (the number of trial documents it was built from, the
    results of round_call when the incremental device build ran it -- the
    dense labels' round under the host's tie-order argsorts -- else None)."""
    labels = list(specs)
    if view is not None:
        n_docs = view[2]
        n_obs = sum(len(view[3][k][0]) for k in labels)
    if view is None or n_docs == 0:
        tids, losses, obs = gathered or _history.gather(domain, trials, labels)
        n_docs = len(tids)
        n_obs = sum(len(obs[k][0]) for k in labels)
    on_device = n_docs > 0 and (builder == 'device' or (builder == 'auto' and
                                                         n_obs >= DEVICE_BUILD_MIN_OBS))
    if on_device:
        try:
            if view is not None:   # upload only the observations that are new
                up = getattr(eng, '_history_uploader', None)
                if up is None:
                    up = eng._history_uploader = _post.DeviceHistoryUploader()
                _, res = up.build(eng, [(s.label, s.kind, s.args) for s in specs.values()], view, gamma,
                                  prior_weight, prepare=((n_candidates, n_rounds)
                                                         if n_candidates * n_rounds >= PREPARE_MIN else None),
                                  round_call=round_call)
                return n_docs, res
            eng.build_posterior(*device_inputs(specs, tids, losses, obs), gamma=gamma,
                                prior_weight=prior_weight)
            return n_docs, None
        except _post.NonFiniteObservation:
            # NaN observations: the host build raises what the reference's
            # adaptive_parzen_normal raises (tpe.py:469)
            if view is not None:
                tids, losses, obs = _history.gather(domain, trials, labels)
    elif view is not None and n_docs > 0:
        tids, losses, obs = _history.gather(domain, trials, labels)
    splitter = _post.Splitter(tids, losses, gamma)
    posts = []
    for label, sp in specs.items():
        b, a = splitter.split(*obs[label])
        posts.append(_post.label_posterior(label, sp.kind, sp.args, b, a, prior_weight))
    eng.set_posterior(*_post.pack(posts))
    return n_docs, None


def suggest(new_ids, domain, trials, seed,
            prior_weight=_default_prior_weight,
            n_startup_jobs=_default_n_startup_jobs,
            n_EI_candidates=_default_n_EI_candidates,
            gamma=_default_gamma,
            linear_forgetting=_default_linear_forgetting,
            precision='f64', device=0, batch=False, posterior_builder='auto', devices=None):
    """tpe.py:823-916.  Past the startup phase one document for new_ids[0],
    like the reference; `batch` (not in the reference) asks for one document
    per new_id:

    * batch=True -- the documents K sequential calls suggest([new_ids[j]],
      domain, trials, seed) would return with `trials` unchanged between
      them: one posterior, the batch's other suggestions excluded from it;
    * batch='pending' -- past the startup phase, the documents K sequential
      calls return when each call's document is inserted into the trials,
      still pending, before the next call (the reference's view of queued
      trials: loss None -> +inf, tpe.py:844-847; fmin with max_queue_len,
      fmin.py:193-202).  The first k = n_startup_jobs - len(docs) ids (the
      calls that would still be in the startup phase) are answered by ONE
      rand.suggest(new_ids[:k], ...) call -- distinct draws, as the
      reference answers a startup batch -- not by k sequential calls.

    During the startup phase (fewer than n_startup_jobs documents) the
    reference's rand.suggest(new_ids, ...) answers, for every new_id.

    precision='f32' runs the exact fp64 path: a round draws every candidate
    and proves all but ~0.5 % of them out of the race from per-sub-bin score
    bounds before any lpdf is summed, so scoring the rest in fp32 would save
    nothing measurable while giving up the bit-exact
    winner; the fp32 lpdf contract (1e-4 relative) holds trivially.  The raw
    fp32 round stays available as Engine(precision='f32')."""
    t0 = time.time()
    if precision not in ('f64', 'f32'):
        raise ValueError("precision must be 'f64' or 'f32'")
    if posterior_builder not in ('auto', 'host', 'device'):
        raise ValueError('posterior_builder must be auto, host or device')
    if batch not in (False, True, 'pending'):
        raise ValueError("batch must be False, True or 'pending'")
    kw = dict(prior_weight=prior_weight, n_startup_jobs=n_startup_jobs,
              n_EI_candidates=n_EI_candidates, gamma=gamma, linear_forgetting=linear_forgetting,
              precision=precision, device=device, posterior_builder=posterior_builder,
              devices=devices)
    specs = specs_of(domain)
    labels = list(specs)
    # the device-resident history's view of the trials (None when the fast
    # layout does not apply); otherwise the general gather
    view = _history.device_view(domain, trials, labels) if posterior_builder != 'host' else None
    gathered = None
    if view is not None:
        n_docs = view[2]
    else:
        gathered = _history.gather(domain, trials, labels)
        n_docs = len(gathered[0])
    if batch == 'pending' and len(new_ids) > 1:
        # the calls that would still see fewer than n_startup_jobs documents
        # are the startup phase: one rand.suggest over their ids, as the
        # reference answers a startup batch (tpe.py:869-871; distinct draws
        # from one RandomState(seed), the documents batch=True returns) --
        # then one TPE call per remaining id, each seeing the earlier ones
        # as pending trials
        k = max(0, min(len(new_ids), n_startup_jobs - n_docs))
        rval = list(rand.suggest(list(new_ids[:k]), domain, trials, seed)) if k else []
        if k < len(new_ids):
            pview = _PendingView(trials)
            pview.trials.extend(rval)
            for new_id in new_ids[k:]:
                docs = suggest([new_id], domain, pview, seed, batch=False, **kw)
                pview.trials.extend(docs)
                rval.extend(docs)
        return rval
    if n_docs < n_startup_jobs:
        return rand.suggest(new_ids, domain, trials, seed)      # tpe.py:869-871
    if n_docs == 0:
        logger.info('TPE using 0 trials')                     # the prior-only posterior
    # a pending view (batch='pending') keeps its own context: its history
    # (the trials plus the batch's earlier suggestions) would otherwise
    # replace the real trials' device-resident history, and the next call
    # on those would upload it whole again
    eng = _engine.get_engine(list(devices) if devices else device, 'f64',
                             'pending' if isinstance(trials, _PendingView) else 'main')
    ids = list(new_ids) if batch else [new_ids[0]]

    def round_call():
        if len(ids) == 1:
            return eng.suggest(seed, n_EI_candidates, round=ids[0])[None]
        return eng.suggest_batch(seed, ids, n_EI_candidates)
    _, res = _resident_posterior(eng, domain, trials, specs, view, gathered, gamma, prior_weight,
                                 posterior_builder, n_candidates=n_EI_candidates, n_rounds=len(ids),
                                 round_call=round_call)
    if res is None:
        res = round_call()
    rval = []
    for j, new_id in enumerate(ids):
        values = {s.label: _labels.coerce(s.kind, res[j][i]['value'])
                  for i, s in enumerate(specs.values())}
        rval.extend(_doc(new_id, domain, trials, specs, values))
    logger.info('tpe.suggest: %d trials, %d labels, %.1f ms' % (
        n_docs, len(specs), (time.time() - t0) * 1e3))
    return rval


# -- reference operators on the GPU engine (tpe.py:56-307, 769-778) ----------

def _eng():
    return _engine.get_engine(0, 'f64')


def GMM1_lpdf(samples, weights, mus, sigmas, low=None, high=None, q=None):
    return _eng().GMM1_lpdf(samples, weights, mus, sigmas, low, high, q)


def LGMM1_lpdf(samples, weights, mus, sigmas, low=None, high=None, q=None):
    return _eng().LGMM1_lpdf(samples, weights, mus, sigmas, low, high, q)


def categorical_lpdf(sample, p, upper=None):
    return _eng().categorical_lpdf(sample, p, upper)


def broadcast_best(samples, below_llik, above_llik):
    return _eng().broadcast_best(samples, below_llik, above_llik)


def _seed_from(rng):
    if rng is None:
        return np.random.randint(2 ** 31 - 1)
    return int(rng.randint(2 ** 31 - 1))


def GMM1(weights, mus, sigmas, low=None, high=None, q=None, rng=None, size=()):
    """Draws from the truncated mixture (Philox stream seeded from `rng`)."""
    out = _eng().GMM1(weights, mus, sigmas, low, high, q, seed=_seed_from(rng),
                      size=size if size != () else (1,))
    return out if size != () else out[0]


def LGMM1(weights, mus, sigmas, low=None, high=None, q=None, rng=None, size=()):
    out = _eng().LGMM1(weights, mus, sigmas, low, high, q, seed=_seed_from(rng),
                       size=size if size != () else (1,))
    return out if size != () else out[0]
