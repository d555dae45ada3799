"""Random search (hyperopt/rand.py): draws each new trial from the prior.
TPE delegates its first `n_startup_jobs` suggestions here (tpe.py:869-871).

Same protocol and seeding (`np.random.RandomState(seed)`, one draw per
new_id); the draw order over hyperparameters is this package's (choices
first, then the selected branch, labels in graph order), so individual values
differ from the reference's while the distribution is the same."""
import numpy as np

from . import labels as L
from .base import miscs_update_idxs_vals


def _specs(domain):
    specs = getattr(domain, 'specs', None)
    if not isinstance(specs, dict) or not specs or \
            not isinstance(next(iter(specs.values())), L.LabelSpec):
        specs = L.compile_space(domain.expr)
    return specs


def suggest(new_ids, domain, trials, seed):
    rng = np.random.RandomState(seed)
    specs = _specs(domain)
    rval = []
    for new_id in new_ids:
        values = L.sample_config(domain.expr, specs, rng)
        idxs = {k: ([new_id] if k in values else []) for k in specs}
        vals = {k: ([values[k]] if k in values else []) for k in specs}
        misc = dict(tid=new_id, cmd=domain.cmd, workdir=domain.workdir)
        miscs_update_idxs_vals([misc], idxs, vals)
        rval.extend(trials.new_trial_docs([new_id], [None], [domain.new_result()], [misc]))
    return rval


def suggest_batch(new_ids, domain, trials, seed):
    rng = np.random.RandomState(seed)
    specs = _specs(domain)
    idxs = {k: [] for k in specs}
    vals = {k: [] for k in specs}
    for new_id in new_ids:
        values = L.sample_config(domain.expr, specs, rng)
        for k, v in values.items():
            idxs[k].append(new_id)
            vals[k].append(v)
    return idxs, vals
