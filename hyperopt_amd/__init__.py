"""hyperopt_amd -- MI355X-native TPE suggestion engine with hyperopt's API.

    from hyperopt_amd import fmin, tpe, hp, Trials, STATUS_OK
    best = fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -5, 5),
                algo=tpe.suggest, max_evals=100, trials=Trials())

`tpe.suggest` also plugs into the reference package's own `fmin` (the algo
protocol is the same); see INTEGRATION.md.
"""
from . import hp, rand, tpe  # noqa: F401
from .base import (JOB_STATE_DONE, JOB_STATE_ERROR, JOB_STATE_NEW,  # noqa: F401
                   JOB_STATE_RUNNING, STATUS_FAIL, STATUS_NEW, STATUS_OK, STATUS_RUNNING,
                   STATUS_STRINGS, STATUS_SUSPENDED, Ctrl, Domain, Trials, trials_from_docs)
from .exceptions import (AllTrialsFailed, DuplicateLabel, InvalidLoss,  # noqa: F401
                         InvalidResultStatus, InvalidTrial)
from .fmin import fmin, fmin_pass_expr_memo_ctrl, partial, space_eval  # noqa: F401
from .space import scope  # noqa: F401

__version__ = '0.1.0'
