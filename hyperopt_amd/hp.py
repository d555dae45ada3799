"""`hp.*` search-space constructors with the reference's signatures
(hyperopt/hp.py, hyperopt/pyll_utils.py:41-122): every hyperparameter is a
`hyperopt_param(label, <distribution>)` node; continuous kinds are wrapped in
`float`, `choice` / `pchoice` become `switch(index, *options)`."""
from .space import Literal, Node


def _label(label):
    if isinstance(label, Literal):
        label = label.obj
    if not isinstance(label, str):
        raise TypeError('require string label')
    return label


def _param(label, dist):
    return Node('hyperopt_param', [_label(label), dist])


def _continuous(kind):
    def ctor(label, *args, **kwargs):
        return Node('float', [_param(label, Node(kind, args, kwargs.items()))])
    ctor.__name__ = kind
    ctor.__doc__ = '%s hyperparameter (pyll_utils.py hp_%s)' % (kind, kind)
    return ctor


uniform = _continuous('uniform')
quniform = _continuous('quniform')
loguniform = _continuous('loguniform')
qloguniform = _continuous('qloguniform')
normal = _continuous('normal')
qnormal = _continuous('qnormal')
lognormal = _continuous('lognormal')
qlognormal = _continuous('qlognormal')


def randint(label, *args, **kwargs):
    """Integer in [0, upper) (pyll_utils.py:64-66)."""
    return _param(label, Node('randint', args, kwargs.items()))


def choice(label, options):
    """One of `options` (pyll_utils.py:55-60)."""
    options = list(options)
    idx = _param(label, Node('randint', [len(options)]))
    return Node('switch', [idx] + options)


def pchoice(label, p_options):
    """One of the options with the given probabilities (pyll_utils.py:41-52)."""
    p, options = zip(*p_options)
    idx = _param(label, Node('categorical', [tuple(p)], [('upper', len(options))]))
    return Node('switch', [idx] + list(options))
