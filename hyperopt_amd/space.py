"""Search-space expressions: the graph that `hp.*` builds and `fmin` evaluates.

This replaces the pyll IR of the reference (hyperopt/pyll/base.py) for the
purposes the TPE drop-in needs: building spaces with `hp.*`, Python
containers, arithmetic and `scope.<fn>` calls; evaluating a space at a point
(`space_eval`, `Domain.evaluate`); and drawing from the prior.  It is not an
interpreter for the TPE posterior -- that runs as GPU kernels.

Nodes expose the same attributes the reference's `Apply` has (`name`,
`pos_args`, `named_args` as [name, node] pairs, `obj` for literals), so code
that inspects a space (the label compiler in `labels.py`) reads reference
graphs and ours alike.  Evaluation semantics follow the reference's
`rec_eval` (base.py:779-937): `switch` evaluates only the selected option,
Python lists/tuples become tuples (`pos_args`, base.py:944-946), dicts with
string keys become dicts.
"""
import math
import operator

import numpy as np


class Node(object):
    """A call of operator `name` on argument nodes."""

    __slots__ = ('name', 'pos_args', 'named_args', 'o_len', '__weakref__')

    def __init__(self, name, pos_args=(), named_args=(), o_len=None):
        self.name = name
        self.pos_args = [as_apply(a) for a in pos_args]
        self.named_args = sorted([[k, as_apply(v)] for k, v in named_args],
                                 key=lambda kv: kv[0])
        self.o_len = o_len

    def inputs(self):
        return self.pos_args + [v for _, v in self.named_args]

    @property
    def arg(self):
        """Arguments bound to parameter names (known operators only)."""
        return bind_args(self)

    def eval(self, memo=None):
        return rec_eval(self, memo=memo)

    def __repr__(self):
        return 'Node(%s, %d args)' % (self.name, len(self.inputs()))

    # -- python syntax builds new nodes ------------------------------------
    def __add__(self, o): return Node('add', [self, o])
    def __radd__(self, o): return Node('add', [o, self])
    def __sub__(self, o): return Node('sub', [self, o])
    def __rsub__(self, o): return Node('sub', [o, self])
    def __mul__(self, o): return Node('mul', [self, o])
    def __rmul__(self, o): return Node('mul', [o, self])
    def __truediv__(self, o): return Node('truediv', [self, o])
    def __rtruediv__(self, o): return Node('truediv', [o, self])
    def __floordiv__(self, o): return Node('floordiv', [self, o])
    def __rfloordiv__(self, o): return Node('floordiv', [o, self])
    def __pow__(self, o): return Node('pow', [self, o])
    def __rpow__(self, o): return Node('pow', [o, self])
    def __neg__(self): return Node('neg', [self])
    def __gt__(self, o): return Node('gt', [self, o])
    def __ge__(self, o): return Node('ge', [self, o])
    def __lt__(self, o): return Node('lt', [self, o])
    def __le__(self, o): return Node('le', [self, o])

    def __getitem__(self, idx):
        if self.o_len is not None and isinstance(idx, int) and idx >= self.o_len:
            raise IndexError()     # lets `a, b = node` unpack fixed-length nodes
        return Node('getitem', [self, idx])

    def __len__(self):
        if self.o_len is None:
            raise TypeError('length of this expression is not known')
        return self.o_len

    def __call__(self, *args, **kwargs):
        return Node('call', [self, args, kwargs])

    __hash__ = object.__hash__


class Literal(Node):
    __slots__ = ('_obj',)

    def __init__(self, obj=None):
        Node.__init__(self, 'literal')
        self._obj = obj
        try:
            self.o_len = len(obj)
        except TypeError:
            self.o_len = None

    @property
    def obj(self):
        return self._obj

    def __repr__(self):
        return 'Literal(%r)' % (self._obj,)


Apply = Node


def as_apply(obj):
    """Wrap constants and containers as nodes (reference: base.py:207-231)."""
    if isinstance(obj, Node) or (hasattr(obj, 'pos_args') and hasattr(obj, 'named_args')
                                 and hasattr(obj, 'name')):
        return obj     # ours, or a duck-typed foreign (reference pyll) node
    if isinstance(obj, (tuple, list)):
        return Node('pos_args', list(obj), o_len=len(obj) if isinstance(obj, tuple) else None)
    if isinstance(obj, dict):
        if all(isinstance(k, str) for k in obj):
            return Node('dict', [], sorted(obj.items()), o_len=len(obj))
        return Node('dict', [sorted(obj.items(), key=lambda kv: repr(kv[0]))])
    return Literal(obj)


# ---------------------------------------------------------------- operators --

def _call(fn, args, kwargs):
    return fn(*args, **kwargs)


def _categorical(p, upper=None, rng=None, size=()):
    p = np.asarray(p, dtype=float)
    n = int(np.prod(size)) if size != () else 1
    draws = rng.multinomial(1, p, size=n).argmax(axis=1)
    return draws.reshape(size) if size != () else int(draws[0])


def _randint(upper, rng=None, size=()):
    return rng.randint(upper, size=size) if size != () else int(rng.randint(upper))


def _q(draw, q):
    return np.round(draw / q) * q


# name -> implementation (the reference's prior samplers: pyll/stochastic.py:35-147)
IMPLS = {
    'pos_args': lambda *a: a,
    'dict': lambda *a, **k: dict(*a, **k),
    'list': list, 'len': len, 'int': int, 'float': float, 'max': max, 'min': min,
    'range': range, 'getattr': getattr, 'call': _call, 'identity': lambda x: x,
    'getitem': operator.getitem, 'add': operator.add, 'sub': operator.sub,
    'mul': operator.mul, 'truediv': operator.truediv, 'floordiv': operator.floordiv,
    'neg': operator.neg, 'eq': operator.eq, 'lt': operator.lt, 'le': operator.le,
    'gt': operator.gt, 'ge': operator.ge, 'pow': lambda a, b: a ** b,
    'exp': np.exp, 'log': np.log, 'sin': np.sin, 'cos': np.cos, 'tan': np.tan,
    'sqrt': np.sqrt, 'sum': lambda x, axis=None: np.sum(x, axis=axis),
    'minimum': np.minimum, 'maximum': np.maximum, 'asarray': np.asarray,
    'switch': lambda pos, *args: args[pos],
    'hyperopt_param': lambda label, obj: obj,
    'uniform': lambda low, high, rng=None, size=(): rng.uniform(low, high, size=size),
    'loguniform': lambda low, high, rng=None, size=(): np.exp(rng.uniform(low, high, size=size)),
    'quniform': lambda low, high, q, rng=None, size=(): _q(rng.uniform(low, high, size=size), q),
    'qloguniform': lambda low, high, q, rng=None, size=(): _q(np.exp(rng.uniform(low, high, size=size)), q),
    'normal': lambda mu, sigma, rng=None, size=(): rng.normal(mu, sigma, size=size),
    'qnormal': lambda mu, sigma, q, rng=None, size=(): _q(rng.normal(mu, sigma, size=size), q),
    'lognormal': lambda mu, sigma, rng=None, size=(): np.exp(rng.normal(mu, sigma, size=size)),
    'qlognormal': lambda mu, sigma, q, rng=None, size=(): _q(np.exp(rng.normal(mu, sigma, size=size)), q),
    'randint': _randint,
    'categorical': _categorical,
}

STOCHASTIC = ('uniform', 'loguniform', 'quniform', 'qloguniform', 'normal', 'qnormal',
              'lognormal', 'qlognormal', 'randint', 'categorical')

# parameter names of the operators whose arguments are inspected by name
SIGNATURES = {
    'hyperopt_param': ('label', 'obj'),
    'uniform': ('low', 'high'), 'loguniform': ('low', 'high'),
    'quniform': ('low', 'high', 'q'), 'qloguniform': ('low', 'high', 'q'),
    'normal': ('mu', 'sigma'), 'lognormal': ('mu', 'sigma'),
    'qnormal': ('mu', 'sigma', 'q'), 'qlognormal': ('mu', 'sigma', 'q'),
    'randint': ('upper',), 'categorical': ('p', 'upper'),
    'switch': ('pos',),
}


def bind_args(node):
    """{param_name: node} for a node of a known operator (pos + named)."""
    names = SIGNATURES.get(node.name)
    if names is None:
        raise TypeError('no argument binding for operator %r' % node.name)
    out = {}
    for i, a in enumerate(node.pos_args):
        if i < len(names):
            out[names[i]] = a
    for k, v in node.named_args:
        out[k] = v
    return out


class Scope(object):
    """`scope.<name>(...)` builds a node; `scope.define` registers a function."""

    def __init__(self):
        self._impls = IMPLS

    def define(self, f, o_len=None, pure=False):
        self._impls[f.__name__] = f
        return f

    def define_pure(self, f):
        return self.define(f, pure=True)

    def define_info(self, o_len=None, pure=False):
        def wrapper(f):
            return self.define(f, o_len=o_len, pure=pure)
        return wrapper

    def undefine(self, f):
        name = f if isinstance(f, str) else f.__name__
        del self._impls[name]

    def __getattr__(self, name):
        if name.startswith('__') or name not in IMPLS:
            raise AttributeError(name)

        def build(*args, **kwargs):
            return Node(name, args, kwargs.items())
        build.__name__ = name
        return build


scope = Scope()


# --------------------------------------------------------------- traversal --

def dfs(expr):
    """All nodes reachable from expr, inputs before users (each once)."""
    seen, order = set(), []
    stack = [(as_apply(expr), False)]
    while stack:
        node, done = stack.pop()
        if done:
            order.append(node)
            continue
        if id(node) in seen:
            continue
        seen.add(id(node))
        stack.append((node, True))
        for child in reversed(node.inputs()):
            if id(child) not in seen:
                stack.append((child, False))
    return order


class _Missing(object):
    def __repr__(self):
        return '<missing hyperparameter value>'


MISSING = _Missing()


def rec_eval(expr, memo=None, rng=None):
    """Evaluate expr.  memo maps nodes to precomputed values (e.g. the
    hyperopt_param nodes of a configuration); `switch` is lazy."""
    expr = as_apply(expr)
    memo = {} if memo is None else memo
    cache = {id(k): v for k, v in memo.items()} if memo else {}

    def ev(node):
        key = id(node)
        if key in cache:
            v = cache[key]
            if v is MISSING:
                raise KeyError('value for an inactive hyperparameter was needed')
            return v
        name = node.name
        if name == 'literal':
            v = node.obj
        elif name == 'switch':
            pos = ev(node.pos_args[0])
            v = ev(node.pos_args[1 + int(pos)])
        else:
            args = [ev(a) for a in node.pos_args]
            kwargs = {k: ev(a) for k, a in node.named_args}
            if name in STOCHASTIC and kwargs.get('rng') is None:
                if rng is None:
                    raise ValueError('%s node needs an rng' % name)
                kwargs['rng'] = rng
            fn = IMPLS.get(name)
            if fn is None:
                raise KeyError('unknown operator %r' % name)
            v = fn(*args, **kwargs)
        cache[key] = v
        return v

    import sys
    old = sys.getrecursionlimit()
    if old < 10000:
        sys.setrecursionlimit(10000)
    try:
        return ev(expr)
    finally:
        sys.setrecursionlimit(old)


def sample(expr, rng=None):
    """One draw of the whole space from its prior."""
    rng = np.random.RandomState() if rng is None else rng
    return rec_eval(expr, rng=rng)


def isfinite_number(x):
    try:
        return math.isfinite(float(x))
    except (TypeError, ValueError):
        return False
