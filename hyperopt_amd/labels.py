"""Compile a search space into a flat label table (the per-hyperparameter
descriptors the GPU engine works on) and resolve which labels a
configuration activates.

Works on graphs built by `hyperopt_amd.hp` and on the reference's pyll graphs
(a reference `Domain.expr`), through the attributes both share: `name`,
`pos_args`, `named_args` and `obj` for literals.

Reference behaviour followed:
  * labels / DuplicateLabel         base.py:771-777 (Domain.params)
  * conditions from nested switches pyll_utils.py:130-234 (expr_to_config) --
    here resolved directly by walking the graph with the chosen values, the
    way the reference's vectorized switch routes ids (vectorize.py:25-43)
  * distribution arguments must be constants: the reference's
    build_posterior evaluates them from the memo (tpe.py:685) and fails for
    hyperparameter-dependent bounds; we reject such spaces up front.
"""
from collections import OrderedDict

import numpy as np

from .exceptions import DuplicateLabel
from .space import IMPLS, SIGNATURES, as_apply, rec_eval

KINDS = ('uniform', 'quniform', 'loguniform', 'qloguniform', 'normal', 'qnormal',
         'lognormal', 'qlognormal', 'randint', 'categorical')


def is_node(x):
    return hasattr(x, 'name') and hasattr(x, 'pos_args') and hasattr(x, 'named_args')


def inputs(node):
    return list(node.pos_args) + [v for _, v in node.named_args]


def literal_value(node):
    if node.name == 'literal':
        return node.obj
    raise ValueError('expected a literal, got %r' % node.name)


def walk(expr):
    """Every node reachable from expr, each once."""
    seen, out, stack = set(), [], [expr]
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        out.append(n)
        stack.extend(inputs(n))
    return out


def _has_param(node):
    return any(n.name == 'hyperopt_param' for n in walk(node))


def _bind(node):
    names = SIGNATURES[node.name]
    out = {}
    for i, a in enumerate(node.pos_args):
        if i < len(names):
            out[names[i]] = a
    for k, v in node.named_args:
        out[k] = v
    return out


class LabelSpec(object):
    __slots__ = ('label', 'kind', 'args', 'dist', 'param')

    def __init__(self, label, kind, args, dist, param):
        self.label, self.kind, self.args, self.dist, self.param = label, kind, args, dist, param

    def __repr__(self):
        return 'LabelSpec(%r, %s, %r)' % (self.label, self.kind, self.args)


def param_label(node):
    a = _bind(node)
    return literal_value(a['label'])


def compile_space(expr):
    """label -> LabelSpec, in a stable (sorted-label) order."""
    expr = as_apply(expr)
    specs = {}
    for node in walk(expr):
        if node.name != 'hyperopt_param':
            continue
        b = _bind(node)
        label = literal_value(b['label'])
        dist = b['obj']
        if label in specs:
            if specs[label].param is not node:
                raise DuplicateLabel(label)
            continue
        kind = dist.name
        if kind not in KINDS:
            raise NotImplementedError('hyperparameter %r: distribution %r is not supported'
                                      % (label, kind))
        args = {}
        for k, v in _bind(dist).items():
            if k in ('rng', 'size'):
                continue
            if _has_param(v):
                raise ValueError('hyperparameter %r: argument %r depends on another '
                                 'hyperparameter; TPE needs constant distribution '
                                 'parameters (the reference fails on such spaces too)'
                                 % (label, k))
            args[k] = rec_eval(v)
        if kind == 'randint':
            args['upper'] = int(args['upper'])
        if kind == 'categorical':
            args['p'] = [float(x) for x in np.asarray(args['p'], dtype=float).ravel()]
            args['upper'] = int(args.get('upper') or len(args['p']))
        for k in ('low', 'high', 'mu', 'sigma', 'q'):
            if k in args:
                args[k] = float(args[k])
        specs[label] = LabelSpec(label, kind, args, dist, node)
    return OrderedDict(sorted(specs.items()))


def _eval_with(node, values):
    """Evaluate a (switch index) expression given hyperparameter values."""
    if node.name == 'hyperopt_param':
        return values[param_label(node)]
    memo = {}
    for n in walk(node):
        if n.name == 'hyperopt_param':
            memo[n] = values[param_label(n)]
    return rec_eval(node, memo=memo)


def active_labels(expr, values):
    """Labels that take part in evaluating expr when the hyperparameters
    take `values` (only the selected option of each switch is visited)."""
    active, seen, stack = set(), set(), [as_apply(expr)]
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        if n.name == 'hyperopt_param':
            active.add(param_label(n))
            continue
        if n.name == 'switch':
            pos = int(_eval_with(n.pos_args[0], values))
            stack.append(n.pos_args[0])
            stack.append(n.pos_args[1 + pos])
            continue
        stack.extend(inputs(n))
    return active


def always_active(expr):
    """True when no switch (hp.choice / pchoice) has a hyperparameter under
    any of its options: every label then takes part in every evaluation and
    active_labels need not walk the graph."""
    for n in walk(as_apply(expr)):
        if n.name == 'switch':
            for opt in n.pos_args[1:]:
                if any(m.name == 'hyperopt_param' for m in walk(opt)):
                    return False
    return True


def coerce(kind, v):
    """Python type of a hyperparameter value in trial docs."""
    if kind in ('randint', 'categorical'):
        return int(v)
    return float(v)


def sample_config(expr, specs, rng):
    """One prior draw of the ACTIVE hyperparameters (the random-search
    proposal, rand.py:15-31 / pyll/stochastic.py:35-147): choices are drawn
    first and only the selected branch is descended."""
    values = {}
    seen, stack = set(), [as_apply(expr)]
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        if n.name == 'hyperopt_param':
            lab = param_label(n)
            if lab not in values:
                s = specs[lab]
                fn = IMPLS[s.kind]
                values[lab] = coerce(s.kind, fn(rng=rng, **s.args))
            continue
        if n.name == 'switch':
            idx = n.pos_args[0]
            # draw the index's hyperparameters first
            for m in walk(idx):
                if m.name == 'hyperopt_param':
                    lab = param_label(m)
                    if lab not in values:
                        s = specs[lab]
                        values[lab] = coerce(s.kind, IMPLS[s.kind](rng=rng, **s.args))
            pos = int(_eval_with(idx, values))
            stack.append(idx)
            stack.append(n.pos_args[1 + pos])
            continue
        stack.extend(reversed(inputs(n)))
    return values
