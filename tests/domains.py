"""The reference's benchmark domains (hyperopt/tests/test_domains.py:48-200),
rebuilt with hyperopt_amd.hp / scope.  Each returns (name, space, loss_target);
the objective is the identity on the evaluated space (a result dict)."""
import numpy as np

from hyperopt_amd import STATUS_OK, hp, scope
from hyperopt_amd.space import as_apply


def quadratic1():
    return {'loss': (hp.uniform('x', -5, 5) - 3) ** 2, 'status': STATUS_OK}


def q1_choice():
    o_x = hp.choice('o_x', [(-3, hp.uniform('x_neg', -5, 5)), (3, hp.uniform('x_pos', -5, 5))])
    return {'loss': (o_x[0] - o_x[1]) ** 2, 'status': STATUS_OK}


def q1_lognormal():
    return {'loss': scope.min(0.1 * (hp.lognormal('x', 0, 2) - 10) ** 2, 10),
            'status': STATUS_OK}


def n_arms(N=2):
    rng = np.random.RandomState(123)
    x = hp.choice('x', [0, 1])
    reward_mus = as_apply([-1] + [0] * (N - 1))
    reward_sigmas = as_apply([1] * N)
    return {'loss': scope.normal(reward_mus[x], reward_sigmas[x], rng=rng),
            'loss_variance': 1.0, 'status': STATUS_OK}


def distractor():
    x = hp.uniform('x', -15, 15)
    f1 = 1.0 / (1.0 + scope.exp(-x))
    f2 = 2 * scope.exp(-(x + 10) ** 2)
    return {'loss': -f1 - f2, 'status': STATUS_OK}


def gauss_wave():
    x = hp.uniform('x', -20, 20)
    t = hp.choice('curve', [x, x + np.pi])
    f1 = scope.sin(t)
    f2 = 2 * scope.exp(-(t / 5.0) ** 2)
    return {'loss': -(f1 + f2), 'status': STATUS_OK}


def gauss_wave2():
    rng = np.random.RandomState(123)
    var = .1
    x = hp.uniform('x', -20, 20)
    amp = hp.uniform('amp', 0, 1)
    t = (scope.normal(0, var, rng=rng) + 2 * scope.exp(-(x / 5.0) ** 2))
    return {'loss': -hp.choice('hf', [t, t + scope.sin(x) * amp]),
            'loss_variance': var, 'status': STATUS_OK}


def many_dists():
    a = hp.choice('a', [0, 1, 2])
    b = hp.randint('b', 10)
    c = hp.uniform('c', 4, 7)
    d = hp.loguniform('d', -2, 0)
    e = hp.quniform('e', 0, 10, 3)
    f = hp.qloguniform('f', 0, 3, 2)
    g = hp.normal('g', 4, 7)
    h = hp.lognormal('h', -2, 2)
    i = hp.qnormal('i', 0, 10, 2)
    j = hp.qlognormal('j', 0, 2, 1)
    k = hp.pchoice('k', [(.1, 0), (.9, 1)])
    z = a + b + c + d + e + f + g + h + i + j + k
    return {'loss': scope.float(scope.log(1e-12 + z ** 2)), 'status': STATUS_OK}


def branin():
    x = hp.uniform('x', -5., 10.)
    y = hp.uniform('y', 0., 15.)
    pi = float(np.pi)
    loss = ((y - (5.1 / (4 * pi ** 2)) * x ** 2 + 5 * x / pi - 6) ** 2 +
            10 * (1 - 1 / (8 * pi)) * scope.cos(x) + 10)
    return {'loss': loss, 'loss_variance': 0, 'status': STATUS_OK}


ALL = dict(quadratic1=quadratic1, q1_choice=q1_choice, q1_lognormal=q1_lognormal,
           n_arms=n_arms, distractor=distractor, gauss_wave=gauss_wave,
           gauss_wave2=gauss_wave2, many_dists=many_dists, branin=branin)
