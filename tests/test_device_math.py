"""Host checks of the device math constants (no GPU): the fp64 exp scheme
of tpe_device.h (scaled exponent, minimax polynomial, 2^kExpTabBits-entry table) is
re-evaluated in numpy from the constants parsed out of the header and
compared with a 60-digit reference; the Philox4x32-10 round function is
checked against its published known-answer vectors."""
import os
import re
from decimal import Decimal, getcontext

import numpy as np

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    'hyperopt_amd', 'csrc')
HDR = os.path.join(CSRC, 'tpe_device.h')
TAB = os.path.join(CSRC, 'tpe_exp_table.h')


def _consts():
    txt = open(TAB).read()
    num = r'([-+0-9.eEx]+)'
    bits = int(re.search(r'kExpTabBits = (\d+)', txt).group(1))
    scale = float(re.search(r'kExpScale = ' + num, txt).group(1))
    c = [float(m) for m in re.findall(r'kExpC\d = ' + num, txt)]
    body = re.search(r'kExp2Tab\[\d+\] = \{(.*?)\};', txt, re.S).group(1)
    tab = np.array([float.fromhex(t.strip()) for t in body.split(',') if t.strip()])
    return bits, scale, c, tab


def _exp_scaled(u, bits, c, tab):
    """numpy restatement of tpe_device.h:exp_scaled"""
    k = np.rint(u)
    f = u - k
    p = c[-1]
    for cj in reversed(c[:-1]):
        p = p * f + cj
    p = p * f + 1.0
    ki = k.astype(np.int64)
    return np.ldexp(p * tab[ki & ((1 << bits) - 1)], (ki >> bits).astype(np.int32))


def test_exp_constants_and_accuracy():
    getcontext().prec = 60
    ln2 = Decimal(2).ln()
    bits, scale, c, tab = _consts()
    c = [v for v in c if v != 0.0]          # kExpC<d> past kExpDeg are 0
    txt = open(TAB).read()
    deg = int(re.search(r'kExpDeg = (\d+)', txt).group(1))
    poly_err = float(re.search(r'kExpPolyErr = ([-+0-9.e]+)', txt).group(1))
    assert len(c) == deg
    N = 1 << bits
    assert len(tab) == N
    assert scale == float(Decimal(N) / ln2)
    for i in range(0, N, 7):
        assert tab[i] == float(Decimal(2) ** (Decimal(i) / N))
    # the polynomial is within ~10% of Taylor (a minimax refit, not a new form)
    x = ln2 / N
    fact = Decimal(1)
    for n in range(1, deg + 1):
        fact *= n
        assert abs(c[n - 1] / float(x ** n / fact) - 1) < 0.1
    # per-term error budget: polynomial + rounding, far below the 1e-9 bar
    assert poly_err < 5e-14
    L = np.longdouble(str(ln2))
    rng = np.random.RandomState(0)
    for lo in (-1.0, -300.0, -N * 700 / float(ln2)):
        u = rng.uniform(lo, 0, 200000)
        ref = np.exp(u.astype(np.longdouble) * L / N)
        rel = np.abs((_exp_scaled(u, bits, c, tab) - ref) / ref)
        assert float(rel.max()) < poly_err + 6e-16


def _philox(c, k):
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
    c = list(c)
    k0, k1 = k
    for _ in range(10):
        p0, p1 = M0 * c[0], M1 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF,
             ((p0 >> 32) ^ c[3] ^ k1) & 0xFFFFFFFF, p0 & 0xFFFFFFFF]
        k0, k1 = (k0 + W0) & 0xFFFFFFFF, (k1 + W1) & 0xFFFFFFFF
    return c


def test_philox_known_answers():
    """Random123 kat_vectors for philox4x32-10 -- the round structure used by
    tpe_device.h:philox4x32_10."""
    assert _philox([0, 0, 0, 0], [0, 0]) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert _philox([0xffffffff] * 4, [0xffffffff] * 2) == \
        [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert _philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344],
                   [0xa4093822, 0x299f31d0]) == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]
    txt = open(HDR).read()
    for const in ('0xD2511F53u', '0xCD9E8D57u', '0x9E3779B9u', '0xBB67AE85u'):
        assert const in txt


def _np_sum_restated(a):
    """The summation order tpe_build.hip:block_np_sum and the host fold
    (tpe_engine.hip:np_pairwise_sum) implement: 8192-element chunks added in
    order to 0.0, each chunk summed pairwise (leaves <= 128, 8 accumulators)."""
    def leaf(x):
        n = len(x)
        if n < 8:
            r = 0.0
            for v in x:
                r += v
            return r
        r = list(x[:8])
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] += x[i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        for v in x[i:]:
            res += v
        return res

    def pw(x):
        if len(x) <= 128:
            return leaf(x)
        n2 = len(x) // 2
        n2 -= n2 % 8
        return pw(x[:n2]) + pw(x[n2:])

    r = 0.0
    for c in range(0, len(a), 8192):
        r += pw(a[c:c + 8192])
    return r


def test_numpy_sum_order():
    """np.sum's float64 summation order, which the device posterior builder
    reproduces to get bit-identical normalised weights and p_accept."""
    rng = np.random.RandomState(0)
    for n in list(range(1, 40)) + [127, 128, 129, 1000, 8191, 8192, 8193, 9976, 20000, 50001]:
        a = rng.uniform(0, 1, n) * 10 ** rng.uniform(-3, 3, n)
        assert _np_sum_restated(a.tolist()) == np.sum(a), n
