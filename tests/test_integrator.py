"""The integrator's coefficient sets (csrc/mk_solver.h namespaces rodas4 /
rodas4_dense) against their derivation and order (tools/rodas_dense.py), and
the Newton constants the oracle shares with the device.  CPU only."""
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, 'tools'))

import rodas_dense as RD  # noqa: E402

HEADER = os.path.join(ROOT, 'pycatkin_amd', 'csrc', 'mk_solver.h')
NAMES = ['a21', 'a31', 'a32', 'a41', 'a42', 'a43', 'a51', 'a52', 'a53', 'a54', 'C21', 'C31', 'C32', 'C41', 'C42',
         'C43', 'C51', 'C52', 'C53', 'C54', 'C61', 'C62', 'C63', 'C64', 'C65', 'D21', 'D22', 'D23', 'D24', 'D25',
         'D31', 'D32', 'D33', 'D34', 'D35']


def _header_sets():
    """{True: RODAS4P constants, False: RODAS4 constants} parsed from the
    header's `#if PCK_RODAS4P ... #else ... #endif` blocks."""
    text = open(HEADER).read()
    out = {True: {}, False: {}}
    for block in re.findall(r'#if PCK_RODAS4P\n(.*?)#else\n(.*?)#endif', text, re.S):
        for flag, body in zip((True, False), block):
            for name, expr in re.findall(r'\b([aCD]\d\d) = ([-0-9.e/ ]+?)[,;]', body):
                out[flag][name] = eval(expr)            # numbers and one division (-40.0 / 7.0)
    return out


def _as_method(c):
    return dict(A=[[], [c['a21']], [c['a31'], c['a32']], [c['a41'], c['a42'], c['a43']],
                   [c['a51'], c['a52'], c['a53'], c['a54']]],
                C=[[], [c['C21']], [c['C31'], c['C32']], [c['C41'], c['C42'], c['C43']],
                   [c['C51'], c['C52'], c['C53'], c['C54']], [c['C61'], c['C62'], c['C63'], c['C64'], c['C65']]],
                D2=[c['D2%d' % j] for j in range(1, 6)], D3=[c['D3%d' % j] for j in range(1, 6)])


def test_header_coefficients_are_the_derived_sets():
    sets = _header_sets()
    for flag, ref in ((True, RD.RODAS4P), (False, RD.RODAS4)):
        c = sets[flag]
        assert sorted(c) == sorted(NAMES), sorted(set(NAMES) ^ set(c))
        m = _as_method(c)
        for key in ('A', 'C'):
            for row, row_ref in zip(m[key], ref[key]):
                assert np.allclose(row, row_ref, rtol=1e-15, atol=0), (flag, key)
        assert np.allclose(m['D2'], ref['D2'], rtol=1e-15, atol=0)
        assert np.allclose(m['D3'], ref['D3'], rtol=1e-15, atol=0)


def test_dense_output_order_conditions():
    """b(s) = s m + s (1 - s) (D2 + s D3) meets the four order-3 conditions as
    polynomials in s, for both sets; RODAS4P's also vanishes in the stiff limit."""
    for M in (RD.RODAS4P, RD.RODAS4):
        W, r2, r3 = RD.dense_conditions(M)
        assert np.abs(W @ np.asarray(M['D2']) - r2).max() < 1e-12
        assert np.abs(W @ np.asarray(M['D3']) - r3).max() < 1e-12
    kinf = RD.stiff_limit_stages(RD.RODAS4P)[:5]
    assert abs(kinf @ np.asarray(RD.RODAS4P['D2'])) < 1e-12
    assert abs(kinf @ np.asarray(RD.RODAS4P['D3'])) < 1e-12


def test_step_order_nonstiff_and_prothero_robinson():
    """Order 4 on a nonstiff problem for both sets; on the Prothero-Robinson
    problem (lam = -1e4) RODAS4 falls to order ~1 and RODAS4P keeps ~3 --
    the reason the device runs RODAS4P (DESIGN.md "Integrator")."""
    def f1(y):
        return np.array([y[1], -np.sin(y[0]) + 0.1 * y[1] ** 2])

    def J1(y):
        return np.array([[0, 1.0], [-np.cos(y[0]), 0.2 * y[1]]])

    def run(M, f, J, y, T, N):
        for _ in range(N):
            y, _ = RD.step(M, f, J, y, T / N)
        return y
    ref = run(RD.RODAS4P, f1, J1, np.array([1.0, 0.5]), 2.0, 4000)
    lam = -1e4

    def f2(z):
        return np.array([lam * (z[0] - np.sin(z[1])) + np.cos(z[1]), 1.0])

    def J2(z):
        return np.array([[lam, -lam * np.cos(z[1]) - np.sin(z[1])], [0, 0]])
    orders = {}
    for name, M in (('4p', RD.RODAS4P), ('4', RD.RODAS4)):
        e = [np.abs(run(M, f1, J1, np.array([1.0, 0.5]), 2.0, N) - ref).max() for N in (20, 40)]
        assert 3.7 < np.log2(e[0] / e[1]) < 4.5, (name, e)
        e = [abs(run(M, f2, J2, np.zeros(2), 1.0, N)[0] - np.sin(1.0)) for N in (10, 20)]
        orders[name] = np.log2(e[0] / e[1])
    assert orders['4p'] > 2.5 and orders['4'] < 1.5, orders


def test_newton_constants_shared_with_the_oracle():
    from oracle import mk_oracle as O
    text = open(HEADER).read()
    for name, value in (('PCK_BALANCE_CONV', O.BALANCE_CONV), ('PCK_STEP_FLOOR', O.STEP_FLOOR),
                        ('PCK_BALANCE_TOL', O.BALANCE_TOL)):
        m = re.search(r'#define %s ([-0-9.e]+)' % name, text)
        assert m and float(m.group(1)) == value, name
