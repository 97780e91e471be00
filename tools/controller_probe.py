"""Diagnostic (CPU, test infrastructure): step counts of the device's Rodas4
controller against Gustafsson's predictive controller on random volcano grid
points, through the numpy mirror (tools/rodas_mirror.py, ctrl='std' / 'pred').

    python tools/controller_probe.py N
"""
import copy
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p_ in (ROOT, os.path.join(ROOT, 'tools'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p_)
os.environ['CLIPMODE'] = 'hybrid'
import rodas_mirror as RM
from oracle import mk_oracle as O
spec0 = O.load_spec(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
rng = np.random.default_rng(1)
pts = -2.5 + 3.0 * rng.uniform(0, 1, (int(sys.argv[1]), 2))
out = []
for ECO, EO in pts:
    spec = copy.deepcopy(spec0); O.set_volcano_point(spec, ECO, EO, None)
    m = O.ClassicModel(spec, T=None)
    dyn = m.dyn; full = m.y0.copy()
    def f(y):
        full[dyn] = y; return m.rhs(full)[dyn]
    def J(y):
        full[dyn] = y; return m.jac(full)[np.ix_(dyn, dyn)]
    C = m.conservation(); Cr, piv = O._rref(C)
    res = {}
    for ctrl in ('std', 'pred'):
        tr = []
        y, st, n = RM.rodas4(f, J, m.y0[dyn].copy(), 0.0, 3600.0, 1e-8, 1e-10, cons=Cr, trace=tr, ctrl=ctrl)
        acc = sum(1 for r in tr if r[3])
        res[ctrl] = (n, acc, n - acc, y)
    d = np.max(np.abs(res['std'][3] - res['pred'][3]) / np.maximum(np.abs(res['std'][3]), 1e-20))
    out.append((res['std'][:3], res['pred'][:3], d))
    print(ECO, EO, res['std'][:3], res['pred'][:3], '%.2e' % d, flush=True)
S = np.array([o[0] for o in out]); P = np.array([o[1] for o in out])
print('std total', S.sum(0), 'pred total', P.sum(0), 'ratio', P[:, 0].sum() / S[:, 0].sum())
