"""Diagnostic (GPU): one Butadiene pathway set at one temperature -- device
rate constants, transient end and steady answer against the oracle's."""
import copy
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
import make_butadiene_fixture as M  # noqa: E402
from oracle import mk_oracle as O  # noqa: E402
from pycatkin_amd.functions.load_input import read_from_input_file  # noqa: E402

ci, ti = int(sys.argv[1]), int(sys.argv[2])
case, pw = M.CASES[ci]
T = float(M.TEMPS[ti])
D = os.path.join(ROOT, 'tests', 'golden', 'inputs', 'Butadiene')
dft = read_from_input_file(os.path.join(D, 'input.json'))
mkm = read_from_input_file(os.path.join(D, 'input_mkm.json'), base_system=dft)
s = copy.deepcopy(mkm)
keep = M.kept_reactions(list(s.reactions), case, pw)
for r in list(s.reactions):
    if r not in keep:
        del s.reactions[r]
s.names_to_indices()
plan = s.plan()
M._init()
spec = M.case_spec(case, pw)
m = O.ClassicModel(spec, T=T)
kf, kr = s.rate_constants_batch(T=np.array([T]))
print(case, T, 'NS', len(plan.dyn))
for a, name in enumerate(plan.reactions):
    j = m.rnames.index(name)
    print('%-22s kf %.6e / %.6e  kr %.6e / %.6e  rel %.1e %.1e' % (
        name, kf[a, 0], m.kf[j], kr[a, 0], m.kr[j], abs(kf[a, 0] / m.kf[j] - 1), abs(kr[a, 0] / m.kr[j] - 1)))
out = O.steady_rule(m, budget=400000)
dyn = [m.snames[i] for i in m.dyn]
rt = s.solve_batch(T=np.array([T]), rtol=1e-6, atol=1e-22)
rs = s.solve_batch(T=np.array([T]), steady=True, screen=None)
print('device steady status', rs['status'][0], 'steps', rs['nsteps'][0], '; transient status', rt['status'][0])
print('%-12s %-13s %-13s %-13s %-13s' % ('species', 'oracle trans', 'device trans', 'oracle root', 'device steady'))
for i, n in enumerate(plan.dyn):
    k = dyn.index(n)
    print('%-12s %.6e %.6e %.6e %.6e' % (n, out['y_tight'][m.dyn][k], rt['y'][i, 0], m.newton_root[k] if out['newton_ok'] else np.nan,
                                         rs['y'][i, 0]))
