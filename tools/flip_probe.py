"""Diagnostic (GPU): where the device's Newton classification of the dense
volcano fixture nodes (tests/golden/volcano_fixture.npz) differs from the
oracle's, separate the integrator from the polish.

For every fixture node the device runs
  A  the transient alone (rtol 1e-8 / atol 1e-10 to t_end): y_T, TOF
  B  transient + Newton (30 iterations, the library default), no retry
  C  transient + Newton with 200 iterations, no retry
  D  Newton alone from A's y_T (t_end = t0, y0 = y_T)
and writes gpurun_out/flip_probe.npz; the oracle side (its Newton from the
device's own y_T) runs on the CPU afterwards (tools/flip_probe.py --analyse).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, 'gpurun_out', 'flip_probe.npz')


def device():
    import pycatkin_amd as P
    from pycatkin_amd.functions.volcano import set_volcano_energies
    fx = dict(np.load(os.path.join(ROOT, 'tests', 'golden', 'volcano_fixture.npz')))
    lo, hi, G = fx['grid']
    be = np.linspace(lo, hi, int(G))
    eco, eo = be[fx['i']], be[fx['j']]
    n = eco.size
    s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    plan = s.plan(('CO_ox',))
    kw = dict(T=np.full(n, 600.0), desc={'ECO': eco, 'EO': eo}, tof_terms=('CO_ox',))
    a = s.solve_batch(steady=False, **kw)
    b = s.solve_batch(steady=True, retry=None, **kw)
    c = s.solve_batch(steady=True, retry=None, newton_iters=200, **kw)
    d = s.solve_batch(steady=True, retry=None, y0=a['y'], t_end=0.0, t0=0.0, **kw)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez(OUT, dyn=np.array(plan.dyn), eco=eco, eo=eo, yT=a['y'], tofT=a['tof'], stA=a['status'],
             stB=b['status'], yB=b['y'], tofB=b['tof'], stC=c['status'], yC=c['y'], stD=d['status'], yD=d['y'])
    for k in 'BCD':
        st = locals()[k.lower()]['status']
        print(k, np.unique(st, return_counts=True), 'regular vs fixture:', int(((st == 0) != fx['regular']).sum()),
              'flips', flush=True)


def analyse():
    import copy
    from oracle import mk_oracle as O
    r = dict(np.load(OUT))
    fx = dict(np.load(os.path.join(ROOT, 'tests', 'golden', 'volcano_fixture.npz')))
    spec = O.load_spec(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    dyn = [str(x) for x in r['dyn']]
    agree = 0
    rows = []
    for k in range(r['eco'].size):
        sp = copy.deepcopy(spec)
        O.set_volcano_point(sp, r['eco'][k], r['eo'][k])
        m = O.ClassicModel(sp)
        y = m.y0.copy()
        for q, nm in enumerate(dyn):
            y[m.idx[nm]] = r['yT'][q, k]
        m.find_steady(y.copy())
        dev = r['stD'][k] == 0
        agree += (dev == m.regular)
        if dev != m.regular or (r['stB'][k] == 0) != fx['regular'][k]:
            rows.append((k, float(r['eco'][k]), float(r['eo'][k]), int(r['stB'][k]), int(r['stC'][k]),
                         int(r['stD'][k]), bool(m.regular), bool(fx['regular'][k])))
    print('device Newton vs oracle Newton from the same device transient end: %d / %d agree'
          % (agree, r['eco'].size))
    print('k, E_CO, E_O, dev(B 30 it), dev(C 200 it), dev(D from y_T), oracle from dev y_T, fixture')
    for row in rows:
        print(row)


if __name__ == '__main__':
    if '--analyse' in sys.argv:
        analyse()
    else:
        device()
