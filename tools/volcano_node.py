"""Diagnostic (GPU): one volcano grid point through the steady rule's pieces
-- the transient at STEADY_TRANSIENT, the rule itself, the rule without the
distance test (root_dist 0) and a Newton polish of the transient end
(t_end = t0) -- with the per-species distances the rule compares.

    python tools/volcano_node.py ECO EO [ECO EO ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import pycatkin_amd as P
    from pycatkin_amd.classes.system import ROOT_DIST, STEADY_TRANSIENT
    from pycatkin_amd.functions.volcano import set_volcano_energies
    vals = [float(x) for x in sys.argv[1:]]
    eco, eo = np.array(vals[0::2]), np.array(vals[1::2])
    n = eco.size
    s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    plan = s.plan(('CO_ox',))
    kw = dict(T=np.full(n, 600.0), desc={'ECO': eco, 'EO': eo}, tof_terms=('CO_ox',))
    tr = s.solve_batch(rtol=STEADY_TRANSIENT[0], atol=STEADY_TRANSIENT[1], **kw)
    rule = s.solve_batch(steady=True, **kw)
    nodist = s.solve_batch(steady=True, root_dist=0.0, **kw)
    pol = s.solve_batch(steady=True, y0=tr['y'], t0=0.0, t_end=0.0, **kw)
    np.set_printoptions(precision=10, linewidth=160)
    print('species', plan.dyn)
    for c in range(n):
        yT, z = tr['y'][:, c], nodist['y'][:, c]
        d = np.abs(z - yT)
        print('E_CO %.12g E_O %.12g: transient steps %d status %d; rule status %d; root_dist 0 status %d; '
              'polish of the transient end status %d' % (eco[c], eo[c], tr['nsteps'][c], tr['status'][c],
                                                         rule['status'][c], nodist['status'][c], pol['status'][c]))
        print('  transient end', yT)
        print('  root (dist 0)', z)
        print('  polish root  ', pol['y'][:, c])
        print('  |root - yT| / (ROOT_DIST |root| + atol)', d / (ROOT_DIST * np.abs(z) + STEADY_TRANSIENT[1]))


if __name__ == '__main__':
    main()
