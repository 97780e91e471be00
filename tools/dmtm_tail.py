"""Diagnostic (GPU): the DMTM DRC bench grid (64 x 64, T 400-800 K x p
1e4-1e6 Pa, eps 5e-2, input tolerances) -- the conditions with the most
integrator steps (summed over the 2R+1 solves), which set the launch's time.

    [PCK_LIB=...] python tools/dmtm_tail.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import pycatkin_amd as P
    s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'DMTM', 'input.json'))
    TT, pp = np.meshgrid(np.linspace(400.0, 800.0, 64), np.logspace(4.0, 6.0, 64), indexing='ij')
    T, p = TT.ravel(), pp.ravel()
    r = s.drc_batch(('r5', 'r9'), T=T, p=p, eps=5.0e-2)
    ns = r['nsteps']
    print('lib', os.environ.get('PCK_LIB', 'default'), 'steps per condition: mean %.1f p99 %.0f max %d'
          % (ns.mean(), np.percentile(ns, 99), ns.max()))
    for k in np.argsort(ns)[::-1][:8]:
        print('  cond %d T %.3f p %.6g: %d steps, status %d' % (k, T[k], p[k], ns[k], r['status'][k]))


if __name__ == '__main__':
    main()
