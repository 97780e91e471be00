"""A/B of the lane-group kernels on one config (GPU): the record-table kernel
(PCK_GRP_CT=0) against the compile-time-network kernel, same inputs.  Prints
per-condition step-count statistics, the conditions whose counts differ most,
and the wall time of each.

    python tools/group_ab.py dmtm_drc|dmtm|ch4 [n]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
INPUTS = os.path.join(ROOT, 'tests', 'golden', 'inputs')


def main():
    import torch
    import pycatkin_amd as P
    which = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    if which.startswith('dmtm'):
        s = P.read_from_input_file(os.path.join(INPUTS, 'DMTM', 'input.json'))
        g = int(round(np.sqrt(n)))
        TT, pp = np.meshgrid(np.linspace(400.0, 800.0, g), np.logspace(4.0, 6.0, g), indexing='ij')
        T, p = TT.ravel(), pp.ravel()
        if which == 'dmtm_drc':
            run = lambda: s.drc_batch(('r5', 'r9'), T=T, p=p, eps=5.0e-2)
        else:
            run = lambda: s.solve_batch(T=T, p=p, tof_terms=('r5', 'r9'))
    else:
        s = P.read_from_input_file(os.path.join(INPUTS, 'CH4', 'input.json'), formulation='patched')
        for r, st in (('C_ads', 'sC'), ('O_ads', 'sO')):
            s.reactions[r].dErxn_user = 1.0
            s.states[st].Gelec = 1.0
        T = np.linspace(473.0, 573.0, n)
        run = lambda: s.solve_batch(T=T, t0=0.0, t_end=1e4, rtol=1e-10, atol=1e-12)
    out = {}
    for mode in ('1', '0'):
        os.environ['PCK_GRP_CT'] = mode
        run()
        torch.cuda.synchronize()
        t = time.time()
        r = run()
        torch.cuda.synchronize()
        dt = time.time() - t
        ns = np.asarray(r['nsteps'] if 'nsteps' in r else r['status'] * 0)
        out[mode] = (dt, r)
        print('PCK_GRP_CT=%s: %.1f ms, statuses %s' % (mode, dt * 1e3, np.unique(r['status'], return_counts=True)))
    if 'nsteps' in out['1'][1]:
        a, b = out['1'][1]['nsteps'].astype(float), out['0'][1]['nsteps'].astype(float)
        print('steps CT: mean %.1f max %d p99 %.0f; tables: mean %.1f max %d p99 %.0f' % (
            a.mean(), a.max(), np.percentile(a, 99), b.mean(), b.max(), np.percentile(b, 99)))
        d = np.argsort(-np.abs(a - b))[:10]
        for k in d:
            print('  condition %d: T %.1f, CT %d steps, tables %d steps' % (k, T[k], a[k], b[k]))


if __name__ == '__main__':
    main()
