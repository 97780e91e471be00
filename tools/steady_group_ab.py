"""Diagnostic (GPU): wall time of steady group solves (System.solve_batch,
steady=True, Newton polish) on the quad-group kernel against the 16-lane
kernel (PCK_GRP_QUAD_NEWTON=0): DMTM over a 64 x 64 T x p grid and the CH4
network over 16 384 temperatures.

    python tools/steady_group_ab.py [OUT.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
INPUTS = os.path.join(ROOT, 'tests', 'golden', 'inputs')


def timed(fn, reps=5):
    import torch
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best, r


def main():
    import pycatkin_amd as P
    out = {}
    d = P.read_from_input_file(os.path.join(INPUTS, 'DMTM', 'input.json'))
    TT, pp = np.meshgrid(np.linspace(400.0, 800.0, 64), np.logspace(4.0, 6.0, 64), indexing='ij')
    c = P.read_from_input_file(os.path.join(INPUTS, 'CH4', 'input.json'), formulation='patched')
    for r, st in (('C_ads', 'sC'), ('O_ads', 'sO')):
        c.reactions[r].dErxn_user = 1.0
        c.states[st].Gelec = 1.0
    cases = {'dmtm_steady_4096': lambda: d.solve_batch(T=TT.ravel(), p=pp.ravel(), tof_terms=('r5', 'r9'), steady=True),
             'ch4_steady_16384': lambda: c.solve_batch(T=np.linspace(473.0, 573.0, 16384), steady=True)}
    for name, fn in cases.items():
        res = {}
        for mode in ('1', '0'):
            os.environ['PCK_GRP_QUAD_NEWTON'] = mode
            t, r = timed(fn)
            res[mode] = dict(wall_ms=1e3 * t, status=dict(zip(*[v.tolist() for v in np.unique(r['status'], return_counts=True)])))
            res[mode]['r'] = r
        a, b = res['1']['r'], res['0']['r']
        ok = (a['status'] == 0) & (b['status'] == 0)
        out[name] = dict(quad_ms=res['1']['wall_ms'], lane16_ms=res['0']['wall_ms'],
                         status_quad=res['1']['status'], status_lane16=res['0']['status'],
                         status_equal=bool(np.array_equal(a['status'], b['status'])),
                         max_rel_y=float((np.abs(a['y'][:, ok] - b['y'][:, ok]) /
                                          np.maximum(np.abs(b['y'][:, ok]), 1e-14)).max(initial=0.0)))
    os.environ.pop('PCK_GRP_QUAD_NEWTON')
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], 'w'), indent=1)


if __name__ == '__main__':
    main()
