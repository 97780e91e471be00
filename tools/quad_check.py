"""Diagnostic (GPU): the quad-group kernel (mk_quad.h, PCK_GRP_QUAD) against
the 16-lane compile-time-network group kernel (PCK_GRP_QUAD=0) on the CH4
transient (SteadyStateSolver's rtol 1e-10 / atol 1e-12, 256 temperatures) and
the DMTM transient DRC (64 temperatures): statuses, states, TOFs, step counts.

    python tools/quad_check.py [OUT.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
INPUTS = os.path.join(ROOT, 'tests', 'golden', 'inputs')


def main():
    import pycatkin_amd as P
    out = {}
    s = P.read_from_input_file(os.path.join(INPUTS, 'CH4', 'input.json'), formulation='patched')
    for r, st in (('C_ads', 'sC'), ('O_ads', 'sO')):
        s.reactions[r].dErxn_user = 1.0
        s.states[st].Gelec = 1.0
    net = s.device()
    kw = dict(T=np.linspace(473.0, 573.0, 256), t0=0.0, t_end=1e4, rtol=1e-10, atol=1e-12)
    res = {}
    for mode in ('2', '0'):
        os.environ['PCK_GRP_QUAD'] = mode
        res[mode] = s.solve_batch(**kw)
        res[mode]['kernel'] = net.group_kernel()
    a, b = res['2'], res['0']
    rel = np.abs(a['y'] - b['y']) / np.maximum(np.abs(b['y']), 1e-30)
    out['ch4'] = dict(kernel_quad=int(a['kernel']), kernel_ref=int(b['kernel']),
                      status_quad=np.unique(a['status'], return_counts=True)[0].tolist(),
                      status_ref=np.unique(b['status'], return_counts=True)[0].tolist(),
                      status_equal=bool(np.array_equal(a['status'], b['status'])),
                      max_rel_y=float(rel.max()), max_rel_y_above_1em12=float(rel[np.abs(b['y']) > 1e-12].max()),
                      steps_quad=int(a['nsteps'].sum()), steps_ref=int(b['nsteps'].sum()))
    d = P.read_from_input_file(os.path.join(INPUTS, 'DMTM', 'input.json'))
    res = {}
    for mode in ('2', '0'):
        os.environ['PCK_GRP_QUAD'] = mode
        res[mode] = d.drc_batch(('r5', 'r9'), T=np.linspace(400.0, 800.0, 64), eps=5.0e-2)
        res[mode]['kernel'] = d.device(('r5', 'r9')).group_kernel()
    a, b = res['2'], res['0']
    out['dmtm_drc'] = dict(kernel_quad=int(a['kernel']), kernel_ref=int(b['kernel']),
                           status_equal=bool(np.array_equal(a['status'], b['status'])),
                           status_quad=np.unique(a['status']).tolist(),
                           max_abs_xi=float(max(np.abs(a[n] - b[n]).max() for n in d.reactions)),
                           max_rel_tof0=float(np.max(np.abs(a['tof0'] - b['tof0']) / np.abs(b['tof0']))),
                           steps_quad=int(a['nsteps'].sum()), steps_ref=int(b['nsteps'].sum()))
    os.environ.pop('PCK_GRP_QUAD')
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], 'w'), indent=1)


if __name__ == '__main__':
    main()
