"""Diagnostic: the volcano network on the lane-group solver against the lane
solver (status flips, TOF agreement) in one process per setting of
PCK_GRP_BALANCE / PCK_GRP_TAB given on the command line as VAR=VALUE pairs.

    python tools/balance_probe.py [PCK_GRP_BALANCE=0] [PCK_GRP_TAB=0]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
for kv in sys.argv[1:]:
    k, v = kv.split('=')
    os.environ[k] = v


def main():
    import pycatkin_amd as P
    from pycatkin_amd.functions.volcano import set_volcano_energies
    s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    net = s.device(('CO_ox',))
    rng = np.random.default_rng(11)
    n = 1024
    kw = dict(T=np.full(n, 600.0), desc={'ECO': rng.uniform(-2.5, 0.5, n), 'EO': rng.uniform(-2.5, 0.5, n)},
              tof_terms=('CO_ox',), steady=False)
    net.set_plan_mode(1)
    a = s.solve_batch(**kw)
    net.set_plan_mode(2)
    b = s.solve_batch(**kw)
    kw['steady'] = True
    net.set_plan_mode(1)
    c = s.solve_batch(**kw)
    net.set_plan_mode(2)
    d = s.solve_batch(**kw)
    rel = np.abs(b['tof'] - a['tof']) / np.maximum(np.abs(a['tof']), 1e-300)
    print(json.dumps(dict(env=sys.argv[1:], transient_status=[np.unique(a['status']).tolist(), np.unique(b['status']).tolist()],
                          transient_tof_rel_max=float(rel.max()), transient_nsteps=[int(a['nsteps'].sum()), int(b['nsteps'].sum())],
                          steady_flip=float(np.mean(c['status'] != d['status'])),
                          steady_status=[np.bincount(c['status'], minlength=6).tolist(), np.bincount(d['status'], minlength=6).tolist()],
                          y0_grp=d['y'][:, 0].tolist(), y0_lane=c['y'][:, 0].tolist())))


if __name__ == '__main__':
    main()
