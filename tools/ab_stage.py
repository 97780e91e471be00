"""A/B of integrator variants selected by environment (PCK_CONS_ROWS=0/1):
DMTM steady states at the reference temperatures (tight tolerances), DMTM
DRC over a T x p grid at the input tolerances, and the synthetic network.
One JSON line per case."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import pycatkin_amd as P
    from pycatkin_amd.functions.synthetic import synthetic_system
    tag = os.environ.get('PCK_CONS_ROWS', '1')
    inp = os.path.join(ROOT, 'tests', 'golden', 'inputs', 'DMTM', 'input.json')
    cases = []
    s = P.read_from_input_file(inp)
    for tol in ((1e-10, 1e-14), (1e-8, 1e-12), (1e-6, 1e-8)):
        t = time.time()
        r = s.solve_batch(T=np.array([400.0, 600.0, 800.0]), tof_terms=('r5', 'r9'), steady=True, rtol=tol[0],
                          atol=tol[1])
        cases.append(dict(case='dmtm_steady %g/%g' % tol, status=r['status'].tolist(), nsteps=r['nsteps'].tolist(),
                          s=time.time() - t))
    TT, pp = np.meshgrid(np.linspace(400.0, 800.0, 64), np.logspace(4.0, 6.0, 64), indexing='ij')
    for tol in ((1e-6, 1e-8), (1e-8, 1e-12)):
        torch.cuda.synchronize()
        t = time.time()
        d = s.drc_batch(('r5', 'r9'), T=TT.ravel(), p=pp.ravel(), eps=5e-2, rtol=tol[0], atol=tol[1])
        torch.cuda.synchronize()
        st = d['status']
        cases.append(dict(case='dmtm_drc64x64 %g/%g' % tol, hist={int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                          s=time.time() - t))
    sim, _ = synthetic_system()
    n = int(os.environ.get('SYN_N', 4096))
    D = np.random.default_rng(0).uniform(-0.5, 0.5, (n, 4))
    torch.cuda.synchronize()
    t = time.time()
    r = sim.solve_batch(T=np.full(n, 500.0), desc={'D%d' % k: D[:, k] for k in range(4)}, tof_terms=('R0',),
                        steady=True)
    torch.cuda.synchronize()
    st = r['status']
    cases.append(dict(case='synthetic %d' % n, hist={int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                      s=time.time() - t, nsteps_med=float(np.median(r['nsteps'])), nsteps_max=int(r['nsteps'].max())))
    for c in cases:
        c['cons_rows'] = tag
        print(json.dumps(c), flush=True)


if __name__ == '__main__':
    main()
