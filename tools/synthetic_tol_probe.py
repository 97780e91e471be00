"""Diagnostic (GPU): the synthetic fixture's 324 conditions
(tests/golden/synthetic_fixture.npz) solved by the steady rule at several
transient tolerances; per tolerance the max / p99 relative error of
log10(TOF) (the TOF itself where negative) and of the coverages against the
oracle's tight answer, and the device time for the bench's 65 536 set.

    python tools/synthetic_tol_probe.py 1e-6 1e-7 1e-8      (rtol values; atol 1e-22)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pycatkin_amd.functions.synthetic import synthetic_system
    sim, _ = synthetic_system()
    plan = sim.plan(('R0',))
    fx = dict(np.load(os.path.join(ROOT, 'tests', 'golden', 'synthetic_fixture.npz')))
    D = fx['desc']
    names = [str(x) for x in fx['dyn']]
    Dall = np.random.default_rng(0).uniform(-0.5, 0.5, (65536, 4))
    out = []
    for rt in [float(a) for a in sys.argv[1:]]:
        r = sim.solve_batch(T=np.full(D.shape[0], 500.0), desc={'D%d' % k: D[:, k] for k in range(4)},
                            tof_terms=('R0',), steady=True, rtol=rt, atol=1e-22)
        tof = r['tof']
        pos = (tof > 0) & (fx['tof'] > 0)
        err = np.where(pos, np.abs(np.log10(np.where(pos, tof, 1)) - fx['l10']) / np.abs(np.where(pos, fx['l10'], 1)),
                       np.abs(tof - fx['tof']) / np.abs(fx['tof']))
        y = r['y'][[plan.dyn.index(nm) for nm in names]].T
        cov = np.max((np.abs(y - fx['y_root']) - 1e-20) / np.abs(fx['y_root']), axis=1)
        torch.cuda.synchronize()
        t = time.time()
        rb = sim.solve_batch(T=np.full(65536, 500.0), desc={'D%d' % k: Dall[:, k] for k in range(4)},
                             tof_terms=('R0',), steady=True, rtol=rt, atol=1e-22)
        torch.cuda.synchronize()
        line = dict(rtol=rt, max_rel_l10=float(err.max()), p99_rel_l10=float(np.percentile(err, 99)),
                    n_over_1e6=int((err > 1e-6).sum()), max_rel_cov=float(cov.max()),
                    p99_rel_cov=float(np.percentile(cov, 99)), s_65536=time.time() - t,
                    statuses={int(k): int(v) for k, v in zip(*np.unique(rb['status'], return_counts=True))})
        print(json.dumps(line), flush=True)
        out.append(line)


if __name__ == '__main__':
    main()
