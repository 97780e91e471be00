"""Diagnostic: step counts of DMTM condition 2552 of tools/group_ab.py (T 647.6 K,
p 6.0e5 Pa) under 1e-12 relative perturbations of T or p, record-table and
compile-time group kernels: is the step count chaotic in rounding?"""
import os, sys, numpy as np
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
import torch, pycatkin_amd as P
ROOT = os.environ.get('GRAFT_REPO_ROOT', '/root/repo')
s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'DMTM', 'input.json'))
T0, p0 = 400 + 400 * 39 / 63, 10 ** (4 + 2 * 56 / 63)
n = 256
rel = np.linspace(-1e-12, 1e-12, n)
for mode in ('0', '1'):
    os.environ['PCK_GRP_CT'] = mode
    for what in ('T', 'p'):
        T = np.full(n, T0) * (1 + (rel if what == 'T' else 0))
        p = np.full(n, p0) * (1 + (rel if what == 'p' else 0))
        r = s.solve_batch(T=T, p=p, tof_terms=('r5', 'r9'))
        ns = r['nsteps']
        print('CT=%s perturb %s: steps min %d median %d max %d; >1000: %d of %d; tof spread %.3e' % (
            mode, what, ns.min(), np.median(ns), ns.max(), (ns > 1000).sum(), n, np.ptp(r['tof']) / abs(r['tof']).mean()), flush=True)
