"""Diagnostic (test infrastructure): run the oracle's scipy BDF path (the
reference's solve_ivp(BDF), old_system.py:350-354) on every condition the
device reported as failed (status 1-3) in a tools/bench_configs.py --dump
file, and record whether scipy BDF fails on it too.

    python tools/check_failures_bdf.py gpurun_out/fail_synthetic.json OUT.json [--n-total 16384]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def _bdf(args):
    idx, D = args
    from _synth import spec_of
    from oracle import mk_oracle as O
    from pycatkin_amd.functions.synthetic import synthetic_network
    m = O.ClassicModel(spec_of(synthetic_network(), np.asarray(D)), T=500.0)
    y, sol = m.solve_odes(rtol=1e-8, atol=1e-10)
    return dict(idx=idx, bdf_status=int(sol.status), message=sol.message, steps=int(len(sol.t)),
                min_y=float(np.min(sol.y[m.dyn])))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dump')
    ap.add_argument('out')
    ap.add_argument('--workers', type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    d = json.load(open(a.dump))
    D = np.array([d['desc']['D%d' % k] for k in range(4)]).T
    jobs = [(int(i), D[k].tolist()) for k, i in enumerate(d['idx'])]
    with mp.get_context('spawn').Pool(a.workers) as pool:
        res = pool.map(_bdf, jobs)
    for r, st in zip(res, d['status']):
        r['device_status'] = int(st)
    both = sum(1 for r in res if r['bdf_status'] != 0)
    out = dict(n_device_failed=len(res), n_bdf_failed_too=both, cases=res)
    json.dump(out, open(a.out, 'w'), indent=1)
    print('device failures %d, scipy BDF fails on %d of them' % (len(res), both))


if __name__ == '__main__':
    main()
