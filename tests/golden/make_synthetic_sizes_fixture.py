"""Oracle fixture of three smaller synthetic networks (pycatkin_amd/functions/
synthetic.py: synthetic_network(n_species, n_reactions, seed=1)), one per
group kernel:

  syn40   40 dynamic species / 120 reactions -> the 64-lane group kernel
  syn24   24 dynamic species / 72 reactions  -> the 32-lane group kernel
  syn12   12 dynamic species / 36 reactions  -> the quad-group kernel

N conditions each, random descriptors (np.random.default_rng(7), uniform in
[-0.5, 0.5]^4), T = 500 K, the steady-state rule to t_end = 1e8 s (long
enough that most conditions settle: the 1e4 s of the 50-species config
leaves every one of them moving).  Per condition the oracle
(mk_oracle.steady_rule: lsoda at rtol 1e-11 / atol 1e-20, Newton, the root
where the transient has reached it to ROOT_DIST) stores the answer y, the
tight transient end y_tight, `regular`, `crit` and the TOF of R0.

    OMP_NUM_THREADS=1 python tests/golden/make_synthetic_sizes_fixture.py [--workers 8]

writes tests/golden/synthetic_sizes_fixture.npz (numpy arrays only).
"""
import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, 'synthetic_sizes_fixture.npz')
NETS = {'syn40': (40, 120), 'syn24': (24, 72), 'syn12': (12, 36)}
SEED_NET = 1
N = 64
T = 500.0
T_END = 1.0e8
ROOT_DIST = 1.0e-6          # pycatkin_amd/classes/system.py ROOT_DIST
STEADY_ATOL = 1.0e-22       # STEADY_TRANSIENT[1]


def descriptors():
    return np.random.default_rng(7).uniform(-0.5, 0.5, (N, 4))


def _cond(arg):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    from _synth import spec_of
    from oracle import mk_oracle as O
    from pycatkin_amd.functions.synthetic import synthetic_network
    key, k, d = arg
    ns, nr = NETS[key]
    m = O.ClassicModel(spec_of(synthetic_network(n_species=ns, n_reactions=nr, seed=SEED_NET), np.asarray(d), T), T=T)
    dyn = m.dyn
    r = O.steady_rule(m, dist=ROOT_DIST, dist_atol=STEADY_ATOL, budget=400000, t_end=T_END)
    names = [m.snames[i] for i in dyn]
    if r is None:
        nan = np.full(len(dyn), np.nan)
        return key, k, dict(ok=False, regular=False, crit=np.inf, y=nan, y_tight=nan, tof=np.nan), names
    return key, k, dict(ok=True, regular=r['regular'], crit=r['crit'], y=r['y'][dyn], y_tight=r['y_tight'][dyn],
                        tof=m.tof(r['y'], ['R0'])), names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workers', type=int, default=8)
    args = ap.parse_args()
    D = descriptors()
    jobs = [(key, k, D[k]) for key in NETS for k in range(N)]
    t = time.time()
    res, names = {}, {}
    with mp.get_context('spawn').Pool(args.workers) as pool:
        for key, k, o, nm in pool.imap_unordered(_cond, jobs):
            res[(key, k)], names[key] = o, nm
    out = dict(desc=D, T=np.array(T), t_end=np.array(T_END))
    for key in NETS:
        rows = [res[(key, k)] for k in range(N)]
        out[key + '_dyn'] = np.array(names[key])
        for f in ('ok', 'regular'):
            out[key + '_' + f] = np.array([r[f] for r in rows], bool)
        for f in ('crit', 'tof'):
            out[key + '_' + f] = np.array([r[f] for r in rows], float)
        for f in ('y', 'y_tight'):
            out[key + '_' + f] = np.array([r[f] for r in rows], float)
        print('%s: %d / %d answered, %d steady state reached' % (key, out[key + '_ok'].sum(), N,
                                                                  out[key + '_regular'].sum()))
    np.savez_compressed(OUT, **out)
    print('wrote %s (%.0f s)' % (OUT, time.time() - t))


if __name__ == '__main__':
    main()
