"""Oracle fixture of the 1 024 random volcano points of
tests/test_gpu_group.py::test_group_solver_matches_lane_solver_on_volcano
(T = 600 K, E_CO and E_O uniform in [-2.5, 0.5] eV from default_rng(11)).

For each point the oracle (oracle/mk_oracle.py) gives the steady-state rule of
System.solve_batch(steady=True) restated exactly as in
make_volcano_fixture.py (point_at): the tight transient at t_end, the Newton
root from it, `regular` (the root is the answer) and the distance criterion
`crit` = max_i (|root_i - tight_i| - atol) / |root_i|, which the rule
compares with ROOT_DIST.  The GPU test then names, for every point where the
lane and group solvers classify differently, how far the oracle's criterion
lies from the threshold.

    OMP_NUM_THREADS=1 python tests/golden/make_split_fixture.py [--workers 8]

writes tests/golden/split_fixture.npz (numpy arrays only).
"""
import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import make_volcano_fixture as F  # noqa: E402

OUT = os.path.join(HERE, 'split_fixture.npz')
N = 1024
SEED = 11


def points():
    """the test's draw: ECO first, then EO (tests/test_gpu_group.py)"""
    rng = np.random.default_rng(SEED)
    eco = rng.uniform(-2.5, 0.5, N)
    eo = rng.uniform(-2.5, 0.5, N)
    return eco, eo


def _one(arg):
    k, eco, eo = arg
    return k, F.point_at(eco, eo)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workers', type=int, default=8)
    args = ap.parse_args()
    eco, eo = points()
    t = time.time()
    res = {}
    with mp.get_context('fork').Pool(args.workers, initializer=F._init) as pool:
        for m, (k, o) in enumerate(pool.imap_unordered(_one, [(k, eco[k], eo[k]) for k in range(N)], chunksize=4)):
            res[k] = o
            if m % 128 == 0:
                print('%d / %d points, %.0f s' % (m, N, time.time() - t), flush=True)
    arr = dict(ECO=eco, EO=eo, dyn=np.array(F.dyn_names()), root_dist=np.array([F.ROOT_DIST, F.STEADY_ATOL]))
    for f in ('tight_ok', 'regular', 'newton_ok'):
        arr[f] = np.array([res[k][f] for k in range(N)], bool)
    arr['crit'] = np.array([res[k]['crit'] for k in range(N)], float)
    for f in ('root', 'tight'):
        arr['y_' + f] = np.array([res[k]['y_' + f] for k in range(N)], float)
        arr['l10_' + f] = np.array([res[k]['l10_' + f] for k in range(N)], float)
    np.savez_compressed(OUT, **arr)
    print('wrote %s: %d points, %d regular, %d not reached, %d without a tight transient, %.0f s'
          % (OUT, N, arr['regular'].sum(), (~arr['regular'] & arr['tight_ok']).sum(), (~arr['tight_ok']).sum(),
             time.time() - t))


if __name__ == '__main__':
    main()
