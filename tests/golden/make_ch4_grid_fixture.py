"""CH4 descriptor-grid fixture: the patched System's steady-state loop over
an E_C x E_O grid (the workflow pycatkin/functions/analysis.py:27-116
post-processes: per point C_ads / O_ads dErxn_user and sC / sO Gelec set to
the descriptors, then SteadyStateSolver.solve_ode, solver.py:374-418 -- the
surface transient from the normalised start state to 1e4 s) at 523 K,
integrated by the oracle (oracle.mk_oracle.PatchedModel, lsoda at rtol 1e-13
/ atol 1e-20).  Points where lsoda does not reach 1e4 s (O-rich corner:
the coverages run away) are stored with status != 0.  lsoda_err: how far
scipy's lsoda at the solve's own tolerances (rtol 1e-10 / atol 1e-12) lands
from that tight answer (max abs) -- the conditioning of the transient end at
points that have not settled by 1e4 s.

Output: tests/golden/ch4_grid_fixture.npz (C_range, O_range, T, y [nC, nO, 16]
in the oracle's surface order `names`, status, max_f, lsoda_err [nC, nO]).

    OMP_NUM_THREADS=1 python tests/golden/make_ch4_grid_fixture.py
"""
import multiprocessing as mp
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
OUT = os.path.join(HERE, 'ch4_grid_fixture.npz')
C_RANGE = np.array([0.5, 1.0, 1.5, 2.0])
O_RANGE = np.array([0.2, 0.6, 1.0, 1.4])
T = 523.0


def _one(k):
    from oracle import mk_oracle as O
    iC, iO = divmod(k, O_RANGE.size)
    spec = O.ch4_setup(O.load_spec(os.path.join(HERE, 'inputs', 'CH4', 'input.json')), C_RANGE[iC], O_RANGE[iO])
    m = O.PatchedModel(spec, T=T)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        y, sol = m.solve_ode(tmax=1e4, rtol=1e-13, atol=1e-20, method='LSODA')
        y2, sol2 = m.solve_ode(tmax=1e4, rtol=1e-10, atol=1e-12, method='LSODA')
    err = float(np.max(np.abs(y2 - y))) if (sol.status == 0 and sol2.status == 0) else np.nan
    names = sorted(m.index, key=m.index.get)[m.ngas:]
    return k, y, int(sol.status), float(np.max(np.abs(m.fun_ss(y)))), names, err


def main():
    with mp.get_context('fork').Pool(8) as pool:
        res = sorted(pool.map(_one, range(C_RANGE.size * O_RANGE.size)))
    shape = (C_RANGE.size, O_RANGE.size)
    np.savez_compressed(OUT, C_range=C_RANGE, O_range=O_RANGE, T=T,
                        y=np.array([r[1] for r in res]).reshape(shape + (-1,)),
                        status=np.array([r[2] for r in res]).reshape(shape),
                        max_f=np.array([r[3] for r in res]).reshape(shape), names=np.array(res[0][4]),
                        lsoda_err=np.array([r[5] for r in res]).reshape(shape))
    for r in res:
        print('EC %.1f EO %.1f status %d max|f| %.2e lsoda at 1e-10 off by %.2e' % (
            C_RANGE[r[0] // O_RANGE.size], O_RANGE[r[0] % O_RANGE.size], r[2], r[3], r[5]))
    print('wrote', OUT)


if __name__ == '__main__':
    main()
