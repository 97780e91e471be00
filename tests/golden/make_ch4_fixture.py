"""CH4 fixture: BASELINE configs[0] as bench.py --config ch4 runs it
(test/CH4_input.json in the patched system.py formulation, descriptor
energies E_C = E_O = 1 eV, SteadyStateSolver.solve_ode from the normalised
start state to 1e4 s; pycatkin/classes/solver.py:374-418) at 8 of the
bench's 16 384 temperatures (473-573 K), integrated by the oracle
(oracle.mk_oracle.PatchedModel) to rtol 1e-13 / atol 1e-20 with lsoda, so
that the fixture's own error sits far below the 1e-6 the device is held to.
scipy BDF at the same tolerances agrees to <= 1.2e-12 relative on every
component above 1e-14 (checked here, `bdf_rel`).

Output: tests/golden/ch4_fixture.npz (T, idx into the bench grid, y [8, 16]
in the oracle's surface order `names`).

    OMP_NUM_THREADS=1 python tests/golden/make_ch4_fixture.py
"""
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
OUT = os.path.join(HERE, 'ch4_fixture.npz')
N_BENCH = 16384
IDX = np.linspace(0, N_BENCH - 1, 8).round().astype(int)


def _one(k):
    from oracle import mk_oracle as O
    spec = O.ch4_setup(O.load_spec(os.path.join(HERE, 'inputs', 'CH4', 'input.json')), 1.0, 1.0)
    T = float(np.linspace(473.0, 573.0, N_BENCH)[k])
    m = O.PatchedModel(spec, T=T)
    y, sol = m.solve_ode(tmax=1e4, rtol=1e-13, atol=1e-20, method='LSODA')
    yb, solb = m.solve_ode(tmax=1e4, rtol=1e-13, atol=1e-20, method='BDF')
    assert sol.status == 0 and solb.status == 0
    big = y > 1e-14
    names = sorted(m.index, key=m.index.get)[m.ngas:]
    return k, T, y, float(np.max(np.abs(yb - y)[big] / y[big])), names


def main():
    with mp.get_context('fork').Pool(8) as pool:
        res = sorted(pool.map(_one, list(IDX)))
    np.savez_compressed(OUT, idx=np.array([r[0] for r in res]), T=np.array([r[1] for r in res]),
                        y=np.array([r[2] for r in res]), bdf_rel=np.array([r[3] for r in res]),
                        names=np.array(res[0][4]))
    print('wrote %s; lsoda vs BDF at 1e-13: max rel %.2e' % (OUT, max(r[3] for r in res)))


if __name__ == '__main__':
    main()
