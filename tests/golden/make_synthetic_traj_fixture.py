"""Oracle trajectory fixture for the 32-lane group kernel's dense output:
the 24-species / 72-reaction synthetic network of
make_synthetic_sizes_fixture.py at four of its conditions (rows 0-3), the
transient from the start state sampled at 0 and 30 log-spaced times in
[1e-8, 1e4] s (old_system.py:359-376: the reference's output grid is
log-spaced) by the oracle's model (mk_oracle.ClassicModel rhs / jac,
scipy LSODA at rtol 1e-12 / atol 1e-20 with t_eval; checked against BDF at
the same tolerances, `bdf_rel`).

    OMP_NUM_THREADS=1 python tests/golden/make_synthetic_traj_fixture.py

writes tests/golden/synthetic_traj_fixture.npz.
"""
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
from make_synthetic_sizes_fixture import NETS, SEED_NET, T, descriptors  # noqa: E402

OUT = os.path.join(HERE, 'synthetic_traj_fixture.npz')
KEY = 'syn24'
ROWS = [0, 1, 2, 3]
T_OUT = np.concatenate([[0.0], np.logspace(-8.0, 4.0, 30)])


def _one(row):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    from scipy.integrate import solve_ivp
    from _synth import spec_of
    from oracle import mk_oracle as O
    from pycatkin_amd.functions.synthetic import synthetic_network
    ns, nr = NETS[KEY]
    m = O.ClassicModel(spec_of(synthetic_network(n_species=ns, n_reactions=nr, seed=SEED_NET), descriptors()[row], T),
                       T=T)
    m._set_reach(m.y0)
    out = {}
    for method in ('LSODA', 'BDF'):
        sol = solve_ivp(lambda t, y: m.rhs(y), (0.0, T_OUT[-1]), m.y0, method=method, jac=lambda t, y: m.jac(y),
                        rtol=1e-12, atol=1e-20, t_eval=T_OUT)
        assert sol.status == 0, (row, method, sol.message)
        out[method] = sol.y[m.dyn].T                   # [n_out, NS]
    big = out['LSODA'] > 1e-12
    rel = float(np.max(np.abs(out['BDF'] - out['LSODA'])[big] / out['LSODA'][big]))
    return row, out['LSODA'], rel, [m.snames[i] for i in m.dyn]


def main():
    with mp.get_context('spawn').Pool(4) as pool:
        res = sorted(pool.map(_one, ROWS), key=lambda r: r[0])
    np.savez_compressed(OUT, rows=np.array(ROWS), t_out=T_OUT, traj=np.array([r[1] for r in res]),
                        bdf_rel=np.array([r[2] for r in res]), dyn=np.array(res[0][3]))
    print('wrote %s; lsoda vs BDF at 1e-12: max rel %.2e on components above 1e-12' % (OUT, max(r[2] for r in res)))


if __name__ == '__main__':
    main()
