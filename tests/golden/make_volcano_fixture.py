"""Dense oracle fixture of the headline COOxVolcano grid (BASELINE configs[2]).

Points are grid nodes (i, j) of the bench grid be = linspace(-2.5, 0.5, 1024)
(activity[iCO, iO], examples/COOxVolcano/cooxvolcano.py:22-47): N_UNIFORM
uniform random nodes plus N_CORNER nodes drawn from the O-poisoned corner,
where the polish meets degenerate roots (device status 4).  For each node the
oracle (oracle/mk_oracle.py, the reference algorithm restated) stores

  root     the Newton polish of `ref` (below); `regular` says whether Newton
           converged quadratically (mk_oracle.ClassicModel._polish)
  tight    the transient at t_end = 3600 s, lsoda (scipy BDF where lsoda
           exceeds its budget) at rtol 1e-11 / atol 1e-20 (pure relative control on the coverages): the
           reference's System.activity semantics (old_system.py:517-529)
           without integrator error -- at every node (NaN where both
           integrators exceed the evaluation budget)
  ref      the reference's own path: lsoda at the input's tolerances
           (ode_solver 'ode', rtol 1e-8 / atol 1e-10, old_system.py:359-376),
           i.e. what cooxvolcano.py:47 computes
  ls       least_squares(trf, xtol 1e-8, ftol 1e-8) from `ref`
           (old_system.py:385-433), what find_steady / activity(ss_solve=True)
           return

as dynamic-species states (plan order CO*, O*, O2*, * is not assumed: the
names are stored) and log10(TOF of CO_ox).

    OMP_NUM_THREADS=1 python tests/golden/make_volcano_fixture.py [--workers 8]

writes tests/golden/volcano_fixture.npz (no pickles: numpy arrays only).
"""
import argparse
import copy
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
INPUT = os.path.join(HERE, 'inputs', 'COOxVolcano', 'input.json')
OUT = os.path.join(HERE, 'volcano_fixture.npz')
G = 1024
N_UNIFORM = 2048
N_CORNER = 512
SEED = 20261017

_spec = None
_dyn = None


def _init():
    global _spec, _dyn
    sys.path.insert(0, ROOT)
    from oracle import mk_oracle as O
    _spec = O.load_spec(INPUT)
    sp = copy.deepcopy(_spec)
    O.set_volcano_point(sp, -1.0, -1.0)       # the user energies the network needs
    m = O.ClassicModel(sp)
    _dyn = [m.snames[i] for i in m.dyn]


def dyn_names():
    _init()
    return list(_dyn)


class _Budget(Exception):
    pass


def _point(ij):
    """One grid node.  The tight transient is computed at every node: the
    device reports it wherever its own Newton meets a degenerate root, which
    near the boundary of the two regimes need not be where the oracle's does.
    Every solve has a budget of 50 000 rhs evaluations (lsoda, then scipy
    BDF; at rtol 1e-11 BDF can crawl through 1e5 steps on coverages of 1e-30);
    a node where both exceed it has ok = False (reference transient) or
    tight_ok = False (tight transient) and is not compared on it."""
    from oracle import mk_oracle as O
    i, j = ij
    be = np.linspace(-2.5, 0.5, G)
    spec = copy.deepcopy(_spec)
    O.set_volcano_point(spec, be[i], be[j])

    class Counted(O.ClassicModel):
        budget = None

        def rhs(self, y):
            if self.budget is not None:
                self.budget -= 1
                if self.budget < 0:
                    raise _Budget()
            return super().rhs(y)
    m = Counted(spec)
    dyn = m.dyn
    out = {}

    def l10(y):
        t = m.tof(y, ['CO_ox'])
        return np.log10(t) if t > 0 else -np.inf

    def solve(rtol, atol):
        """lsoda, or scipy BDF where lsoda exceeds the evaluation budget; None if both do"""
        for method in ('LSODA', 'BDF'):
            m.budget = 50000
            try:
                y, sol = m.solve_odes(rtol=rtol, atol=atol, method=method)
                if sol.status == 0:
                    return y
            except _Budget:
                pass
            finally:
                m.budget = None
        return None

    nan = np.full(len(dyn), np.nan)
    out['y_tight'], out['l10_tight'], out['tight_ok'] = nan, np.nan, False
    # the reference's transient (examples/COOxVolcano/input.json: ode_solver
    # 'ode' = lsoda at rtol 1e-8 / atol 1e-10), the start of both polishes
    yA = solve(1e-8, 1e-10)
    out['ok'] = yA is not None
    if yA is None:                 # no oracle answer at this node (recorded, never compared)
        out['regular'] = False
        for f in ('ref', 'root', 'ls'):
            out['y_' + f], out['l10_' + f] = nan, np.nan
        return i, j, out
    out['y_ref'], out['l10_ref'] = yA[dyn], l10(yA)
    yR = m.find_steady(yA.copy())
    out['regular'] = bool(m.regular)
    out['y_root'], out['l10_root'] = yR[dyn], l10(yR)
    yS = m.find_steady(yA.copy(), polish=False)
    out['y_ls'], out['l10_ls'] = yS[dyn], l10(yS)
    # every node: a device that classifies a node degenerate reports its
    # tight transient, whatever the oracle's classification
    yT = solve(1e-11, 1e-20)
    if yT is not None:
        out['y_tight'], out['l10_tight'], out['tight_ok'] = yT[dyn], l10(yT), True
    return i, j, out


def pick_points(corner_cells=None):
    """N_UNIFORM uniform grid nodes + N_CORNER nodes of the strong-O corner
    (E_O < -1.6 eV, E_CO > -1.3 eV: where the oracle's coarse classification
    finds the degenerate roots), distinct."""
    rng = np.random.default_rng(SEED)
    be = np.linspace(-2.5, 0.5, G)
    uni = rng.choice(G * G, N_UNIFORM, replace=False)
    io = np.nonzero(be < -1.6)[0]
    ic = np.nonzero(be > -1.3)[0]
    cor = rng.choice(ic.size * io.size, 4 * N_CORNER, replace=False)
    cor = ic[cor // io.size] * G + io[cor % io.size]
    cor = [k for k in cor if k not in set(uni.tolist())][:N_CORNER]
    flat = np.concatenate([uni, np.asarray(cor, dtype=np.int64)])
    return [(int(k // G), int(k % G)) for k in flat]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workers', type=int, default=8)
    ap.add_argument('--limit', type=int, default=0, help='first N points only (a quick check)')
    args = ap.parse_args()
    pts = pick_points()
    if args.limit:
        pts = pts[:args.limit]
    t = time.time()
    res = {}
    with mp.get_context('fork').Pool(args.workers, initializer=_init) as pool:
        for k, (i, j, o) in enumerate(pool.imap_unordered(_point, pts, chunksize=4)):
            res[(i, j)] = o
            if k % 100 == 0:
                print('%d / %d points, %.0f s' % (k, len(pts), time.time() - t), flush=True)
    keys = [p for p in pts]
    arr = {'i': np.array([p[0] for p in keys], np.int32), 'j': np.array([p[1] for p in keys], np.int32),
           'dyn': np.array(dyn_names()), 'grid': np.array([-2.5, 0.5, G], float)}
    for f in ('ok', 'regular', 'tight_ok'):
        arr[f] = np.array([res[p][f] for p in keys], bool)
    for f in ('root', 'tight', 'ref', 'ls'):
        arr['y_' + f] = np.array([res[p]['y_' + f] for p in keys], float)
        arr['l10_' + f] = np.array([res[p]['l10_' + f] for p in keys], float)
    np.savez_compressed(OUT, **arr)
    print('wrote %s: %d points, %d regular, %d degenerate, %.0f s' % (OUT, len(keys), arr['regular'].sum(),
                                                                      (~arr['regular']).sum(), time.time() - t))


if __name__ == '__main__':
    main()
