"""Dense oracle fixture of the headline COOxVolcano grid (BASELINE configs[2]).

Points are grid nodes (i, j) of the bench grid be = linspace(-2.5, 0.5, 1024)
(activity[iCO, iO], examples/COOxVolcano/cooxvolcano.py:22-47): N_UNIFORM
uniform random nodes plus N_CORNER nodes drawn from the O-poisoned corner,
where the transient is still moving at t_end.  For each node the oracle
(oracle/mk_oracle.py, the reference algorithm restated) stores

  tight    the transient at t_end = 3600 s, lsoda (scipy BDF where lsoda
           exceeds its budget) at rtol 1e-11 / atol 1e-20 (pure relative
           control on the coverages): the reference's System.activity
           semantics (old_system.py:517-529) without integrator error -- at
           every node (NaN where both integrators exceed the evaluation budget)
  root     the steady-state rule of the device (System.solve_batch(steady=
           True), DESIGN.md "Steady state"), restated: Newton from `tight`;
           the root is the answer (`regular`) only if `tight` lies within
           ROOT_DIST * |root| + STEADY_ATOL of it in every species, else the
           answer is `tight` itself.  `newton_ok` says whether Newton found a
           resolved root at all, `crit` is the distance criterion
           max_i (|root_i - tight_i| - STEADY_ATOL) / |root_i| (inf: no root)
  ref      lsoda at the input's tolerances (ode_solver 'ode', rtol 1e-8 /
           atol 1e-10, old_system.py:359-376), i.e. what cooxvolcano.py:47
           computes, restated
  ls       least_squares(trf, xtol 1e-8, ftol 1e-8) from `ref` with the
           reference's transposed jacfun (old_system.py:385-433), restated:
           what find_steady / activity(ss_solve=True) return

as dynamic-species states (the names are stored) and log10(TOF of CO_ox).
The reference's own code run on a subset of these nodes is added by
tests/golden/make_volcano_reference.py (columns *_reference).

    OMP_NUM_THREADS=1 python tests/golden/make_volcano_fixture.py [--workers 8] [--reuse]

writes tests/golden/volcano_fixture.npz (no pickles: numpy arrays only).
--reuse keeps the stored ref / tight transients (the expensive part) and
recomputes the columns derived from them.
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
# pycatkin_amd/classes/system.py: ROOT_DIST, STEADY_TRANSIENT[1]
# (tests/test_oracle.py checks that they agree)
ROOT_DIST = 1.0e-6
STEADY_ATOL = 1.0e-22

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


def _point(arg):
    """One grid node.  The tight transient is computed at every node: it is
    the answer wherever the transient has not reached a root by t_end.  Every
    solve has a budget of 50 000 rhs evaluations (lsoda, then scipy BDF; at
    rtol 1e-11 BDF can crawl through 1e5 steps on coverages of 1e-30); a node
    where both exceed it has ok = False (reference transient) or tight_ok =
    False (tight transient) and is not compared on it.  With `reuse` (the
    stored y_ref, y_tight) only the derived columns are recomputed."""
    (i, j), reuse = arg
    be = np.linspace(-2.5, 0.5, G)
    return (i, j) + (point_at(be[i], be[j], reuse),)


def point_at(eco, eo, reuse=None):
    """The oracle columns at one (E_CO, E_O) point (see _point)."""
    from oracle import mk_oracle as O
    spec = copy.deepcopy(_spec)
    O.set_volcano_point(spec, eco, eo)

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

    def full(yd):
        y = m.y0.copy()
        y[dyn] = yd
        return y

    nan = np.full(len(dyn), np.nan)
    if reuse is not None:
        yA = full(reuse['y_ref']) if np.all(np.isfinite(reuse['y_ref'])) else None
        yT = full(reuse['y_tight']) if np.all(np.isfinite(reuse['y_tight'])) else None
    else:
        # the reference's transient (examples/COOxVolcano/input.json: ode_solver
        # 'ode' = lsoda at rtol 1e-8 / atol 1e-10)
        yA = solve(1e-8, 1e-10)
        yT = solve(1e-11, 1e-20)
    out['ok'] = yA is not None
    if yA is None:
        out['y_ref'], out['l10_ref'], out['y_ls'], out['l10_ls'] = nan, np.nan, nan, np.nan
    else:
        out['y_ref'], out['l10_ref'] = yA[dyn], l10(yA)
        yS = m.find_steady(yA.copy(), polish=False)
        out['y_ls'], out['l10_ls'] = yS[dyn], l10(yS)
    out['tight_ok'] = yT is not None
    if yT is None:
        out['y_tight'], out['l10_tight'] = nan, np.nan
        out['regular'], out['newton_ok'], out['crit'] = False, False, np.inf
        out['y_root'], out['l10_root'] = nan, np.nan
        return out
    out['y_tight'], out['l10_tight'] = yT[dyn], l10(yT)
    yR = m.find_steady(yT.copy(), dist=ROOT_DIST, dist_atol=STEADY_ATOL)
    out['regular'], out['newton_ok'], out['crit'] = bool(m.regular), bool(m.newton_ok), float(m.root_crit)
    out['y_root'], out['l10_root'] = yR[dyn], l10(yR)
    return out


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
    ap.add_argument('--reuse', action='store_true', help='keep the stored ref / tight transients')
    args = ap.parse_args()
    pts = pick_points()
    if args.limit:
        pts = pts[:args.limit]
    old = None
    if args.reuse:
        old = dict(np.load(OUT))
        assert [(int(a), int(b)) for a, b in zip(old['i'], old['j'])][:len(pts)] == pts
    jobs = [(p, None if old is None else dict(y_ref=old['y_ref'][k], y_tight=old['y_tight'][k]))
            for k, p in enumerate(pts)]
    t = time.time()
    res = {}
    with mp.get_context('fork').Pool(args.workers, initializer=_init) as pool:
        for k, (i, j, o) in enumerate(pool.imap_unordered(_point, jobs, chunksize=4)):
            res[(i, j)] = o
            if k % 100 == 0:
                print('%d / %d points, %.0f s' % (k, len(pts), time.time() - t), flush=True)
    keys = [p for p in pts]
    arr = {'i': np.array([p[0] for p in keys], np.int32), 'j': np.array([p[1] for p in keys], np.int32),
           'dyn': np.array(dyn_names()), 'grid': np.array([-2.5, 0.5, G], float)}
    for f in ('ok', 'regular', 'tight_ok', 'newton_ok'):
        arr[f] = np.array([res[p][f] for p in keys], bool)
    arr['crit'] = np.array([res[p]['crit'] for p in keys], float)
    arr['root_dist'] = np.array([ROOT_DIST, STEADY_ATOL])
    if old is not None:               # columns of make_volcano_reference.py survive a --reuse
        for k, v in old.items():
            if k.endswith('_reference') or k.startswith('ref_'):
                arr[k] = v
    for f in ('root', 'tight', 'ref', 'ls'):
        arr['y_' + f] = np.array([res[p]['y_' + f] for p in keys], float)
        arr['l10_' + f] = np.array([res[p]['l10_' + f] for p in keys], float)
    np.savez_compressed(OUT, **arr)
    print('wrote %s: %d points, %d regular, %d degenerate, %.0f s' % (OUT, len(keys), arr['regular'].sum(),
                                                                      (~arr['regular']).sum(), time.time() - t))


if __name__ == '__main__':
    main()
