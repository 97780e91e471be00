"""Run the REFERENCE PyCatKin code (importable in this build container from
/root/reference, never on the GPU box) on nodes of the dense volcano fixture
and add its answers to tests/golden/volcano_fixture.npz:

  y_ref_reference / l10_ref_reference
        old_system.System.solve_odes() with the input's ode_solver 'ode'
        (lsoda, rtol 1e-8 / atol 1e-10, nsteps 1e5 log-spaced output times,
        old_system.py:359-376) -> solution[-1]: what the volcano driver's
        activity() reports (examples/COOxVolcano/cooxvolcano.py:47)
  y_ls_reference / l10_ls_reference
        old_system.System.find_steady() from there (least_squares trf with the
        reference's own jacfun, old_system.py:385-433): what
        activity(ss_solve=True) / find_steady report
  ref_ok_reference
        lsoda reached t_end (the reference's loop stops at the first
        unsuccessful step and leaves zero rows behind)

on all N_CORNER corner nodes and the first N_UNI uniform nodes of the
fixture.  The states come from tests/golden/make_golden.py's duck-typed
states (the reference's state.py needs `ase`, absent here); everything else
-- reactions, rate constants, species ODEs, Jacobian, the integrator and
least_squares calls -- is the reference's code, unmodified.

    OMP_NUM_THREADS=1 python tests/golden/make_volcano_reference.py [--workers 8]
"""
import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, 'volcano_fixture.npz')
N_UNI = 256
N_CORNER = 512
SCOg, SO2g = 2.0487e-3, 2.1261e-3          # cooxvolcano.py:13-14

_sys = None
_spec = None


def _init():
    global _sys, _spec
    sys.path.insert(0, HERE)
    import make_golden as MG                 # noqa: E402 (puts /root/reference on sys.path)
    from oracle import mk_oracle as O
    _spec = O.load_spec(os.path.join(MG.REF, 'examples/COOxVolcano/input.json'))
    _sys = MG.build_reference_system(_spec, 'classic')
    sysd = _spec['system']
    _sys.params['ode_solver'] = 'ode'       # examples/COOxVolcano/input.json
    _sys.params['nsteps'] = int(sysd.get('nsteps', 1e5))


def _node(arg):
    """cooxvolcano.py:28-47 at one (E_CO, E_O), then find_steady."""
    from oracle import mk_oracle as O
    k, ECO, EO = arg
    s, spec = _sys, _spec
    T = spec['system']['T']
    s.reactions['CO_ads'].dErxn_user = ECO
    s.reactions['CO_ads'].dGrxn_user = ECO + SCOg * T
    s.reactions['2O_ads'].dErxn_user = 2.0 * EO
    s.reactions['2O_ads'].dGrxn_user = 2.0 * EO + SO2g * T
    # the duck states' energies (descriptor-scaled states) read the same user
    # energies from the spec they share (make_golden.volcano_vectors)
    spec['reactions']['CO_ads']['user'].update(dErxn_user=ECO, dGrxn_user=ECO + SCOg * T)
    spec['reactions']['2O_ads']['user'].update(dErxn_user=2.0 * EO, dGrxn_user=2.0 * EO + SO2g * T)
    th = O.Thermo(spec, T, spec['system']['p'])
    EO2 = th.elec('sO2')
    s.reactions['O2_ads'].dErxn_user = EO2
    s.reactions['O2_ads'].dGrxn_user = EO2 + SO2g * T
    s.reactions['CO_ox'].dEa_fwd_user = np.max((th.elec('SRTS_ox') - (ECO + EO), 0.0))
    s.reactions['O2_2O'].dEa_fwd_user = np.max((th.elec('SRTS_O2') - EO2, 0.0))
    s.solution = None
    s.solve_odes()
    y_end = np.array(s.solution[-1], float)
    ok = bool(np.any(y_end != 0.0))
    s.reaction_terms(y_end)
    names = list(s.species_map.keys())
    t_end = float(s.rates[names.index('CO_ox'), 0] - s.rates[names.index('CO_ox'), 1])
    y_ls = np.array(s.find_steady(), float)
    s.reaction_terms(y_ls)
    t_ls = float(s.rates[names.index('CO_ox'), 0] - s.rates[names.index('CO_ox'), 1])
    return k, ok, y_end, t_end, y_ls, t_ls, list(s.snames)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workers', type=int, default=8)
    ap.add_argument('--limit', type=int, default=0)
    args = ap.parse_args()
    fx = dict(np.load(OUT))
    lo, hi, G = fx['grid']
    be = np.linspace(lo, hi, int(G))
    n = fx['i'].size
    sel = list(range(N_UNI)) + list(range(n - N_CORNER, n))
    if args.limit:
        sel = sel[:args.limit]
    jobs = [(k, float(be[fx['i'][k]]), float(be[fx['j'][k]])) for k in sel]
    dyn = [str(x) for x in fx['dyn']]
    cols = {c: np.full((n, len(dyn)), np.nan) for c in ('y_ref_reference', 'y_ls_reference')}
    l10 = {c: np.full(n, np.nan) for c in ('l10_ref_reference', 'l10_ls_reference')}
    okc = np.zeros(n, bool)
    done = np.zeros(n, bool)
    t = time.time()
    with mp.get_context('fork').Pool(args.workers, initializer=_init) as pool:
        for m, (k, ok, y_end, t_end, y_ls, t_ls, snames) in enumerate(pool.imap_unordered(_node, jobs, chunksize=2)):
            pos = [snames.index(d) for d in dyn]
            cols['y_ref_reference'][k] = y_end[pos]
            cols['y_ls_reference'][k] = y_ls[pos]
            l10['l10_ref_reference'][k] = np.log10(t_end) if t_end > 0 else -np.inf
            l10['l10_ls_reference'][k] = np.log10(t_ls) if t_ls > 0 else -np.inf
            okc[k], done[k] = ok, True
            if m % 50 == 0:
                print('%d / %d nodes, %.0f s' % (m, len(jobs), time.time() - t), flush=True)
    fx.update(cols)
    fx.update(l10)
    fx['ref_ok_reference'] = okc
    fx['ref_done_reference'] = done
    np.savez_compressed(OUT, **fx)
    print('wrote %s: reference run on %d nodes (%d reached t_end), %.0f s' % (OUT, done.sum(), okc.sum(),
                                                                            time.time() - t))


if __name__ == '__main__':
    main()
