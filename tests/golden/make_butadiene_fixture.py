"""Butadiene MKM fixture: examples/Butadiene/butadiene_mkm.py:35-80, the
reference's 24-adsorbate microkinetic model (input_mkm.json) whose
'reaction derived reactions' take their energies from the DFT base system
(input.json; pycatkin/classes/reaction.py:312-339), over the script's 17
temperatures (523-923 K) and its 8 pathway sets.

Two answers per (pathway set, T):

  oracle (oracle/mk_oracle.py, load_spec(..., base_spec=...)):
    y_tight   the transient to t_end = 86 400 s at rtol 1e-11 / atol 1e-20
    y_rule    the device's steady-state rule from there (steady_rule: Newton,
              the root where the transient has reached it to 1e-6, else the
              transient end); regular / crit say which
  reference (the reference's own old_system.py / reaction.py code, run here
  with tests/golden/make_golden.py's duck-typed states -- pycatkin's
  state.py needs `ase`, absent in this image):
    y_ref     System.solve_odes() -> solution[-1]: scipy solve_ivp BDF at the
              input's rtol 1e-6 / atol 1e-8 (old_system.py:315-357)
    y_ls      System.find_steady(store_steady=True) from there
              (least_squares trf, old_system.py:385-433)
    bd_ref    get_tof_for_given_reactions(['3F-3G', '4I-4K', '6G-6H']) at
              solution[-1] (presets.py:585-597), the script's bd_tof

Every vector is over the case's dynamic species (`dyn_<case>`, the
reference's sorted adsorbate order).  Output: tests/golden/butadiene_fixture.npz.

    OMP_NUM_THREADS=1 python tests/golden/make_butadiene_fixture.py [--workers 8]
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
INPUTS = os.path.join(HERE, 'inputs', 'Butadiene')
OUT = os.path.join(HERE, 'butadiene_fixture.npz')
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

TEMPS = np.linspace(523.0, 923.0, 17)                 # butadiene_mkm.py:33
BD_TERMS = ['3F-3G', '4I-4K', '6G-6H']

# butadiene_mkm.py:16-28
ADS = ['9D-9C', 'ethanol-1A', '8A-8C', 'H2O-9B', 'acetaldehyde-10B', 'crotonaldehyde-2N']
P123 = ['1A-1C', '2A-2C', '2F-2H', '2J-2L', '2L-2N', '3A-3C', '3D-3F', '3F-3G'] + ADS
P124 = ['1A-1C', '2A-2C', '2F-2H', '4A-4C', '4D-4Ca', '4D-4F', '4F-4H', '4I-4K'] + ADS
P156 = ['1A-1C', '5A-5C', '6A-6C', '6C-6E', '6E-6G', '6G-6H'] + ADS
SOUZA = ['12A-12C', '12C-12E', '12E-12G', 'butanol-12G']
JONAS = ['3Ci-3Ciii', '3Civ-3Cvi', 'butanol-3Cvi']
ALL3 = sorted(set(P123 + P124 + P156))
WITH_SOUZA = ALL3 + SOUZA + ['7Ei-7Eiii', 'ethylacetate-7Eiii']
WITH_JONAS = ALL3 + JONAS + ['7Ei-7Eiii', 'ethylacetate-7Eiii']
DOPED = ['1A-1C', '2F-2H', '5A-5C', '6A-6C']
CASES = [('p123_p124_p156', ALL3), ('p123', P123), ('p124', P124), ('p156', P156),
         ('with_souza_byproducts', WITH_SOUZA), ('with_jonas_byproducts', WITH_JONAS),
         ('with_Cu_dopant', WITH_JONAS), ('with_Zn_dopant', WITH_JONAS)]


def kept_reactions(all_names, case, pathways):
    """butadiene_mkm.py:48-61: the reactions a pathway set keeps (in the
    system's order), a dopant case swapping each doped step for its
    '<step>_<Cu|Zn>' version."""
    discard, add = [], []
    for r in all_names:
        if r not in pathways:
            discard.append(r)
        elif 'dopant' in case and r in DOPED:
            discard.append(r)
            add.append(r + '_' + case.split('_')[1])
    return [r for r in all_names if not (r in discard and r not in add)]


_base = _mkm = None
REF_BUDGET = 200000


class _Budget(Exception):
    pass


def _init():
    global _base, _mkm
    from oracle import mk_oracle as O
    _base = O.load_spec(os.path.join(INPUTS, 'input.json'))
    _mkm = O.load_spec(os.path.join(INPUTS, 'input_mkm.json'), base_spec=_base)


def case_spec(case, pathways):
    spec = copy.copy(_mkm)
    keep = kept_reactions(list(_mkm['reactions']), case, pathways)
    spec['reactions'] = {r: _mkm['reactions'][r] for r in keep}
    return spec


def reference_system(spec, base):
    """old_system.System built from the reference's own classes over duck
    states (make_golden.build_reference_system, plus the derived reactions'
    base reactions, built from the base system's duck states)."""
    import make_golden as MG
    RR, RS, RX = MG.RR, MG.RS, MG.RX
    bstates = {n: MG.DuckState(base, n) for n in base['states']}
    states = {n: MG.DuckState(spec, n) for n in spec['states']}
    sysd = spec['system']
    s = RS.System()
    s.set_parameters(times=list(sysd['times']), start_state=dict(sysd.get('start_state') or {}),
                     inflow_state=dict(sysd.get('inflow_state') or {}), T=sysd['T'], p=sysd['p'],
                     use_jacobian=sysd.get('use_jacobian', True), ode_solver='solve_ivp',
                     nsteps=sysd.get('nsteps', 1e4), rtol=sysd.get('rtol', 1e-8), atol=sysd.get('atol', 1e-10),
                     xtol=sysd.get('xtol', 1e-8), ftol=sysd.get('ftol', 1e-8))
    for st in states.values():
        s.add_state(st)
    base_rx = {}
    for name, r in spec['reactions'].items():
        kw = dict(reac_type=r['reac_type'], reversible=r['reversible'],
                  reactants=[states[x] for x in r['reactants']], products=[states[x] for x in r['products']],
                  TS=None if r['TS'] is None else [states[x] for x in r['TS']], area=r['area'],
                  name=name, scaling=r['scaling'])
        if r['kind'] == 'user':
            cls = RR.UserDefinedReaction
            kw.update({k: v for k, v in r['user'].items()})
        elif r['kind'] == 'derived':
            b = base['reactions'][r['base']]
            if r['base'] not in base_rx:
                base_rx[r['base']] = RR.Reaction(
                    reac_type=b['reac_type'], reversible=b['reversible'],
                    reactants=[bstates[x] for x in b['reactants']], products=[bstates[x] for x in b['products']],
                    TS=None if b['TS'] is None else [bstates[x] for x in b['TS']], area=b['area'],
                    name=r['base'], scaling=b['scaling'])
            cls = RR.ReactionDerivedReaction
            kw['base_reaction'] = base_rx[r['base']]
        else:
            cls = RR.Reaction
        s.add_reaction(MG.classic_reaction(cls)(**kw))
    s.add_reactor(RX.InfiniteDilutionReactor())
    s.names_to_indices()
    return s


def _job(arg):
    from oracle import mk_oracle as O
    ci, ti = arg
    case, pathways = CASES[ci]
    T = float(TEMPS[ti])
    t0 = time.time()
    spec = case_spec(case, pathways)
    m = O.ClassicModel(spec, T=T)
    dyn = [m.snames[i] for i in m.dyn]
    out = O.steady_rule(m, budget=400000)
    t1 = time.time()
    res = dict(ci=ci, ti=ti, dyn=dyn)
    if out is None:
        res.update(ok=False)
    else:
        res.update(ok=True, y_rule=out['y'][m.dyn], y_tight=out['y_tight'][m.dyn], regular=out['regular'],
                   crit=out['crit'], bd_rule=m.tof(out['y'], BD_TERMS), bd_tight=m.tof(out['y_tight'], BD_TERMS))
    # the reference's own code (old_system.py solve_odes / find_steady)
    s = reference_system(spec, _base)
    s.params['temperature'] = T
    # scipy's BDF at the input tolerances can creep at tiny steps for good
    # (p123 at 923 K: no end after 10 min); a budget of species_odes calls
    # marks such a run as not finished (ref_ok False) instead of hanging
    odes = s.species_odes

    def counted(*a, **kw):
        counted.left -= 1
        if counted.left < 0:
            raise _Budget()
        return odes(*a, **kw)
    counted.left = REF_BUDGET
    s.species_odes = counted
    pos = [s.snames.index(d) for d in dyn]
    try:
        s.solve_odes()
        ok = True
    except _Budget:
        ok = False
    s.species_odes = odes
    if ok:
        y_ref = np.array(s.solution[-1], float)
        s.reaction_terms(y_ref)
        names = list(s.species_map.keys())
        bd_ref = float(sum(s.rates[names.index(r), 0] - s.rates[names.index(r), 1] for r in BD_TERMS if r in names))
        y_ls = np.array(s.find_steady(store_steady=True), float)
        res.update(y_ref=y_ref[pos], y_ls=y_ls[pos], bd_ref=bd_ref, ref_nt=int(len(s.times)), ref_ok=True)
    else:
        res.update(ref_ok=False)
    print('  %s T=%.0f oracle %.1f s, reference %.1f s' % (case, T, t1 - t0, time.time() - t1), flush=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workers', type=int, default=8)
    args = ap.parse_args()
    jobs = [(ci, ti) for ci in range(len(CASES)) for ti in range(len(TEMPS))]
    t0 = time.time()
    rows = {}
    with mp.get_context('fork').Pool(args.workers, initializer=_init) as pool:
        for k, res in enumerate(pool.imap_unordered(_job, jobs)):
            rows[(res['ci'], res['ti'])] = res
            if k % 16 == 0:
                print('%d / %d, %.0f s' % (k, len(jobs), time.time() - t0), flush=True)
    out = dict(temperatures=TEMPS, cases=np.array([c for c, _ in CASES]), bd_terms=np.array(BD_TERMS))
    for ci, (case, _) in enumerate(CASES):
        rs = [rows[(ci, ti)] for ti in range(len(TEMPS))]
        ns = len(rs[0]['dyn'])
        out['dyn_' + case] = np.array(rs[0]['dyn'])
        for key in ('y_rule', 'y_tight', 'y_ref', 'y_ls'):
            out[key + '_' + case] = np.array([r[key] if r.get(key) is not None else np.full(ns, np.nan)
                                              for r in rs])
        for key in ('regular', 'ok', 'ref_ok'):
            out[key + '_' + case] = np.array([bool(r.get(key, False)) for r in rs])
        for key in ('crit', 'bd_rule', 'bd_tight', 'bd_ref'):
            out[key + '_' + case] = np.array([float(r.get(key, np.nan)) for r in rs])
        print('%-22s %2d species: oracle ok %d / 17, regular %d / 17, reference finished %d / 17' % (
            case, ns, out['ok_' + case].sum(), out['regular_' + case].sum(), out['ref_ok_' + case].sum()))
    np.savez_compressed(OUT, **out)
    print('wrote %s (%.0f s)' % (OUT, time.time() - t0))


if __name__ == '__main__':
    main()
