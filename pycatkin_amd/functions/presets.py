"""Sweep drivers of pycatkin/functions/presets.py, batched onto the device.

The reference loops over temperatures / parameter values in Python and runs
one scipy solve per point (presets.py:31-168, 170-305); here the whole sweep
is one launch of the batched solver (and one of the DRC kernel).
Outputs (CSV names and columns) follow the reference.
"""
from __future__ import annotations

import os
import warnings

import numpy as np

from ..constants.physical_constants import bartoPa


def _no_plots(what, *flags):
    """Plotting is out of scope: every driver warns and skips it,
    so a reference script that asks for figures still gets its numbers."""
    if any(flags):
        warnings.warn('%s: plotting is not part of pycatkin_amd; the figures are skipped '
                      '(use save_results for the CSVs)' % what, stacklevel=3)


def run(sim_system, steady_state_solve=False, plot_results=False, save_results=False, fig_path=None, csv_path=''):
    """presets.py:16-28 (plotting is out of scope: plot_results warns and is skipped)."""
    _no_plots('run', plot_results)
    sim_system.solve_odes()
    if save_results:
        sim_system.write_results(path=csv_path)
    if steady_state_solve:
        sim_system._find_steady_classic(store_steady=True)


def _net_rates(sim_system, plan, finals, T, p=None):
    """rates[n, n_reactions] = r_fwd - r_rev at each final state (old_system.py:202-225)."""
    kf, kr = sim_system.rate_constants_batch(T=T, p=p)
    pos = {s: i for i, s in enumerate(plan.species)}
    gas_fac = bartoPa if plan.formulation == 'classic' else sim_system.params['pressure']
    out = np.zeros((finals.shape[0], len(plan.all_reactions)))
    for j, name in enumerate(plan.all_reactions):
        if name not in plan.reactions:
            continue
        a = plan.reactions.index(name)
        rx = sim_system.reactions[name]
        rf, rr = kf[a].copy(), kr[a].copy()
        for s in rx.reactants:
            if s.name in pos:
                rf *= finals[:, pos[s.name]] * (gas_fac if s.state_type == 'gas' else 1.0)
        for s in rx.products:
            if s.name in pos:
                rr *= finals[:, pos[s.name]] * (gas_fac if s.state_type == 'gas' else 1.0)
        out[:, j] = rf - rr
    return out


def _failed(status):
    """Indices of failed solves.  Status 4 (the transient end at t_end is not
    at a steady state: that transient is reported) and 5 (the same, its tight
    re-integration failed: the first pass's transient) are results, as the
    reference's find_steady returns wherever least_squares stops
    (System._check with degenerate_ok), and so is 6 (a DRC whose 2R+1
    solves mix reached roots and transient ends: its xi are written, and
    System.degree_of_rate_control warns); 1-3 are integrator failures."""
    st = np.asarray(status)
    return np.nonzero((st != 0) & (st != 4) & (st != 5) & (st != 6))[0]


def _finals(sim_system, plan, ydyn, n):
    base = sim_system._full(plan, plan.y0_default)
    final = np.tile(base, (n, 1))
    pos = {s: i for i, s in enumerate(plan.species)}
    for i, s in enumerate(plan.dyn):
        final[:, pos[s]] = ydyn[i]
    return final


def run_temperatures(sim_system, temperatures, steady_state_solve=False, tof_terms=None, eps=5.0e-2,
                     plot_results=False, save_results=False, plot_transient=False, save_transient=False,
                     fig_path=None, csv_path=''):
    """presets.py:31-167 as one batch over `temperatures`.  Returns
    (final [nT, n_states], rates [nT, n_reactions], drcs {T: {reaction: xi}})."""
    _no_plots('run_temperatures', plot_results, plot_transient)
    temps = np.asarray(temperatures, float).ravel()
    plan = sim_system.plan()
    r = sim_system.solve_batch(T=temps, steady=steady_state_solve)
    bad = _failed(r['status'])
    if bad.size:
        raise RuntimeError('device solver failed for T = %s (status %s)' % (temps[bad], r['status'][bad]))
    final = _finals(sim_system, plan, r['y'], temps.size)
    rates = _net_rates(sim_system, plan, final, temps)
    drcs = {}
    if tof_terms is not None:
        d = sim_system.drc_batch(tof_terms, T=temps, eps=eps, steady=False)
        for k, T in enumerate(temps):
            drcs[T] = {name: float(d[name][k]) for name in sim_system.reactions}
    sim_system.params['temperature'] = temps[-1]
    if save_results:
        _save(sim_system, plan, 'Temperature (K)', 'temperature', temps, final, rates, drcs, tof_terms, csv_path)
    return final, rates, drcs


def run_parameters(sim_system, parameters, params_name, steady_state_solve=False, tof_terms=None, eps=5.0e-2,
                   plot_results=False, save_results=False, plot_transient=False, save_transient=False,
                   fig_path=None, csv_path=''):
    """presets.py:170-305.  'temperature', 'pressure', 'start_state_<gas>' and
    'inflow_state_<gas>' vary per condition inside one batch; any other
    `params` key (presets.py:187-188: rtol, atol, times, ...) is set value by
    value, one launch each.  As in the reference, sim_system.params keeps the
    last value afterwards."""
    vals = np.asarray(parameters, float).ravel()
    _no_plots('run_parameters', plot_results, plot_transient)
    batched = (params_name in ('temperature', 'pressure') or params_name.startswith('start_state_')
               or params_name.startswith('inflow_state_'))
    if batched:
        final, rates, drcs = _run_batch(sim_system, params_name, vals, steady_state_solve, tof_terms, eps)
    else:
        parts = [_run_batch(sim_system, params_name, vals[k:k + 1], steady_state_solve, tof_terms, eps,
                            set_param=True) for k in range(vals.size)]
        final = np.concatenate([q[0] for q in parts], axis=0)
        rates = np.concatenate([q[1] for q in parts], axis=0)
        drcs = {}
        for q in parts:
            drcs.update(q[2])
    _keep_last(sim_system, params_name, vals[-1])
    if save_results:
        _save(sim_system, sim_system.plan(), params_name, params_name, vals, final, rates, drcs, tof_terms, csv_path)
    return final, rates, drcs


def _keep_last(sim_system, params_name, v):
    """the reference's loop leaves its last value in sim_system.params (presets.py:181-188)"""
    if params_name.startswith('start_state_'):
        sim_system.params['start_state'][params_name.split('start_state_')[1]] = v
    elif params_name.startswith('inflow_state_'):
        sim_system.params['inflow_state'][params_name.split('inflow_state_')[1]] = v
    else:
        sim_system.params[params_name] = v
    sim_system._plans.clear()


def _run_batch(sim_system, params_name, vals, steady_state_solve, tof_terms, eps, set_param=False):
    if set_param:
        sim_system.params[params_name] = float(vals[0])
        sim_system._plans.clear()
    plan = sim_system.plan()
    kw = {}
    if params_name == 'temperature':
        kw['T'] = vals
    elif params_name == 'pressure':
        kw['p'] = vals
    elif params_name.startswith('start_state_'):
        s = params_name.split('start_state_')[1]
        if s in plan.fix:
            fix = np.tile(plan.fix_default[:, None], (1, vals.size))
            fix[plan.fix.index(s)] = vals
            kw['fix'] = fix
        else:
            y0 = np.tile(plan.y0_default[:, None], (1, vals.size))
            y0[plan.dyn.index(s)] = vals
            kw['y0'] = y0
    elif params_name.startswith('inflow_state_'):
        s = params_name.split('inflow_state_')[1]
        inflow = np.tile(plan.inflow_default[:, None], (1, vals.size))
        inflow[plan.dyn.index(s)] = vals
        kw['inflow'] = inflow
    n = vals.size
    if 'T' not in kw:
        kw['T'] = np.full(n, float(sim_system.params['temperature']))
    r = sim_system.solve_batch(steady=steady_state_solve, **kw)
    bad = _failed(r['status'])
    if bad.size:
        raise RuntimeError('device solver failed for %s = %s' % (params_name, vals[bad]))
    final = _finals(sim_system, plan, r['y'], n)
    rates = _net_rates(sim_system, plan, final, kw['T'], kw.get('p'))
    drcs = {}
    if tof_terms is not None:
        d = sim_system.drc_batch(tof_terms, eps=eps, **kw)
        for k, v in enumerate(vals):
            drcs[v] = {name: float(d[name][k]) for name in sim_system.reactions}
    return final, rates, drcs


def _save(sim_system, plan, label, stem, xs, final, rates, drcs, tof_terms, csv_path):
    import pandas as pd
    if csv_path and not os.path.isdir(csv_path):
        os.makedirs(csv_path, exist_ok=True)
    suffix = 'temperature' if stem == 'temperature' else stem
    names = list(plan.species)
    st = sim_system.states
    ads = [i for i, s in enumerate(names) if st[s].state_type in ('adsorbate', 'surface') and s in plan.dyn + plan.fix]
    gas = [i for i, s in enumerate(names) if st[s].state_type == 'gas' and s in plan.dyn + plan.fix]
    col = np.reshape(xs, (-1, 1))
    pd.DataFrame(np.concatenate((col, rates), axis=1), columns=[label] + list(plan.all_reactions)).to_csv(
        csv_path + 'rates_vs_%s.csv' % suffix, index=False)
    pd.DataFrame(np.concatenate((col, final[:, ads]), axis=1), columns=[label] + [names[i] for i in ads]).to_csv(
        csv_path + 'coverages_vs_%s.csv' % suffix, index=False)
    pd.DataFrame(np.concatenate((col, final[:, gas]), axis=1),
                 columns=[label] + ['p' + names[i] + ' (bar)' for i in gas]).to_csv(
        csv_path + 'pressures_vs_%s.csv' % suffix, index=False)
    if tof_terms is not None:
        vals = np.array([[x] + [drcs[x][r] for r in sim_system.reactions] for x in xs])
        pd.DataFrame(vals, columns=[label] + list(sim_system.reactions)).to_csv(
            csv_path + 'drcs_vs_%s.csv' % suffix, index=False)


# ----------------------------------------------------------------------------
# energy tables (presets.py:378-472), every number from one pck_energies launch
# ----------------------------------------------------------------------------
def _mkdir(csv_path):
    if csv_path and not os.path.isdir(csv_path):
        os.makedirs(csv_path, exist_ok=True)


def _reaction_energy_rows(sim_system, T, p):
    """[dEr, dGr, dEa, dGa] (J/mol) of every reaction at (T, p): the reference's
    get_reaction_energy('electronic' / 'free') and get_reaction_barriers(...)[0]
    (reaction.py:171-200), evaluated for all reactions in one device launch."""
    from ..engine import evaluate_forms
    keys = ('dErxn', 'dGrxn', 'dEa_fwd', 'dGa_fwd')
    forms, slots = [], []
    for r in sim_system.reactions.values():
        e = r.energy_forms()
        for k in keys:
            slots.append(None if e[k] is None else len(forms))
            if e[k] is not None:
                forms.append(e[k])
    states = list(sim_system.states.values())
    vals = evaluate_forms(forms, T, p, states=states) if forms else []
    out = []
    for i, _ in enumerate(sim_system.reactions):
        row = []
        for k in range(len(keys)):
            s = slots[i * len(keys) + k]
            row.append(None if s is None else vals[s] * 1.0e3 * 96.485)
        out.append(row)
    return out


def save_energies(sim_system, csv_path=''):
    """presets.py:378-406: reaction_energies_and_barriers_<T>K_<p>bar.csv with
    columns Reaction, dEr, dGr, dEa, dGa (J/mol) at params' T and p."""
    import pandas as pd
    _mkdir(csv_path)
    T, p = sim_system.params['temperature'], sim_system.params['pressure']
    rows = _reaction_energy_rows(sim_system, T, p)
    df = pd.DataFrame(data=[[r] + v for r, v in zip(sim_system.reactions, rows)],
                      columns=['Reaction', 'dEr (J/mol)', 'dGr (J/mol)', 'dEa (J/mol)', 'dGa (J/mol)'])
    df.to_csv(csv_path + 'reaction_energies_and_barriers_%1.1fK_%1.1fbar.csv' % (T, p / bartoPa), index=False)


def save_energies_temperatures(sim_system, temperatures, csv_path=''):
    """presets.py:409-438: reaction_energies_and_barriers_<reaction>.csv, one row
    per temperature.  As in the reference, params['temperature'] is left at the
    last temperature."""
    import pandas as pd
    _mkdir(csv_path)
    p = sim_system.params['pressure']
    temps = [float(T) for T in np.ravel(temperatures)]
    per_T = [_reaction_energy_rows(sim_system, T, p) for T in temps]
    for i, r in enumerate(sim_system.reactions):
        df = pd.DataFrame(data=[[T] + per_T[k][i] for k, T in enumerate(temps)],
                          columns=['Temperature (K)', 'dEr (J/mol)', 'dGr (J/mol)', 'dEa (J/mol)', 'dGa (J/mol)'])
        df.to_csv(csv_path + 'reaction_energies_and_barriers_%s.csv' % r, index=False)
    if temps:
        sim_system.params['temperature'] = temps[-1]


def state_energy_table(sim_system, T=None, p=None):
    """{state: [Gfree, Gelec, Gvibr, Grota, Gtran]} (eV) -- the values
    State.calc_free_energy leaves on each state (state.py:367-386), in the row
    order save_state_energies writes them.  A state whose free energy is given
    in the input keeps its given components (None where absent)."""
    from ..engine import evaluate_forms
    T = sim_system.params['temperature'] if T is None else T
    p = sim_system.params['pressure'] if p is None else p
    names = sorted(sim_system.states)
    forms, slots = [], {}
    for s in names:
        st = sim_system.states[s]
        if st.Gfree is not None:
            slots[s] = [len(forms)] + [None] * 4
            forms.append(st.free_form())
            continue
        slots[s] = list(range(len(forms), len(forms) + 5))
        forms += [st.free_form(), st.elec_form(), st.vib_form(), st.rot_form(), st.tran_form()]
    vals = evaluate_forms(forms, T, p, states=[sim_system.states[s] for s in names]) if forms else []
    out = {}
    for s in names:
        st = sim_system.states[s]
        given = [None, st.Gelec, st.Gvibr, st.Grota, st.Gtran]
        out[s] = [vals[k] if k is not None else (None if g is None else float(g))
                  for k, g in zip(slots[s], given)]
    return out


def save_state_energies(sim_system, csv_path=''):
    """presets.py:441-471: state_energies_<T>K_<p>bar.csv.  The reference writes
    [Gfree, Gelec, Gvibr, Grota, Gtran] under the header Free, Electronic,
    Vibrational, Translational, Rotational -- Grota sits in the
    'Translational (eV)' column and Gtran in 'Rotational (eV)' -- and its
    goldens (test/test_1.py:78-81) are read from those columns, so the same
    placement is kept."""
    import pandas as pd
    _mkdir(csv_path)
    T, p = sim_system.params['temperature'], sim_system.params['pressure']
    tab = state_energy_table(sim_system, T, p)
    df = pd.DataFrame(data=[[s] + tab[s] for s in sorted(sim_system.states)],
                      columns=['State', 'Free (eV)', 'Electronic (eV)', 'Vibrational (eV)', 'Translational (eV)',
                               'Rotational (eV)'])
    df.to_csv(csv_path + 'state_energies_%1.1fK_%1.1fbar.csv' % (T, p / bartoPa), index=False)


def get_tof_for_given_reactions(sim_system, tof_terms):
    """presets.py:585-597: sum of (r_fwd - r_rev) over tof_terms at the last
    transient state (sim_system.solution[-1]); the system's stored rates are
    left as they were (the reference works on a deep copy)."""
    if sim_system.solution is None:
        raise RuntimeError('get_tof_for_given_reactions: run solve_odes() first')
    keep = sim_system.rates
    try:
        rates = sim_system.reaction_terms(sim_system.solution[-1])
    finally:
        sim_system.rates = keep
    names = list(sim_system.plan().all_reactions)
    return float(sum(rates[names.index(r), 0] - rates[names.index(r), 1] for r in tof_terms if r in names))
