"""Descriptor-grid post-processing of the patched System
(pycatkin/functions/analysis.py), and the C x O grid it post-processes as
one batched launch.

The reference's workflow (test/CH4_input.json, the patched system.py /
solver.py classes) loops over an E_C x E_O grid in Python: per point it sets
the descriptor reactions' energies (reactions C_ads / O_ads dErxn_user,
states sC / sO Gelec; analysis.py:54-58), builds the System and runs
SteadyStateSolver.solve_ode (solver.py:374-418), collecting
{(iC, iO): SteadyStateResults} -- the `log` that check_convergence and
average_neighborhood take.  `solve_descriptor_grid` makes the same
assignments ONCE as Descriptor forms ('EC', 'EO') and solves the whole grid
as a batch of conditions (one RODAS4P launch, then the convergence checks of
every point in two launches).

check_convergence / average_neighborhood / the convergence map keep the
reference's semantics to the letter, including two quirks a drop-in user may
depend on (both documented at the function):
  - check_convergence's diagnostic composition is
    initial_system[len(gas):] ++ x (analysis.py:64), not the gas part ++ x;
  - average_neighborhood returns after the first averaged point, and None
    when no point was averaged (analysis.py:116 sits inside the loop);
    `all_points=True` averages every misfit.
Plotting (seaborn / matplotlib, absent here) is out of scope: the heatmap
functions return the arrays the reference would draw.
"""
from __future__ import annotations

import copy
import warnings

import numpy as np

from ..classes.system import SteadyStateResults
from ..energy import Descriptor

# (descriptor reaction, its state, descriptor name): analysis.py:54-58
DESCRIPTOR_TERMS = (('C_ads', 'sC', 'EC'), ('O_ads', 'sO', 'EO'))


def set_descriptor_energies(sim_system, terms=DESCRIPTOR_TERMS):
    """analysis.py:54-58's per-point assignments as descriptor forms: the
    scaling states' energies (state.py:490-517) follow them as linear forms."""
    for rxn, state, name in terms:
        sim_system.reactions[rxn].dErxn_user = Descriptor(name)
        sim_system.states[state].Gelec = Descriptor(name)
    sim_system._plans.clear()
    return tuple(name for _, _, name in terms)


def descriptor_grid(C_range, O_range):
    """Flattened (E_C, E_O) pairs in [iC, iO] row-major order."""
    EC, EO = np.meshgrid(np.asarray(C_range, float), np.asarray(O_range, float), indexing='ij')
    return EC.ravel(), EO.ravel()


def solve_descriptor_grid(sim_system, C_range, O_range, T=None, tmax=1e4, test_convergence_kwargs=None,
                          max_steps=200000):
    """{(iC, iO): SteadyStateResults(x, success)} for every grid point: what
    the reference's per-point loop of SteadyStateSolver(system).solve_ode()
    returns (solver.py:374-418: the surface transient from the normalised
    initial state to tmax at rtol 1e-10 / atol 1e-12, then test_convergence),
    as one launch over the len(C_range) x len(O_range) conditions.
    `sim_system` is not modified (a deep copy carries the descriptor forms).
    x is the surface part in index_map order, as solve_ode returns it."""
    from ..classes.solver import SteadyStateSolver
    s = copy.deepcopy(sim_system)
    names = set_descriptor_energies(s)
    s.build()
    EC, EO = descriptor_grid(C_range, O_range)
    n = EC.size
    desc = dict(zip(names, (EC, EO)))
    T = np.full(n, float(s.T if T is None else T))
    plan = s.plan()
    y0 = s._to_plan(plan, s.initial_system[len(s.gas_indices):][:, None])
    r = s.solve_batch(T=T, desc=desc, y0=np.repeat(y0, n, axis=1), t0=0.0, t_end=tmax, rtol=1e-10, atol=1e-12,
                      steady=False, max_steps=max_steps)
    Y = r['y'][s._from_plan(plan)]
    kw = dict(test_convergence_kwargs or {})
    kw.pop('log', None)
    solver = SteadyStateSolver(s, ss_guess=Y[:, 0])
    ok = (r['status'] == 0) & solver.test_convergence_batch(Y, desc=desc, T=T, **kw)
    nO = np.size(O_range)
    return {(c // nO, c % nO): SteadyStateResults(Y[:, c], bool(ok[c])) for c in range(n)}


def check_convergence(log, sim_system, C_range, O_range):
    """analysis.py:27-76: (misfit_list, worked_list) of the log's keys by
    success, in the log's order.  For every failed point the reference
    rebuilds the system at its descriptors and prints a diagnosis of the
    composition initial_system[len(gas_indices):] ++ x (analysis.py:64, as
    written: the surface part of the initial state, not the gas part, goes in
    front of x): 'SURF SUM FAILED' when a coverage_map group of it does not sum
    to 1 within 0.05, else 'RATE FAILED' when a get_dydt component exceeds
    1e-6 in magnitude.  Here the get_dydt of every failed point comes from one
    launch with per-point descriptor energies."""
    misfit_list, worked_list = [], []
    for k, v in log.items():
        (worked_list if v.success else misfit_list).append(k)
    if not misfit_list:
        return misfit_list, worked_list
    s = copy.deepcopy(sim_system)
    names = set_descriptor_energies(s)
    s.build()
    head = s.initial_system[len(s.gas_indices):]
    Y = np.stack([np.concatenate((head, np.asarray(log[k].x, float))) for k in misfit_list], axis=1)
    desc = dict(zip(names, (np.array([C_range[k[0]] for k in misfit_list], float),
                            np.array([O_range[k[1]] for k in misfit_list], float))))
    # the reference's builtin sum over y[list(indices)] (left to right)
    surf = np.array([[sum(Y[list(idx), c]) for c in range(Y.shape[1])] for idx in s.coverage_map.values()])
    dydt = s.get_dydt_batch(Y, desc)
    for c, k in enumerate(misfit_list):
        if np.any(np.abs(surf[:, c] - 1) > 0.05):
            print(f"{k} : SURF SUM FAILED: {' , '.join(str(x)[:8] for x in surf[:, c])}")
        elif np.any(np.abs(dydt[:, c]) > 1e-6):
            print(f"{k} : RATE FAILED: {max(dydt[:, c]):.4e}")
    return misfit_list, worked_list


def average_neighborhood(misfit_list, worked_list, log, all_points=False):
    """analysis.py:79-116: a failed point's coverage becomes the mean x of
    its successful 8-neighbours (at least 2 of them; fewer: a message and the
    point is skipped), stored as SteadyStateResults(mean, success=False) in a
    deep copy of the log.  As the reference is written, the function returns
    after the FIRST averaged point and returns None when it averages none
    (its `return` sits inside the loop); all_points=True averages every
    misfit and always returns the new log."""
    new_log = copy.deepcopy(log)
    worked = set(worked_list)
    for iC, iO in misfit_list:
        neighborhood = [(iC + k, iO + j) for k in (-1, 0, 1) for j in (-1, 0, 1)
                        if (k, j) != (0, 0) and (iC + k, iO + j) in worked]
        if len(neighborhood) < 2:
            print(f"FAILED FINDING SURROUNDINGS FOR {iC, iO}")
            continue
        L = [new_log[pair].x for pair in neighborhood]
        new_log[(iC, iO)] = SteadyStateResults(x=np.mean(L, axis=0), success=False)
        if not all_points:
            return new_log
    return new_log if all_points else None


def convergence_map(C_range, O_range, misfit_list):
    """analysis.py:131-136: ones, 0 at the failed points ([iC, iO])."""
    work_map = np.ones((len(C_range), len(O_range)))
    for iC, iO in misfit_list:
        if 0 <= iC < len(C_range) and 0 <= iO < len(O_range):
            work_map[iC, iO] = 0
    return work_map


def convergence_heatmap(C_range, O_range, misfit_list):
    """analysis.py:120-140 draws convergence_map(...).T with seaborn; plotting
    is out of scope here: warns and returns the map."""
    warnings.warn('convergence_heatmap: plotting is not supported (no seaborn / matplotlib); '
                  'returning the map', stacklevel=2)
    return convergence_map(C_range, O_range, misfit_list)


def heatmap_scores(labels, results, C_range, O_range, use_log=True):
    """analysis.py:206-233, the data make_heatmap draws: scores[label, iC, iO]
    = log|v[label]| (or |v[label]|) over the results dict, log values clipped
    below at -25; and the colour range (vmin, vmax) rounded to 2 decimals."""
    labels = [labels] if isinstance(labels, str) else list(labels)
    scores = np.zeros((len(labels), len(C_range), len(O_range)))
    for idx, case in enumerate(labels):
        for k, v in results.items():
            scores[(idx, *k)] = np.log(np.abs(v[case])) if use_log else np.abs(v[case])
    if use_log:
        scores[np.where(scores < -25)] = -25
    return scores, (float(np.round(np.min(scores), 2)), float(np.round(np.max(scores), 2)))


def make_heatmap(labels, results, C_range, O_range, use_log=True, **kwargs):
    """analysis.py:175-266 without the figure: warns and returns
    heatmap_scores(...)."""
    warnings.warn('make_heatmap: plotting is not supported (no matplotlib); returning the scores', stacklevel=2)
    return heatmap_scores(labels, results, C_range, O_range, use_log)
