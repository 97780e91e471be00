"""Drop-in parity of the reference's drivers on the device, against committed
oracle fixtures (tests/golden/make_*_fixture.py) and the reference's goldens:

  * the headline volcano grid (BASELINE configs[2]) at 2 560 fixture nodes,
    regular roots and degenerate (status 4) points alike;
  * the DMTM degree of rate control over temperatures and pressures
    (BASELINE configs[3], run_parameters(..., 'pressure', tof_terms=...));
  * reference test/test_1.py steps 4, 5 and 7 through run / run_temperatures /
    save_state_energies / save_energies (the energy-span step 6 is out of
    scope).
"""
import copy
import json
import os

import numpy as np
import pytest

from oracle import mk_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, 'golden')


@pytest.fixture(scope='module')
def P():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    import pycatkin_amd
    return pycatkin_amd


def _record(name, obj):
    """Diagnostics of a GPU run (gpurun_out/ on the box; nothing if absent)."""
    if os.path.isdir('gpurun_out'):
        json.dump(obj, open(os.path.join('gpurun_out', name), 'w'), indent=1, default=float)


# ----------------------------------------------------------------------------
# headline volcano grid vs the dense oracle fixture
# ----------------------------------------------------------------------------
# north_star: steady-state coverages and log10(TOF) within 1e-6 relative.
RTOL = 1e-6


def test_volcano_fixture_parity(P, inputs):
    """Every node of tests/golden/volcano_fixture.npz solved as the bench
    solves it (System.solve_batch(steady=True): the transient to t_end =
    3600 s at STEADY_TRANSIENT, Newton from its end, the root reported where
    the transient has reached it to ROOT_DIST, else the transient end), against
    the oracle's restatement of the same rule from its tight transient (lsoda,
    rtol 1e-11 / atol 1e-20; make_volcano_fixture.py):

    * every node, whatever either side's classification: log10(TOF) within
      1e-6 relative of the oracle's answer (the rule makes the answer
      classification-independent: where the two sides classify a node
      differently, both answers lie within ~ROOT_DIST of the transient end);
    * nodes both sides call regular (status 0): coverages within 1e-6
      relative of the oracle's root (floor 1e-15); nodes both call
      "not reached" (status 4): within 1e-6 of the tight transient (floor
      1e-20, its atol);
    * the classification differs on at most 1 % of the nodes (0.2 % of the
      uniform ones), and only where the oracle's criterion lies within a
      factor 2 of ROOT_DIST -- the integrators' own error (~1e-7) moving it
      across the threshold.  There the coverages agree to 2 * ROOT_DIST.
    The reference's own numbers are reported next to these (not asserted
    here): its lsoda transient at 1e-8 / 1e-10 and least_squares' answer."""
    from pycatkin_amd.classes.system import ROOT_DIST, STEADY_TRANSIENT
    from pycatkin_amd.functions.volcano import set_volcano_energies
    fx = dict(np.load(os.path.join(GOLDEN, 'volcano_fixture.npz')))
    assert tuple(fx['root_dist']) == (ROOT_DIST, STEADY_TRANSIENT[1])
    lo, hi, G = fx['grid']
    be = np.linspace(lo, hi, int(G))
    eco, eo = be[fx['i']], be[fx['j']]
    n = eco.size
    s = P.read_from_input_file(os.path.join(inputs, 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    r = s.solve_batch(T=np.full(n, 600.0), desc={'ECO': eco, 'EO': eo}, tof_terms=('CO_ox',), steady=True)
    plan = s.plan(('CO_ox',))
    names = [str(x) for x in fx['dyn']]
    y = r['y'][[plan.dyn.index(nm) for nm in names]].T          # [n, species] in the fixture's order
    st = r['status']
    assert np.all((st == 0) | (st == 4)), np.unique(st, return_counts=True)
    l10 = np.log10(r['tof'])
    dev_reg = st == 0
    reg = fx['regular']
    ok = fx['tight_ok']                       # nodes with an oracle answer (12 of 2 560 exceed its budget)

    def rel(a, b):
        return np.abs(a - b) / np.maximum(np.abs(b), 1e-300)

    err = rel(l10, fx['l10_root'])            # l10_root: the oracle's answer (root, or the tight transient)
    both_reg, both_deg = dev_reg & reg & ok, ~dev_reg & ~reg & ok
    cov_reg = np.abs(y - fx['y_root']) <= RTOL * np.abs(fx['y_root']) + 1e-15
    cov_deg = np.abs(y - fx['y_root']) <= RTOL * np.abs(fx['y_root']) + 1e-20
    flips = np.nonzero((dev_reg != reg) & ok)[0]
    uni = np.arange(n) < 2048                 # the uniform part of the fixture
    info = dict(n=int(n), n_compared=int(ok.sum()), n_regular=int(dev_reg.sum()), n_not_reached=int((~dev_reg).sum()),
                oracle_regular=int(reg.sum()), n_flips=int(flips.size),
                flip_rate_uniform_nodes=float(np.mean((dev_reg != reg)[uni & ok])),
                flips=[dict(E_CO=float(eco[k]), E_O=float(eo[k]), device_status=int(st[k]), l10=float(l10[k]),
                            l10_oracle=float(fx['l10_root'][k]), l10_tight=float(fx['l10_tight'][k]),
                            oracle_crit=float(fx['crit'][k]), oracle_newton_ok=bool(fx['newton_ok'][k]),
                            max_rel_cov=float(np.max((np.abs(y[k] - fx['y_root'][k]) - 1e-20) /
                                                     np.abs(fx['y_root'][k]))))
                       for k in flips],
                max_rel_l10_all=float(err[ok].max()),
                max_rel_l10_regular=float(err[both_reg].max()) if both_reg.any() else 0.0,
                max_rel_l10_not_reached=float(err[both_deg].max()) if both_deg.any() else 0.0,
                reference_lsoda_vs_tight_max_abs_l10=float(np.nanmax(np.abs(fx['l10_ref'] - fx['l10_tight'])[ok])),
                reference_lsoda_vs_device_max_abs_l10=float(np.nanmax(np.abs(fx['l10_ref'] - l10)[ok])))
    ls_ok = np.isfinite(fx['l10_ls']) & ok
    info['least_squares_within_1e-6_of_device'] = float(np.mean(rel(fx['l10_ls'][ls_ok], l10[ls_ok]) <= RTOL))
    for key in ('l10_ref_reference', 'l10_ls_reference'):      # the reference's own code (make_volcano_reference.py)
        if key in fx:
            sel = np.isfinite(fx[key]) & ok
            info[key + '_n'] = int(sel.sum())
            info[key + '_within_1e-6_of_device'] = float(np.mean(rel(fx[key][sel], l10[sel]) <= RTOL))
            info[key + '_max_abs_l10_vs_device'] = float(np.max(np.abs(fx[key][sel] - l10[sel])))
    _record('volcano_fixture_parity.json', info)
    if 'l10_ls_reference' in fx:
        # the reference's own find_steady (least_squares from its lsoda
        # transient) where the transient has reached the steady state: the
        # device's root, at 1e-6 on all but a handful of nodes (measured
        # 451 / 452 in the oracle: least_squares stops at xtol on the rest)
        sel = ok & reg & dev_reg & np.isfinite(fx['l10_ls_reference'])
        agree = rel(fx['l10_ls_reference'][sel], l10[sel]) <= RTOL
        info['reference_find_steady_agrees_on_reached'] = [int(agree.sum()), int(sel.size and sel.sum())]
        _record('volcano_fixture_parity.json', info)
        assert agree.mean() >= 0.99, info['reference_find_steady_agrees_on_reached']
        # the reference's own volcano driver value (lsoda at the input's rtol
        # 1e-8 / atol 1e-10) is the device's answer up to that integrator's
        # error: measured <= 1.04e-3 in log10(TOF) against the tight transient
        sel = ok & fx['ref_ok_reference'] & np.isfinite(fx['l10_ref_reference'])
        assert np.max(np.abs(fx['l10_ref_reference'][sel] - l10[sel])) <= 2e-3, info
    assert np.all(err[ok] <= RTOL), (err[ok].max(), np.nonzero(ok)[0][np.argmax(err[ok])])
    assert np.all(cov_reg[both_reg]), np.nonzero(both_reg & ~np.all(cov_reg, axis=1))[0][:5]
    assert np.all(cov_deg[both_deg]), np.nonzero(both_deg & ~np.all(cov_deg, axis=1))[0][:5]
    assert flips.size <= 0.01 * n, info['flips'][:10]
    assert info['flip_rate_uniform_nodes'] <= 0.002, info['flip_rate_uniform_nodes']
    for f in info['flips']:
        assert 0.5 * ROOT_DIST <= f['oracle_crit'] <= 2.0 * ROOT_DIST, f
        assert f['max_rel_cov'] <= 2.0 * ROOT_DIST + RTOL, f


def test_newton_step_floor_node(P, inputs):
    """Fixture node 2502 (E_CO -0.606, E_O -2.040: sO 0.99996, sO2 3.6e-5)
    is a reached steady state (the oracle's criterion 1.9e-13), but Newton's
    second step from the transient end is rounding amplified ~1e6 by the
    Jacobian.  The step floor (mk_solver.h: PCK_STEP_FLOOR) returns the
    iterate before that step: status 0 and the oracle's root at 1e-9, where
    the iteration used to wander to its linear-convergence exit (status 4)."""
    from pycatkin_amd.functions.volcano import set_volcano_energies
    fx = dict(np.load(os.path.join(GOLDEN, 'volcano_fixture.npz')))
    lo, hi, G = fx['grid']
    be = np.linspace(lo, hi, int(G))
    k = 2502
    assert fx['regular'][k] and fx['crit'][k] < 1e-12
    s = P.read_from_input_file(os.path.join(inputs, 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    r = s.solve_batch(T=np.full(1, 600.0), desc={'ECO': be[fx['i'][k:k + 1]], 'EO': be[fx['j'][k:k + 1]]},
                      tof_terms=('CO_ox',), steady=True)
    assert r['status'][0] == 0, r['status']
    plan = s.plan(('CO_ox',))
    y = r['y'][[plan.dyn.index(str(n)) for n in fx['dyn']], 0]
    np.testing.assert_allclose(y, fx['y_root'][k], rtol=1e-9, atol=1e-20)


def test_degenerate_points_through_drop_in_api(P, inputs):
    """System.find_steady() / activity(ss_solve=True) on a degenerate root
    (status 4) return -- as the reference's least_squares path returns -- the
    transient end instead of raising; activity() (the volcano driver's call)
    gives the same number."""
    fx = np.load(os.path.join(GOLDEN, 'volcano_fixture.npz'))
    lo, hi, G = fx['grid']
    be = np.linspace(lo, hi, int(G))
    # the degenerate fixture node deepest in the O-poisoned corner (strong O, weak CO)
    cand = np.nonzero(~fx['regular'])[0]
    k = int(cand[np.argmax(be[fx['i'][cand]] - be[fx['j'][cand]])])
    ECO, EO = float(be[fx['i'][k]]), float(be[fx['j'][k]])
    sim_system = P.read_from_input_file(os.path.join(inputs, 'COOxVolcano', 'input.json'))
    # examples/COOxVolcano/cooxvolcano.py:28-44, verbatim in effect
    T = sim_system.params['temperature']
    SCOg, SO2g = 2.0487e-3, 2.1261e-3
    sim_system.reactions['CO_ads'].dErxn_user = ECO
    sim_system.reactions['CO_ads'].dGrxn_user = ECO + SCOg * T
    sim_system.reactions['2O_ads'].dErxn_user = 2.0 * EO
    sim_system.reactions['2O_ads'].dGrxn_user = 2.0 * EO + SO2g * T
    EO2 = sim_system.states['sO2'].get_potential_energy()
    sim_system.reactions['O2_ads'].dErxn_user = EO2
    sim_system.reactions['O2_ads'].dGrxn_user = EO2 + SO2g * T
    ETS_CO_ox = sim_system.states['SRTS_ox'].get_potential_energy()
    sim_system.reactions['CO_ox'].dEa_fwd_user = np.max((ETS_CO_ox - (ECO + EO), 0.0))
    ETS_O2_2O = sim_system.states['SRTS_O2'].get_potential_energy()
    sim_system.reactions['O2_2O'].dEa_fwd_user = np.max((ETS_O2_2O - EO2, 0.0))
    s = sim_system
    a_ss = s.activity(tof_terms=['CO_ox'], ss_solve=True)
    l10 = np.log10(s.run_and_return_tof(['CO_ox'], ss_solve=True))
    assert abs(l10 - fx['l10_tight'][k]) <= RTOL * abs(fx['l10_tight'][k]), (ECO, EO, l10, fx['l10_tight'][k])
    assert np.isfinite(a_ss)
    s.solve_odes()
    full = s.find_steady()
    assert np.all(np.isfinite(full))


# ----------------------------------------------------------------------------
# DMTM degree of rate control over T x p (BASELINE configs[3])
# ----------------------------------------------------------------------------
def test_dmtm_drc_pressure_sweep_vs_fixture(P, inputs):
    """run_parameters(dmtm, [1e4, 1e5, 1e6], 'pressure', tof_terms=['r5', 'r9'])
    at 450 / 600 / 750 K (presets.py:170-201): the transient DRC the
    reference's driver computes, at the input's tolerances (rtol 1e-6 / atol
    1e-8 to t = 1e12 s), and the steady DRC of every (T, p) in one drc_batch
    launch, against tests/golden/dmtm_drc_fixture.json.

    Bounds: steady DRC 1e-6 (absolute on xi, relative above 1): both sides
    polish each perturbed system to its root.  Transient DRC at the input
    tolerances: within 1e-4 of the oracle's tight transient DRC (rtol 1e-10):
    two integrators at rtol 1e-6 differ by their error, divided by
    2 eps = 0.1 in the central difference."""
    from pycatkin_amd.functions.presets import run_parameters
    fx = json.load(open(os.path.join(GOLDEN, 'dmtm_drc_fixture.json')))
    ps = np.array(fx['pressures'])
    worst = dict(steady=0.0, input_vs_tight=0.0, oracle_input_vs_tight=0.0)
    for T in fx['temperatures']:
        s = P.read_from_input_file(os.path.join(inputs, 'DMTM', 'input.json'))
        s.params['temperature'] = T
        final, rates, drcs = run_parameters(s, ps, 'pressure', tof_terms=fx['tof_terms'], eps=fx['eps'])
        s.params['temperature'] = T
        d = s.drc_batch(tuple(fx['tof_terms']), T=np.full(ps.size, T), p=ps, eps=fx['eps'], steady=True,
                        rtol=1e-10, atol=1e-14)
        assert np.all(d['status'] == 0), d['status']
        for k, p in enumerate(ps):
            c = [x for x in fx['conditions'] if x['T'] == T and x['p'] == p][0]
            for name, ref in c['drc_steady'].items():
                e = abs(d[name][k] - ref) / max(1.0, abs(ref))
                worst['steady'] = max(worst['steady'], e)
                assert e <= 1e-6, (T, p, name, d[name][k], ref)
            for name, ref in c['drc_tight'].items():
                e = abs(drcs[p][name] - ref)
                worst['input_vs_tight'] = max(worst['input_vs_tight'], e)
                worst['oracle_input_vs_tight'] = max(worst['oracle_input_vs_tight'], abs(c['drc_input'][name] - ref))
                assert e <= 1e-4, (T, p, name, drcs[p][name], ref)
            # the rate-controlling step is the reference's
            assert max(drcs[p], key=drcs[p].get) == max(c['drc_input'], key=c['drc_input'].get)
    _record('dmtm_drc_pressure.json', worst)


# ----------------------------------------------------------------------------
# reference test/test_1.py through the drop-in drivers
# ----------------------------------------------------------------------------
def test_reference_test_1_steps_4_5_7(P, inputs, tmp_path):
    """test/test_1.py:40-90 (step 6, the energy-span model, is out of scope):
    run() -> solution[-1] (step 4); run_temperatures(400..800, tof_terms,
    steady_state_solve=True, save_results=True) -> drcs_vs_temperature.csv with
    r9 rate-controlling at 400 K (step 5); save_state_energies / save_energies
    -> the energy CSVs and their goldens (step 7).  Every number on the device."""
    import pandas as pd
    from pycatkin_amd.functions.presets import (get_tof_for_given_reactions, run, run_temperatures,
                                                save_energies, save_energies_temperatures, save_state_energies)
    sim_system = P.read_from_input_file(os.path.join(inputs, 'DMTM', 'input.json'))
    tmpdir = str(tmp_path) + '/'
    # (4/7)
    run(sim_system=sim_system)
    ads = sim_system.adsorbate_indices
    assert abs(1 - np.sum(sim_system.solution[-1][ads])) <= 1e-6
    assert np.max(sim_system.solution[-1][ads]) > 0.999
    assert sim_system.snames[[i for i in ads if sim_system.solution[-1][i] ==
                              np.max(sim_system.solution[-1][ads])][0]] == 'sCH3OH'
    # presets.get_tof_for_given_reactions at that state = the oracle's rates there
    spec = O.load_spec(os.path.join(inputs, 'DMTM', 'input.json'))
    m = O.ClassicModel(spec)
    full = np.zeros(len(m.snames))
    for nm, v in zip(sim_system.snames, sim_system.solution[-1]):
        full[m.idx[nm]] = v
    tof = get_tof_for_given_reactions(sim_system, ['r5', 'r9'])
    assert abs(tof - m.tof(full, ['r5', 'r9'])) <= 1e-9 * abs(m.tof(full, ['r5', 'r9'])) + 1e-300
    # (5/7)
    tof_terms = ['r5', 'r9']
    temperatures = np.linspace(start=400, stop=800, num=2, endpoint=True)
    run_temperatures(sim_system=sim_system, temperatures=temperatures, tof_terms=tof_terms,
                     steady_state_solve=True, save_results=True, csv_path=tmpdir)
    assert os.path.isfile(tmpdir + 'drcs_vs_temperature.csv')
    df = pd.read_csv(filepath_or_buffer=tmpdir + 'drcs_vs_temperature.csv')
    assert [i for i in df.columns[1::] if df[i][0] == max(df.T[0][1::])][0] == 'r9'
    # (7/7)
    save_state_energies(sim_system=sim_system, csv_path=tmpdir)
    assert os.path.isfile(tmpdir + 'state_energies_800.0K_1.0bar.csv')
    df = pd.read_csv(filepath_or_buffer=tmpdir + 'state_energies_800.0K_1.0bar.csv')
    assert abs(max(df['Free (eV)']) - (-7.864)) <= 1e-3
    assert abs(max(df['Vibrational (eV)']) - 1.142) <= 1e-3
    assert abs(min(df['Rotational (eV)']) - (-1.259)) <= 1e-3
    assert abs(min(df['Translational (eV)']) - (-0.659)) <= 1e-3
    save_energies(sim_system=sim_system, csv_path=tmpdir)
    assert os.path.isfile(tmpdir + 'reaction_energies_and_barriers_800.0K_1.0bar.csv')
    df = pd.read_csv(filepath_or_buffer=tmpdir + 'reaction_energies_and_barriers_800.0K_1.0bar.csv')
    assert abs(max(df['dEr (J/mol)']) - 220788.916) <= 1e-3
    assert abs(max(df['dGr (J/mol)']) - 66358.978) <= 1e-3
    assert abs(max(df['dEa (J/mol)']) - 138934.617) <= 1e-3
    assert abs(max(df['dGa (J/mol)']) - 230155.396) <= 1e-3
    # the same energies against the oracle, every state / reaction (not only the extremes)
    th = O.Thermo(spec, 800.0, spec['system']['p'])
    st = pd.read_csv(tmpdir + 'state_energies_800.0K_1.0bar.csv').set_index('State')
    for nm in st.index:
        sd = spec['states'][nm]
        np.testing.assert_allclose(st.loc[nm, 'Free (eV)'], th.free(nm), rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(st.loc[nm, 'Vibrational (eV)'], th.vib(sd), rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(st.loc[nm, 'Translational (eV)'], th.rot(sd), rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(st.loc[nm, 'Rotational (eV)'], th.tran(sd), rtol=1e-10, atol=1e-12)
    save_energies_temperatures(sim_system=sim_system, temperatures=[500.0, 700.0], csv_path=tmpdir)
    assert sim_system.params['temperature'] == 700.0
    for rname in spec['reactions']:
        dfr = pd.read_csv(tmpdir + 'reaction_energies_and_barriers_%s.csv' % rname)
        for k, T in enumerate((500.0, 700.0)):
            e = O.Thermo(spec, T, spec['system']['p']).energies(rname)
            for col, key in (('dEr (J/mol)', 'dErxn'), ('dGr (J/mol)', 'dGrxn'), ('dEa (J/mol)', 'dEa_fwd'),
                             ('dGa (J/mol)', 'dGa_fwd')):
                np.testing.assert_allclose(dfr[col][k], e[key], rtol=1e-10, atol=1e-6)


def _not_reached_node(P, inputs):
    """A fixture node deep in the O-poisoned corner whose transient has not
    reached a steady state at t_end (status 4), set up as cooxvolcano.py:28-44."""
    from pycatkin_amd.functions.volcano import set_volcano_energies
    fx = np.load(os.path.join(GOLDEN, 'volcano_fixture.npz'))
    lo, hi, G = fx['grid']
    be = np.linspace(lo, hi, int(G))
    cand = np.nonzero(~fx['regular'] & fx['tight_ok'])[0]
    k = int(cand[np.argmax(be[fx['i'][cand]] - be[fx['j'][cand]])])
    s = P.read_from_input_file(os.path.join(inputs, 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    return s, float(be[fx['i'][k]]), float(be[fx['j'][k]])


def test_drc_at_a_not_reached_node(P, inputs):
    """degree_of_rate_control(ss_solve=True) at a node whose transient has not
    reached a steady state returns its xi, as the reference's does (it never
    raises on least_squares' answer): every one of the 2R+1 solves reports by
    the steady rule, and the batch's status says 4, or 6 where
    some of the perturbed solves reach a root and others do not (ADVICE r4:
    PCK_ST_DRC_MIXED, the central difference then mixes the rule's two
    answers)."""
    s, eco, eo = _not_reached_node(P, inputs)
    d = s.drc_batch(('CO_ox',), T=[600.0], desc={'ECO': [eco], 'EO': [eo]}, eps=1e-3, steady=True)
    assert d['status'][0] in (4, 6), d['status']
    assert all(np.isfinite(d[name][0]) for name in s.reactions)
    assert np.isfinite(d['tof0'][0]) and d['tof0'][0] > 0


def test_trajectory_untouched_by_a_retry_pass(P, inputs):
    """solve_batch(steady=True, t_out=..., retry=...): the optional second
    launch over the status-4 conditions re-integrates their end state but never
    writes trajectory samples (a failed retry keeps the first pass's outputs,
    and a partly rewritten trajectory would mix the two -- ADVICE r3): the
    trajectory equals the one of the same solve without the retry."""
    s, eco, eo = _not_reached_node(P, inputs)
    t_out = np.concatenate([[0.0], np.logspace(-6, np.log10(3600.0), 40)])
    kw = dict(T=[600.0], desc={'ECO': [eco], 'EO': [eo]}, tof_terms=('CO_ox',), steady=True, t_out=t_out)
    a = s.solve_batch(**kw)
    b = s.solve_batch(retry=(1e-8, 1e-22), **kw)
    assert a['status'][0] == 4 and b['status'][0] in (4, 5)
    np.testing.assert_array_equal(a['traj'], b['traj'])
    assert not np.array_equal(a['y'], b['y'])       # the retry did re-integrate the end state


def test_drc_screening_pass_matches_single_pass(P, inputs):
    """drc_batch(steady=True) screens each of the 2R+1 lane solves on its own
    ('auto' on the one-lane volcano network): statuses equal and the degrees
    of rate control within 1e-8 of the single pass on a reached node, the
    not-reached fixture node and a few grid points."""
    s, eco, eo = _not_reached_node(P, inputs)
    E1 = np.array([eco, -1.0, -1.5, -0.5, -2.0])
    E2 = np.array([eo, -1.0, -0.5, -1.5, -0.25])
    kw = dict(T=np.full(5, 600.0), desc={'ECO': E1, 'EO': E2}, eps=1e-3, steady=True)
    a = s.drc_batch(('CO_ox',), screen=None, **kw)
    b = s.drc_batch(('CO_ox',), **kw)
    np.testing.assert_array_equal(a['status'], b['status'])
    assert np.any(a['status'] == 0)
    for name in s.reactions:
        np.testing.assert_allclose(b[name], a[name], rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(b['tof0'], a['tof0'], rtol=1e-10)
