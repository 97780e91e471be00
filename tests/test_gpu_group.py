"""Lane-group solver (csrc/mk_group.h): networks with more than 8 dynamic
species, through the C-ABI, against the oracle and the reference's vectors.

Tolerances as in test_gpu_parity.py: rates / Jacobians 1e-11 relative,
steady-state coverages 1e-6 relative (1e-15 absolute floor)."""
import copy
import json
import os

import numpy as np
import pytest

from oracle import mk_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, 'golden', 'ref_vectors.json')))


@pytest.fixture(scope='module')
def P():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    import pycatkin_amd
    return pycatkin_amd


def close(a, b, rtol=1e-6, floor=1e-15):
    a, b = np.asarray(a), np.asarray(b)
    return np.all(np.abs(a - b) <= rtol * np.abs(b) + floor)


def _volcano(P, inputs):
    from pycatkin_amd.functions.volcano import set_volcano_energies
    s = P.read_from_input_file(os.path.join(inputs, 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    return s


SPLIT_FIXTURE = os.path.join(HERE, 'golden', 'split_fixture.npz')


def _counts(x):
    return dict(zip(*[v.tolist() for v in np.unique(x, return_counts=True)]))


def _vs_oracle(name, r, ids, fx, near):
    """A one-line account of one side's classification against the oracle's
    rule (status 0 = the root is the answer), or '' if it agrees."""
    reg = fx['regular']
    got0 = r['status'] == 0
    wrong = (got0 != reg) & ~near
    odd = ~np.isin(r['status'], (0, 4))
    if not wrong.any() and not odd.any():
        return ''
    idx = np.flatnonzero(wrong | odd)
    pairs = _counts(np.array(['%d/%s' % (s, 'reg' if g else 'nr') for s, g in zip(r['status'][idx], reg[idx])]))
    ex = ['#%d (E_CO %.4f, E_O %.4f, oracle crit %.3g, status %d, steps %d)' % (
        k, fx['ECO'][k], fx['EO'][k], fx['crit'][k], r['status'][k], r['nsteps'][k]) for k in idx[:6]]
    return ('%s (plan id %d, group kernel %d): statuses %s; %d of %d points off the oracle rule '
            '(status/oracle pairs %s), e.g. %s' % (name, ids[0], ids[1], _counts(r['status']), idx.size,
                                                   r['status'].size, pairs, '; '.join(ex)))


def test_group_solver_matches_lane_solver_on_volcano(P, inputs):
    """The volcano network forced onto the lane-group solver (PCK_PLAN_GROUP)
    against the one-lane-per-condition runtime-plan solver, and each of them
    against the oracle's steady-state rule on the same 1024 points
    (tests/golden/split_fixture.npz, make_split_fixture.py): a point may be
    classified differently only where the oracle's criterion lies within 2x of
    ROOT_DIST (none of these 1024 does; the nearest is 2.35x away).  A failure
    names the side that is off, its status / oracle pairs and whether an
    immediate repeat of that side gives bitwise the same statuses."""
    from pycatkin_amd.classes.system import ROOT_DIST
    fx = np.load(SPLIT_FIXTURE)
    s = _volcano(P, inputs)
    net = s.device(('CO_ox',))
    rng = np.random.default_rng(11)
    n = 1024
    kw = dict(T=np.full(n, 600.0), desc={'ECO': rng.uniform(-2.5, 0.5, n), 'EO': rng.uniform(-2.5, 0.5, n)},
              tof_terms=('CO_ox',), steady=True, activity=True)
    assert np.array_equal(kw['desc']['ECO'], fx['ECO']) and np.array_equal(kw['desc']['EO'], fx['EO'])
    crit = fx['crit']
    with np.errstate(divide='ignore', invalid='ignore'):
        near = np.isfinite(crit) & (np.abs(np.log(crit / ROOT_DIST)) <= np.log(2.0))

    def run(mode):
        net.set_plan_mode(mode)
        try:
            r = s.solve_batch(**kw)
            return r, (net.plan_id(), net.group_kernel())
        finally:
            net.set_plan_mode(0)

    a, ida = run(1)
    b, idb = run(2)
    msgs = []
    for name, mode, (r, ids) in (('lane runtime plan', 1, (a, ida)), ('lane group', 2, (b, idb))):
        m = _vs_oracle(name, r, ids, fx, near)
        if m:
            r2, _ = run(mode)
            m += '; a repeat of this side gives %s statuses (%d differ)' % (
                'the same' if np.array_equal(r2['status'], r['status']) else 'different',
                int((r2['status'] != r['status']).sum()))
            msgs.append(m)
    assert not msgs, ' || '.join(msgs)
    ok = (a['status'] == 0) & (b['status'] == 0)
    same = np.isclose(b['tof'], a['tof'], rtol=1e-9, atol=0.0) | (b['tof'] == a['tof'])
    bad = ok & ~same
    assert bad.sum() <= max(2, 0.005 * ok.sum()), [(int(k), a['tof'][k], b['tof'][k]) for k in np.flatnonzero(bad)[:8]]
    np.testing.assert_allclose(b['y'][:, ok & same], a['y'][:, ok & same], rtol=1e-8, atol=1e-15)
    # transient only (no polish): same integrator, same steps up to rounding
    kw['steady'] = False
    a, ida = run(1)
    b, idb = run(2)
    assert np.all(a['status'] == 0) and np.all(b['status'] == 0), (ida, _counts(a['status']), idb, _counts(b['status']))
    np.testing.assert_allclose(b['tof'], a['tof'], rtol=1e-6)


def test_group_drift_removal_keeps_species_outside_the_laws(P, inputs):
    """The group integrator removes the stage increments' conserved-total
    drift along y restricted to each law's own species (mk_group.h: kproj).
    On the COOxReactor Pd111 CSTR the gas species (CO, O2, CO2) are dynamic
    and outside the site balance: forced onto the lane-group solver, every
    species of the transient and of the steady state matches the lane solver
    (which has no drift removal), and the site total stays at its start."""
    s = P.read_from_input_file(os.path.join(inputs, 'COOxReactor', 'input_Pd111.json'))
    plan = s.plan(('CO_ox',))
    net = s.device(('CO_ox',))
    C = np.asarray(plan.conservation, float)
    assert C.shape[0] >= 1
    outside = np.all(C == 0.0, axis=0)
    assert outside.any(), (plan.dyn, C)        # species outside every law exist
    T = np.linspace(423.0, 623.0, 256)
    for steady in (False, True):
        kw = dict(T=T, tof_terms=('CO_ox',), steady=steady, rtol=1e-9, atol=1e-14)
        a = s.solve_batch(**kw)
        net.set_plan_mode(2)
        try:
            b = s.solve_batch(**kw)
            gk = net.group_kernel()
        finally:
            net.set_plan_mode(0)
        assert np.all(a['status'] == 0) and np.all(b['status'] == 0), (steady, _counts(a['status']), _counts(b['status']))
        y0 = np.asarray(plan.y0_default, float)
        np.testing.assert_allclose(C @ b['y'], np.repeat((C @ y0)[:, None], T.size, 1), rtol=1e-12, atol=1e-15,
                                   err_msg='site totals, group kernel %d' % gk)
        tol = 1e-7 if steady else 1e-6
        assert close(b['y'][outside], a['y'][outside], rtol=tol, floor=1e-14), \
            ('gas species', steady, np.max(np.abs(b['y'][outside] - a['y'][outside]) / np.abs(a['y'][outside])))
        assert close(b['y'], a['y'], rtol=tol, floor=1e-14), ('all species', steady, gk)


def test_group_rates_jacobian_on_volcano(P, inputs):
    s = _volcano(P, inputs)
    plan = s.plan()
    net = s.device()
    rng = np.random.default_rng(4)
    n = 200
    d = {'ECO': rng.uniform(-2.5, 0.5, n), 'EO': rng.uniform(-2.5, 0.5, n)}
    T = rng.uniform(450, 750, n)
    y = rng.uniform(0, 1, (len(plan.dyn), n))
    Tt, p, dd, fx, y0, inflow = s._inputs(net, plan, n, T, None, d, None, None, None)
    kf, kr = net.rate_constants(n, Tt, p, dd)
    out = {}
    for mode in (1, 2):
        net.set_plan_mode(mode)
        out[mode] = (net.species_rates(n, Tt, p, y, kf, kr, dd, fx, inflow).cpu().numpy(),
                     net.jacobian(n, Tt, p, y, kf, kr, dd, fx, inflow).cpu().numpy())
    net.set_plan_mode(0)
    np.testing.assert_allclose(out[2][0], out[1][0], rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(out[2][1], out[1][1], rtol=1e-12, atol=1e-300)


def _dmtm(P, inputs, mode='classic'):
    return P.read_from_input_file(os.path.join(inputs, 'DMTM', 'input.json'), rate_model=mode)


@pytest.mark.parametrize('mode', ['classic', 'patched'])
def test_dmtm_rates_jacobian_vs_oracle(P, inputs, mode):
    """11 dynamic species: pck_species_rates / pck_jacobian (lane groups of 16)
    vs old_system species_odes / species_jacobian (oracle, pinned by the
    reference's own species_odes vectors)."""
    s = _dmtm(P, inputs, mode)
    plan = s.plan()
    net = s.device()
    assert net.NDYN == 11
    spec = O.load_spec(os.path.join(inputs, 'DMTM', 'input.json'))
    rng = np.random.default_rng(8)
    n = 24
    T = np.linspace(350.0, 900.0, n)
    y = rng.uniform(0, 1, (11, n))
    Tt, p, d, fx, y0, inflow = s._inputs(net, plan, n, T, None, None, None, None, None)
    kf, kr = net.rate_constants(n, Tt, p, d)
    f = net.species_rates(n, Tt, p, y, kf, kr, d, fx, inflow).cpu().numpy()
    J = net.jacobian(n, Tt, p, y, kf, kr, d, fx, inflow).cpu().numpy()
    for c in range(n):
        m = O.ClassicModel(spec, T=T[c], mode=mode)
        full = m.y0.copy()
        dyn = [m.idx[nm] for nm in plan.dyn]
        full[dyn] = y[:, c]
        np.testing.assert_allclose(f[:, c], m.rhs(full)[dyn], rtol=1e-11, atol=1e-300)
        Jr = m.jac(full)[np.ix_(dyn, dyn)]
        np.testing.assert_allclose(J[:, :, c], Jr, rtol=1e-11, atol=1e-12 * np.abs(Jr).max())


def test_dmtm_steady_and_tof_vs_reference(P, inputs):
    """examples/DMTM: transient to t = 1e12 s then Newton polish at 400 / 600 /
    800 K.  Steady coverages vs the oracle's polished root (1e-6) and vs the
    reference's find_steady output (least_squares, 1e-5 on coverages > 1e-6);
    TOF(r5 + r9) vs the reference's run_and_return_tof."""
    s = _dmtm(P, inputs)
    g = GOLD['dmtm_classic']
    T = np.array(g['temperatures'])
    r = s.solve_batch(T=T, tof_terms=('r5', 'r9'), steady=True, rtol=1e-10, atol=1e-14)
    assert np.all(r['status'] == 0), r['status']
    plan = s.plan(('r5', 'r9'))
    spec = O.load_spec(os.path.join(inputs, 'DMTM', 'input.json'))
    for k, t in enumerate(T):
        m = O.ClassicModel(spec, T=t)
        yT, _ = m.solve_odes(rtol=1e-10, atol=1e-14)
        ys = m.find_steady(yT)
        assert m.regular
        dyn = [m.idx[nm] for nm in plan.dyn]
        assert close(r['y'][:, k], ys[dyn]), (t, r['y'][:, k], ys[dyn])
        ref = np.array(g['y_steady'][k])[[g['snames'].index(nm) for nm in plan.dyn]]
        big = ref > 1e-6
        np.testing.assert_allclose(r['y'][big, k], ref[big], rtol=1e-5)
        np.testing.assert_allclose(r['tof'][k], g['tof'][k], rtol=1e-4)


def test_dmtm_drc_vs_reference(P, inputs):
    """degree_of_rate_control(['r5', 'r9'], eps=5e-2) at 400 / 600 / 800 K
    (test/test_1.py:421-432 pins r9 as rate-controlling at 400 K).  The group
    path runs 2R+1 = 23 perturbed solves per condition and combines them."""
    s = _dmtm(P, inputs)
    g = GOLD['dmtm_classic']
    T = np.array(g['temperatures'])
    r = s.drc_batch(('r5', 'r9'), T=T, eps=5.0e-2, steady=True, rtol=1e-10, atol=1e-14)
    assert np.all(r['status'] == 0), r['status']
    xi = np.array([r[name] for name in g['reactions']])
    assert g['reactions'][int(np.argmax(xi[:, 0]))] == 'r9'
    spec = O.load_spec(os.path.join(inputs, 'DMTM', 'input.json'))
    for k, t in enumerate(T):
        m = O.ClassicModel(spec, T=t)
        ref = m.drc(['r5', 'r9'], eps=5.0e-2, steady=True)
        for j, name in enumerate(g['reactions']):
            assert abs(xi[j, k] - ref[name]) <= 1e-6 * max(1.0, abs(ref[name])), (t, name, xi[j, k], ref[name])
        # the reference's own (transient, rtol 1e-6) DRC
        np.testing.assert_allclose(xi[:, k], g['drc'][k], atol=2e-3)


def _ch4(P, inputs, EC=1.5, EO=0.2):
    """test/CH4_input.json in the patched system.py formulation (the class the
    reference's read_from_input_file builds), descriptor energies as in
    test/tests.py:40-42; sC / sO get the matching electronic energies (the
    input gives them none -- oracle.ch4_setup)."""
    s = P.read_from_input_file(os.path.join(inputs, 'CH4', 'input.json'), formulation='patched')
    s.reactions['C_ads'].dErxn_user = EC
    s.reactions['O_ads'].dErxn_user = EO
    s.states['sC'].Gelec = EC
    s.states['sO'].Gelec = EO
    spec = O.ch4_setup(O.load_spec(os.path.join(inputs, 'CH4', 'input.json')), EC, EO)
    return s, spec


def test_ch4_rates_jacobian_vs_oracle(P, inputs):
    """16 dynamic species, 58 reactions, 8 fixed gases: system.py _fun_ss /
    _jac_ss (oracle PatchedModel) vs pck_species_rates / pck_jacobian."""
    s, spec = _ch4(P, inputs)
    plan = s.plan()
    net = s.device()
    assert net.NDYN == 16
    rng = np.random.default_rng(21)
    n = 8
    T = np.linspace(450.0, 650.0, n)
    y = rng.uniform(0.01, 1.0, (16, n))
    Tt, p, d, fx, y0, inflow = s._inputs(net, plan, n, T, None, None, None, None, None)
    kf, kr = net.rate_constants(n, Tt, p, d)
    f = net.species_rates(n, Tt, p, y, kf, kr, d, fx, inflow).cpu().numpy()
    J = net.jacobian(n, Tt, p, y, kf, kr, d, fx, inflow).cpu().numpy()
    for c in range(n):
        m = O.PatchedModel(spec, T=T[c])
        names = sorted(m.index, key=m.index.get)[m.ngas:]
        perm = [names.index(nm) for nm in plan.dyn]
        ys = np.zeros(len(names))
        ys[perm] = y[:, c]
        fr = m.fun_ss(ys)[perm]
        Jr = m.jac_ss(ys)[np.ix_(perm, perm)]
        np.testing.assert_allclose(f[:, c], fr, rtol=1e-10, atol=1e-12 * np.abs(fr).max())
        np.testing.assert_allclose(J[:, :, c], Jr, rtol=1e-10, atol=1e-12 * np.abs(Jr).max())


@pytest.mark.parametrize('EC,EO,tmax', [(1.0, 1.0, 1e4), (1.5, 0.2, 1e-6)])
def test_ch4_transient_vs_oracle(P, inputs, EC, EO, tmax):
    """BASELINE configs[0]: SteadyStateSolver.solve_ode (solver.py:374-418,
    rtol 1e-10 / atol 1e-12) from the normalised start state, at 1e-6
    relative against the oracle integrated to rtol 1e-13 / atol 1e-20
    (lsoda), with an absolute floor of the solve's atol 1e-12: a component at
    the atol level carries an absolute error of that order by the definition
    of the error control (the reference's own scipy BDF at 1e-10 / 1e-12 is
    2.1e-6 off the tight solution on a 1e-10 component at 473 K).  The
    patched +-1 reaction matrix does not conserve the s-site group, and at
    the tests.py descriptors (1.5, 0.2) scipy BDF itself fails beyond ~1e-3 s
    (O poisoning drives s negative), so that case is compared at 1e-6 s."""
    s, spec = _ch4(P, inputs, EC, EO)
    plan = s.plan()
    m = O.PatchedModel(spec, T=523.0)
    names = sorted(m.index, key=m.index.get)[m.ngas:]
    perm = [names.index(nm) for nm in plan.dyn]
    np.testing.assert_allclose(plan.y0_default, m.y0[m.ngas:][perm], rtol=1e-15)
    yT, sol = m.solve_ode(tmax=tmax, rtol=1e-13, atol=1e-20, method='LSODA')
    assert sol.status == 0
    r = s.solve_batch(T=np.array([523.0]), t0=0.0, t_end=tmax, rtol=1e-10, atol=1e-12)
    assert r['status'][0] == 0
    assert s.device().group_lanes() == 4                   # the default quad-group kernel
    assert close(r['y'][:, 0], yT[perm], rtol=1e-6, floor=1e-12), (r['y'][:, 0], yT[perm])


def test_ch4_bench_config_vs_fixture(P, inputs):
    """bench.py --config ch4 itself: 16 384 temperatures (473-573 K, E_C =
    E_O = 1 eV) to 1e4 s at rtol 1e-10 / atol 1e-12 in one launch on the
    default quad-group kernel, against tests/golden/ch4_fixture.npz (the
    oracle at rtol 1e-13 / atol 1e-20, make_ch4_fixture.py) at 8 of those
    temperatures: 1e-6 relative with the solve's atol as absolute floor."""
    import json
    s, _ = _ch4(P, inputs, 1.0, 1.0)
    plan = s.plan()
    fx = dict(np.load(os.path.join(HERE, 'golden', 'ch4_fixture.npz')))
    T = np.linspace(473.0, 573.0, 16384)
    np.testing.assert_array_equal(T[fx['idx']], fx['T'])
    r = s.solve_batch(T=T, t0=0.0, t_end=1e4, rtol=1e-10, atol=1e-12)
    assert s.device().group_lanes() == 4
    assert np.all(r['status'] == 0), np.unique(r['status'], return_counts=True)
    names = [str(x) for x in fx['names']]
    perm = [names.index(nm) for nm in plan.dyn]
    y = r['y'][:, fx['idx']].T
    ref = fx['y'][:, perm]
    err = np.abs(y - ref)
    rel = np.where(ref > 1e-10, err / np.maximum(ref, 1e-300), 0.0)
    info = {"max_rel_above_1e-10": float(rel.max()), "max_abs": float(err.max()),
                "worst": [plan.dyn[int(i)] for i in np.argmax(rel, axis=1)]}
    if os.path.isdir('gpurun_out'):
        json.dump(info, open('gpurun_out/ch4_bench_fixture.json', 'w'), indent=1)
    assert np.all(err <= 1e-6 * np.abs(ref) + 1e-12), info


@pytest.fixture(scope='module')
def synthetic(P):
    from pycatkin_amd.functions.synthetic import synthetic_system
    return synthetic_system()


def test_synthetic_rates_jacobian_vs_oracle(P, synthetic):
    """BASELINE configs[4] network (50 dynamic species, 150 reactions, groups
    of 64 lanes): rates / Jacobian at random states and random descriptors."""
    from _synth import spec_of
    sim, net = synthetic
    plan = sim.plan()
    dnet = sim.device()
    assert dnet.NDYN == 50 and dnet.NRXN == 150
    rng = np.random.default_rng(31)
    n = 6
    D = rng.uniform(-0.5, 0.5, (4, n))
    T = np.linspace(450.0, 650.0, n)
    y = rng.uniform(0.0, 0.05, (50, n))
    desc = {'D%d' % k: D[k] for k in range(4)}
    Tt, p, d, fx, y0, inflow = sim._inputs(dnet, plan, n, T, None, desc, None, None, None)
    kf, kr = dnet.rate_constants(n, Tt, p, d)
    f = dnet.species_rates(n, Tt, p, y, kf, kr, d, fx, inflow).cpu().numpy()
    J = dnet.jacobian(n, Tt, p, y, kf, kr, d, fx, inflow).cpu().numpy()
    for c in range(n):
        m = O.ClassicModel(spec_of(net, D[:, c], T[c]), T=T[c])
        full = m.y0.copy()
        dyn = [m.idx[nm] for nm in plan.dyn]
        full[dyn] = y[:, c]
        fr = m.rhs(full)[dyn]
        Jr = m.jac(full)[np.ix_(dyn, dyn)]
        np.testing.assert_allclose(f[:, c], fr, rtol=1e-10, atol=1e-12 * np.abs(fr).max())
        np.testing.assert_allclose(J[:, :, c], Jr, rtol=1e-10, atol=1e-12 * np.abs(Jr).max())


def test_synthetic_fixture_parity(P, synthetic):
    """BASELINE configs[4] against tests/golden/synthetic_fixture.npz
    (make_synthetic_fixture.py: 324 rows of the bench's own condition set,
    the former stragglers 17825 / 39547 / 37890 / 30513 among them; the
    oracle's restatement of the steady-state rule from its tight transient,
    lsoda at rtol 1e-11 / atol 1e-20).

    The fixture rows are solved inside the whole 65 536-condition bench set
    (one launch at the bench's rtol 1e-7 / atol 1e-22, the library's default
    step budget): every condition ends
    with status 0 (steady state reached) or 4 (the transient end), the site
    balance holds everywhere, and at the fixture rows
      * log10(TOF of R0) within 1e-6 relative of the oracle's answer (the
        TOF itself where it is negative: G0 desorbing on balance);
      * coverages within 1e-6 relative of the root where both sides find the
        steady state reached, within 1e-5 of the tight transient where
        neither does (these random networks still drift along a slow
        manifold at t_end = 1e4 s; floor 1e-20, the oracle's atol);
      * the classification differs only where the oracle's criterion lies
        within a factor 2 of ROOT_DIST."""
    import json
    from pycatkin_amd.classes.system import ROOT_DIST
    sim, net = synthetic
    plan = sim.plan(('R0',))
    fx = dict(np.load(os.path.join(HERE, 'golden', 'synthetic_fixture.npz')))
    D = np.random.default_rng(0).uniform(-0.5, 0.5, (65536, 4))
    np.testing.assert_array_equal(D[fx['idx']], fx['desc'])
    # the bench's tolerances (bench.SYNTHETIC_TOL): at the default 1e-6 two of
    # the 324 rows miss 1e-6 (max 4.4e-6; tools/synthetic_tol_probe.py)
    r = sim.solve_batch(T=np.full(D.shape[0], 500.0), desc={'D%d' % k: D[:, k] for k in range(4)},
                        tof_terms=('R0',), steady=True, rtol=1e-7, atol=1e-22)
    st = r['status']
    counts = {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))}
    assert set(counts) <= {0, 4}, counts
    Cm = plan.conservation
    tot0 = Cm @ plan.y0_default
    np.testing.assert_allclose(Cm @ r['y'], np.repeat(tot0[:, None], D.shape[0], axis=1), rtol=0, atol=1e-10)
    k = fx['idx']
    ok = fx['ok']
    names = [str(x) for x in fx['dyn']]
    y = r['y'][[plan.dyn.index(nm) for nm in names]][:, k].T
    tof = r['tof'][k]
    dev = st[k] == 0
    # log10(TOF) at 1e-6 relative where the TOF is positive; a negative TOF
    # (G0 desorbing on balance) at 1e-6 relative on the TOF itself
    pos = (fx['tof'] > 0) & (tof > 0)
    err = np.where(pos, np.abs(np.log10(np.where(pos, tof, 1.0)) - fx['l10']) / np.abs(np.where(pos, fx['l10'], 1.0)),
                   np.abs(tof - fx['tof']) / np.abs(fx['tof']))
    # coverages: a root to 1e-6; a transient still moving at t_end to the two
    # integrators' accuracy on its smallest components, 1e-5 at rtol 1e-7
    # (measured max 3.0e-6, p99 7.7e-7: profiles/r4/synthetic_tol_probe.jsonl)
    cov_rtol = np.where(fx['regular'], 1e-6, 1e-5)[:, None]
    cov = np.abs(y - fx['y_root']) <= cov_rtol * np.abs(fx['y_root']) + 1e-20
    flips = np.nonzero((dev != fx['regular']) & ok)[0]
    info = dict(counts=counts, n_fixture=int(k.size), n_compared=int(ok.sum()), oracle_reached=int(fx['regular'].sum()),
                device_reached=int(dev.sum()), max_rel_l10=float(err[ok].max()),
                worst=int(k[ok][np.argmax(err[ok])]), flips=[(int(k[f]), int(st[k[f]]), float(fx['crit'][f])) for f in flips])
    if os.path.isdir('gpurun_out'):
        json.dump(info, open('gpurun_out/synthetic_fixture_parity.json', 'w'), indent=1)
    assert ok.sum() >= 300, info
    assert np.all(err[ok] <= 1e-6), info
    same = ok & (dev == fx['regular'])
    assert np.all(cov[same]), [int(k[q]) for q in np.nonzero(same & ~np.all(cov, axis=1))[0][:5]]
    for f in flips:
        assert 0.5 * ROOT_DIST <= fx['crit'][f] <= 2.0 * ROOT_DIST, info['flips']


def test_screening_refused_on_64_lane_groups(P, synthetic):
    """The 64-lane group kernel carries one integrator copy and no screening
    trip: an explicit screen on the 50-species network is refused (C-ABI
    PCK_E_ARG), not silently run as a single pass."""
    sim, _ = synthetic
    D = np.zeros((2, 4))
    with pytest.raises(RuntimeError, match='screen'):
        sim.solve_batch(T=np.full(2, 500.0), desc={'D%d' % k: D[:, k] for k in range(4)}, steady=True,
                        screen=3e-2, max_steps=50)


def test_group_exact_size_kernel_matches_compiled(P, inputs, monkeypatch):
    """The lane-group solver hipRTC specialises for the network's exact size
    (k_solve_grp<11, 16, 1> for DMTM) and the compiled-in padded kernel
    (k_solve_grp<16, 16, 1>, PCK_JIT=0) do the same arithmetic in the same
    order: bitwise-equal states, TOFs and step counts.  Two runs of the same
    launch are bitwise equal too (no cross-lane atomics in the sums).  Both
    are the record-table kernels (PCK_GRP_CT=0; the compile-time network is
    checked against them in test_group_compile_time_network_matches_tables)."""
    s = _dmtm(P, inputs)
    T = np.linspace(400.0, 800.0, 64)
    kw = dict(T=T, tof_terms=('r5', 'r9'), steady=True)
    monkeypatch.setenv('PCK_GRP_CT', '0')
    a = s.solve_batch(**kw)
    assert s.device(('r5', 'r9')).group_kernel() == 1
    b = s.solve_batch(**kw)
    monkeypatch.setenv('PCK_JIT', '0')
    c = s.solve_batch(**kw)
    assert s.device(('r5', 'r9')).group_kernel() == 0
    monkeypatch.delenv('PCK_JIT')
    monkeypatch.delenv('PCK_GRP_CT')
    for k in ('y', 'tof', 'status', 'nsteps'):
        np.testing.assert_array_equal(a[k], b[k])
        np.testing.assert_array_equal(a[k], c[k])
    assert np.all(a['status'] == 0)


@pytest.mark.parametrize('which', ['dmtm', 'ch4', 'dmtm_drc'])
def test_group_compile_time_network_matches_tables(P, inputs, monkeypatch, which):
    """The lane-group solver with the network compiled in (hipRTC, mk_group.h:
    ct_rhs / ct_jac: every lane evaluates every reaction in straight-line
    code) against the record-table kernel of the same size (PCK_GRP_CT=0):
    the same statuses, states and TOFs to rounding -- the two sum the same
    terms in a different order.  DMTM steady states over T, the CH4 transient
    (SteadyStateSolver's rtol 1e-10 / atol 1e-12) and the DMTM transient DRC."""
    if which == 'ch4':
        s, _ = _ch4(P, inputs)
        net = s.device()
        kw = dict(T=np.linspace(473.0, 573.0, 256), t0=0.0, t_end=1e4, rtol=1e-10, atol=1e-12)
        run = lambda: s.solve_batch(**kw)
        tol = 1e-7
    elif which == 'dmtm':
        s = _dmtm(P, inputs)
        net = s.device(('r5', 'r9'))
        run = lambda: s.solve_batch(T=np.linspace(400.0, 800.0, 256), tof_terms=('r5', 'r9'), steady=True)
        tol = 1e-9
    else:
        s = _dmtm(P, inputs)
        net = s.device(('r5', 'r9'))
        run = lambda: s.drc_batch(('r5', 'r9'), T=np.linspace(400.0, 800.0, 64), eps=5.0e-2)
        tol = 1e-5
    monkeypatch.setenv('PCK_GRP_QUAD', '0')
    a = run()
    assert net.group_kernel() == 2
    monkeypatch.setenv('PCK_GRP_CT', '0')
    b = run()
    assert net.group_kernel() == 1
    monkeypatch.delenv('PCK_GRP_CT')
    monkeypatch.delenv('PCK_GRP_QUAD')
    np.testing.assert_array_equal(a['status'], b['status'])
    assert np.all(a['status'] == 0), np.unique(a['status'], return_counts=True)
    if which == 'dmtm_drc':
        for name in s.reactions:
            np.testing.assert_allclose(a[name], b[name], rtol=0, atol=tol)
        # transients at the input's rtol 1e-6: rounding moves the step sequence
        # (measured 3.5e-8 relative on the base TOF)
        np.testing.assert_allclose(a['tof0'], b['tof0'], rtol=1e-6)
        return
    assert close(a['y'], b['y'], rtol=tol, floor=1e-14), np.abs(a['y'] - b['y']).max()
    if which != 'ch4':
        np.testing.assert_allclose(a['tof'], b['tof'], rtol=tol)


def test_dmtm_pressure_sweep_vs_oracle(P, inputs):
    """BASELINE configs[3] pressure axis: run_parameters(..., 'pressure') at
    3 pressures x 3 temperatures, each condition with its own pressure in the
    gas free energies (state.py:329-331), steady state vs the oracle at 1e-6."""
    from pycatkin_amd.functions.presets import run_parameters
    spec = O.load_spec(os.path.join(inputs, 'DMTM', 'input.json'))
    for T in (450.0, 600.0, 750.0):
        s = _dmtm(P, inputs)
        s.params['temperature'] = T
        ps = np.array([1.0e4, 1.0e5, 1.0e6])
        final, rates, _ = run_parameters(s, ps, 'pressure', steady_state_solve=True)
        plan = s.plan()
        for k, p in enumerate(ps):
            m = O.ClassicModel(spec, T=T, p=p)
            yT, _ = m.solve_odes(rtol=1e-10, atol=1e-14)
            ys = m.find_steady(yT)
            assert m.regular
            got = np.array([final[k, plan.species.index(n)] for n in plan.dyn])
            ref = np.array([ys[m.idx[n]] for n in plan.dyn])
            assert close(got, ref), (T, p, got, ref)
            # rates_vs_pressure: r_fwd - r_rev of every reaction at the steady state
            rr = m.rates(ys)
            np.testing.assert_allclose(rates[k], rr[:, 0] - rr[:, 1], rtol=1e-6, atol=1e-12 * np.abs(rr).max())
        # the pressure really enters: the three steady states differ
        assert np.abs(final[0] - final[2]).max() > 1e-6


def test_dmtm_steady_state_at_large_steps_does_not_stall(P, inputs):
    """The DMTM DRC bench grid's slowest condition (622.2 K, 6.45e5 Pa; gross
    fluxes ~1e11 /s): on its steady state the rounding of the site balance,
    multiplied by h g at h ~ 1e9 s, used to drift the stage increments' site
    total and reject step after step (7 532 steps instead of 176; mk_group.h
    PCK_GRP_KPROJ, DESIGN.md "Integrator").  The plain solve and its 23-solve
    DRC take the ordinary step counts and the state matches the oracle's."""
    s = _dmtm(P, inputs)
    T = np.full(3, np.linspace(400.0, 800.0, 64)[35])    # bench.py dmtm_drc grid, condition 2297
    p = np.logspace(4.0, 6.0, 64)[[57, 56, 58]]
    r = s.solve_batch(T=T, p=p, tof_terms=('r5', 'r9'))
    assert np.all(r['status'] == 0), r['status']
    assert r['nsteps'].max() < 400, r['nsteps']
    d = s.drc_batch(('r5', 'r9'), T=T, p=p, eps=5.0e-2)
    assert np.all(d['status'] == 0) and d['nsteps'].max() < 23 * 400, d['nsteps']
    spec = O.load_spec(os.path.join(inputs, 'DMTM', 'input.json'))
    m = O.ClassicModel(spec, T=float(T[0]), p=float(p[0]))
    yT, _ = m.solve_odes(rtol=1e-10, atol=1e-14)
    plan = s.plan(('r5', 'r9'))
    ref = np.array([yT[m.idx[n]] for n in plan.dyn])
    # the transient at the input tolerances (1e-6 / 1e-8) against a tight one
    assert np.all(np.abs(r['y'][:, 0] - ref) <= 1e-4 * np.abs(ref) + 1e-8), (r['y'][:, 0], ref)


def _six_species_net():
    """A 12-species network whose reaction R0 has 6 dynamic participants and
    6 stoichiometric entries (the widest record of the lane-group plan)."""
    from pycatkin_amd.functions.synthetic import synthetic_network
    net = synthetic_network(n_species=12, n_reactions=24, seed=3)
    ads = net['adsorbates']
    net['reactions'][10] = ('surf', [ads[0], ads[1], ads[2]], [ads[3], ads[4], ads[5]])
    return net


def test_group_six_participant_reaction_vs_oracle(P):
    """Rates and Jacobian of a reaction with 6 participants / 6 stoichiometric
    species on the lane-group path (packed records, mk_group.h) vs the oracle."""
    from _synth import spec_of
    from pycatkin_amd.functions.synthetic import synthetic_system
    net = _six_species_net()
    sim, _ = synthetic_system(net)
    plan = sim.plan()
    dnet = sim.device()
    assert dnet.NDYN == 12
    rng = np.random.default_rng(5)
    n = 5
    D = rng.uniform(-0.3, 0.3, (4, n))
    T = np.linspace(480.0, 560.0, n)
    y = rng.uniform(0.01, 0.2, (12, n))
    desc = {'D%d' % k: D[k] for k in range(4)}
    Tt, p, d, fx, y0, inflow = sim._inputs(dnet, plan, n, T, None, desc, None, None, None)
    kf, kr = dnet.rate_constants(n, Tt, p, d)
    f = dnet.species_rates(n, Tt, p, y, kf, kr, d, fx, inflow).cpu().numpy()
    J = dnet.jacobian(n, Tt, p, y, kf, kr, d, fx, inflow).cpu().numpy()
    for c in range(n):
        m = O.ClassicModel(spec_of(net, D[:, c], T[c]), T=T[c])
        full = m.y0.copy()
        dyn = [m.idx[nm] for nm in plan.dyn]
        full[dyn] = y[:, c]
        fr, Jr = m.rhs(full)[dyn], m.jac(full)[np.ix_(dyn, dyn)]
        np.testing.assert_allclose(f[:, c], fr, rtol=1e-10, atol=1e-12 * np.abs(fr).max())
        np.testing.assert_allclose(J[:, :, c], Jr, rtol=1e-10, atol=1e-12 * np.abs(Jr).max())


def test_ch4_patched_api_vs_oracle(P, inputs):
    """The patched System's per-call API on the device (system.py:345-564):
    _calc_rates, get_dydt (every tracked species, gas rows included),
    _fun_ss, _jac_ss and the surface columns of get_jacobian, vs the oracle's
    PatchedModel at a random composition."""
    s, spec = _ch4(P, inputs)
    s.T = 523.0
    s.build()
    m = O.PatchedModel(spec, T=523.0)
    names = sorted(m.index, key=m.index.get)
    assert names == sorted(s.index_map, key=s.index_map.get)
    np.testing.assert_allclose(s.initial_system, m.y0, rtol=1e-15)
    rng = np.random.default_rng(7)
    y = m.normalize(rng.uniform(0.01, 1.0, len(names)))
    np.testing.assert_allclose(s.get_dydt(y), m.dydt(y), rtol=1e-10, atol=1e-12 * np.abs(m.dydt(y)).max())
    ys = y[m.ngas:]
    fr, Jr = m.fun_ss(ys), m.jac_ss(ys)
    np.testing.assert_allclose(s._fun_ss(ys), fr, rtol=1e-10, atol=1e-12 * np.abs(fr).max())
    np.testing.assert_allclose(s._jac_ss(ys), Jr, rtol=1e-10, atol=1e-12 * np.abs(Jr).max())
    Jf = s.get_jacobian(y)
    Jo = m.jacobian(y)
    np.testing.assert_allclose(Jf[:, m.ngas:], Jo[:, m.ngas:], rtol=1e-10, atol=1e-12 * np.abs(Jo).max())
    # gas columns as the reference returns them: P_term = p only for the OTHER
    # species of a side (system.py:478-484), so the exact column divided by p
    np.testing.assert_allclose(Jf[:, :m.ngas], Jo[:, :m.ngas] / float(s.p), rtol=1e-10,
                               atol=1e-12 * np.abs(Jo).max())
    rates = s._calc_rates(y)
    assert rates.shape == (len(s.rate_map), 2)
    np.testing.assert_allclose(s.reaction_matrix @ (rates[:, 0] - rates[:, 1]), m.dydt(y), rtol=1e-10,
                               atol=1e-12 * np.abs(m.dydt(y)).max())


def test_ch4_steady_state_solver(P, inputs):
    """BASELINE configs[0] on the drop-in: SteadyStateSolver(system).solve_ode()
    (solver.py:374-418: transient from the normalised start state to 1e4 s at
    rtol 1e-10 / atol 1e-12, then test_convergence), against the oracle's
    scipy BDF run of the same path at 1e-6.  The patched +-1 formulation does
    not conserve its site groups and never settles (the oracle's max|f| stays
    ~1e-4 out to 1e8 s and BDF blows up by 1e10 s), so solve_root's device
    Newton root is pinned by the oracle's own equations: fun_ss of the
    oracle vanishes there and the network's linear invariants keep their
    start values.  The batched solve_ode over temperatures equals single calls."""
    s, spec = _ch4(P, inputs, 1.0, 1.0)
    s.T = 523.0
    solver = P.SteadyStateSolver(s, ss_guess=None)
    res = solver.solve_ode(tmax=1e4)
    m = O.PatchedModel(spec, T=523.0)
    yT, sol = m.solve_ode(tmax=1e4, rtol=1e-10, atol=1e-12, method='BDF')
    assert sol.status == 0
    assert close(res.x, yT, rtol=1e-6, floor=1e-12), np.abs(res.x - yT).max()
    assert res.success == solver.test_convergence(yT)
    solver2 = P.SteadyStateSolver(s, ss_guess=yT)
    x, st = solver2._newton(solver2._norm(yT), 30)
    assert st == 0, st
    scale = np.abs(m.fun_ss(yT)).max() + np.abs(m.jac_ss(yT)).max() * 1e-12
    assert np.abs(m.fun_ss(x)).max() <= 1e-6 * scale + 1e-12, np.abs(m.fun_ss(x)).max()
    C = np.array(s.plan().conservation)
    if C.size:
        xp, yp = s._to_plan(s.plan(), x[:, None])[:, 0], s._to_plan(s.plan(), solver2._norm(yT)[:, None])[:, 0]
        np.testing.assert_allclose(C @ xp, C @ yp, rtol=1e-10, atol=1e-14)
    r2 = solver2.solve_root()
    # success only when the root itself passes the reference's checks
    # (solver.py:279-291); otherwise the best-scored candidate comes back
    assert (not r2.success) or solver2.test_convergence(r2.x)
    Y, ok = solver.solve_ode_batch(T=[473.0, 523.0, 573.0])
    assert ok[1] == res.success
    np.testing.assert_allclose(Y[:, 1], res.x, rtol=1e-12, atol=1e-300)


@pytest.mark.gpu
def test_dmtm_patched_rate_model_steady_vs_oracle(P, inputs):
    """rate_model='patched' (reaction.py:135-162: kads / kdes for non-activated
    adsorption) through a full device solve: transient to 1e12 s + Newton at
    three temperatures vs the oracle's scipy BDF + polished root on the same
    rate constants (1e-6 on coverages above 1e-6)."""
    s = P.read_from_input_file(os.path.join(inputs, 'DMTM', 'input.json'), rate_model='patched')
    T = np.array([450.0, 600.0, 750.0])
    r = s.solve_batch(T=T, tof_terms=('r5', 'r9'), steady=True, rtol=1e-10, atol=1e-14)
    plan = s.plan(('r5', 'r9'))
    spec = O.load_spec(os.path.join(inputs, 'DMTM', 'input.json'))
    for k, t in enumerate(T):
        m = O.ClassicModel(spec, T=t, mode='patched')
        yT, _ = m.solve_odes(rtol=1e-10, atol=1e-14)
        ys = m.find_steady(yT)
        dyn = [m.idx[nm] for nm in plan.dyn]
        if not m.regular:
            assert r['status'][k] in (0, 4), r['status'][k]
            continue
        assert r['status'][k] == 0, (t, r['status'][k])
        big = ys[dyn] > 1e-6
        np.testing.assert_allclose(r['y'][big, k], ys[dyn][big], rtol=1e-6)
        np.testing.assert_allclose(r['tof'][k], m.tof(ys, ['r5', 'r9']), rtol=1e-6)


def test_balanced_walk_matches_row_loops(P, inputs, synthetic, monkeypatch):
    """The balanced walk of the species CSR (mk_group.h GrpView::sch: long
    rows cut into pieces packed over the group's lanes) against the per-row
    loops it replaces (PCK_GRP_BALANCE=0 at network creation): the same sums
    in another order, so rates and Jacobians agree to rounding, and a CH4
    steady solve lands on the same root.  The synthetic network takes it
    (10 entries per lane instead of 56); CH4 (17 vs 35) does not by default,
    so its 'balanced' leg forces it (PCK_GRP_BALANCE=2)."""
    from pycatkin_amd.functions.synthetic import synthetic_system

    def evaluate(make, n, T, y, desc=None):
        s = make()
        plan = s.plan()
        net = s.device()
        Tt, p, d, fx, y0, inflow = s._inputs(net, plan, n, T, None, desc, None, None, None)
        kf, kr = net.rate_constants(n, Tt, p, d)
        f = net.species_rates(n, Tt, p, y, kf, kr, d, fx, inflow).cpu().numpy()
        J = net.jacobian(n, Tt, p, y, kf, kr, d, fx, inflow).cpu().numpy()
        return f, J

    rng = np.random.default_rng(5)
    cases = [(lambda: _ch4(P, inputs)[0], 8, np.linspace(450.0, 650.0, 8), rng.uniform(0.01, 1.0, (16, 8)), None)]
    D = rng.uniform(-0.5, 0.5, (4, 6))
    cases.append((lambda: synthetic_system()[0], 6, np.linspace(450.0, 650.0, 6), rng.uniform(0.0, 0.05, (50, 6)),
                  {'D%d' % k: D[k] for k in range(4)}))
    for make, n, T, y, desc in cases:
        monkeypatch.setenv('PCK_GRP_BALANCE', '2')
        fb, Jb = evaluate(make, n, T, y, desc)
        monkeypatch.setenv('PCK_GRP_BALANCE', '0')
        fr, Jr = evaluate(make, n, T, y, desc)
        monkeypatch.delenv('PCK_GRP_BALANCE')
        np.testing.assert_allclose(fb, fr, rtol=1e-12, atol=1e-14 * np.abs(fr).max())
        np.testing.assert_allclose(Jb, Jr, rtol=1e-12, atol=1e-14 * np.abs(Jr).max())
    # the bench's CH4 solve (SteadyStateSolver.solve_ode to 1e4 s): the two
    # walks' transients differ by the rounding of the rate sums only
    T = np.linspace(473.0, 573.0, 64)
    monkeypatch.setenv('PCK_GRP_BALANCE', '2')
    a = _ch4(P, inputs, 1.0, 1.0)[0].solve_batch(T=T, t_end=1e4, rtol=1e-10, atol=1e-12)
    monkeypatch.setenv('PCK_GRP_BALANCE', '0')
    b = _ch4(P, inputs, 1.0, 1.0)[0].solve_batch(T=T, t_end=1e4, rtol=1e-10, atol=1e-12)
    monkeypatch.delenv('PCK_GRP_BALANCE')
    assert np.all(a['status'] == 0) and np.all(b['status'] == 0)
    assert close(a['y'], b['y'], rtol=1e-7, floor=1e-13), np.abs(a['y'] - b['y']).max()


def test_group_screening_pass_matches_single_pass(P, inputs, monkeypatch):
    """The screening pass on the lane-group kernel (System.solve_batch with
    screen=rtol; 'auto' screens one-lane networks only): DMTM steady states
    over a T x p grid -- the rule at rtol 1e-2 first, the full solve where it
    is not accepted (group-uniform) -- report what the single pass reports:
    the same statuses, the same roots to the refinement's rounding, the same
    transient ends bitwise (mk_group.h: k_solve_grp).  The quad kernel,
    which runs the plain steady solves of this network by default, has no
    screening trip: an explicit screen runs on the 16-lane kernel
    (pck_network_group_lanes reports 16), and the single pass is pinned to
    that kernel too (PCK_GRP_QUAD_NEWTON=0) for the bitwise comparison."""
    from pycatkin_amd.classes.system import SCREEN_RTOL
    s = _dmtm(P, inputs)
    TT, pp = np.meshgrid(np.linspace(450.0, 750.0, 8), np.logspace(4.0, 6.0, 8), indexing='ij')
    kw = dict(T=TT.ravel(), p=pp.ravel(), steady=True)
    b = s.solve_batch(screen=SCREEN_RTOL, **kw)
    assert s.device().group_lanes() == 16
    monkeypatch.setenv('PCK_GRP_QUAD_NEWTON', '0')
    a = s.solve_batch(screen=None, **kw)
    monkeypatch.delenv('PCK_GRP_QUAD_NEWTON')
    assert np.array_equal(a['status'], b['status']), (a['status'], b['status'])
    ok = a['status'] == 0
    assert ok.mean() > 0.5
    ry = np.abs(b['y'][:, ok] - a['y'][:, ok]) / np.maximum(np.abs(a['y'][:, ok]), 1e-300)
    assert ry.max(initial=0.0) <= 1e-8, ry.max()
    np.testing.assert_array_equal(b['y'][:, ~ok], a['y'][:, ~ok])
    # the screened solve took fewer integrator steps (both trips counted)
    assert b['nsteps'].astype(np.int64).sum() < a['nsteps'].astype(np.int64).sum()


@pytest.mark.parametrize('which', ['ch4', 'dmtm_drc'])
def test_quad_group_kernel_matches_lane_group(P, inputs, monkeypatch, which):
    """The quad-group kernel (mk_quad.h: k_solve_q4, four lanes per condition,
    four species rows per lane, DPP broadcasts, threshold-pivoted LU) against
    the 16-lane compile-time-network group kernel (PCK_GRP_QUAD=0): the same
    statuses and, to rounding, the same states / TOFs / DRC coefficients.  The
    CH4 transient (SteadyStateSolver's rtol 1e-10 / atol 1e-12) is the
    default user of the quad kernel (R >= 2 NS); the DMTM transient DRC is
    forced onto it (PCK_GRP_QUAD=2) to cover the DRC and retry paths."""
    if which == 'ch4':
        s, _ = _ch4(P, inputs)
        net = s.device()
        kw = dict(T=np.linspace(473.0, 573.0, 256), t0=0.0, t_end=1e4, rtol=1e-10, atol=1e-12)
        run = lambda: s.solve_batch(**kw)
    else:
        s = _dmtm(P, inputs)
        net = s.device(('r5', 'r9'))
        run = lambda: s.drc_batch(('r5', 'r9'), T=np.linspace(400.0, 800.0, 64), eps=5.0e-2)
    monkeypatch.setenv('PCK_GRP_QUAD', '2')
    a = run()
    assert net.group_kernel() == 3
    monkeypatch.setenv('PCK_GRP_QUAD', '0')
    b = run()
    assert net.group_kernel() == 2
    monkeypatch.delenv('PCK_GRP_QUAD')
    np.testing.assert_array_equal(a['status'], b['status'])
    assert np.all(a['status'] == 0), np.unique(a['status'], return_counts=True)
    if which == 'ch4':
        # measured 2.3e-12 relative above 1e-12, identical step counts
        assert close(a['y'], b['y'], rtol=1e-9, floor=1e-14), np.abs(a['y'] - b['y']).max()
        return
    # transients at the input's rtol 1e-6 (measured 1.4e-6 on xi)
    for name in s.reactions:
        np.testing.assert_allclose(a[name], b[name], rtol=0, atol=1e-5)
    np.testing.assert_allclose(a['tof0'], b['tof0'], rtol=1e-6)


@pytest.mark.parametrize('n', [1, 5, 17, 33])
def test_quad_group_kernel_ragged_batches(P, inputs, monkeypatch, n):
    """Batches that do not fill a wavefront of 16 quads (and one condition
    alone): the quad kernel's tail quads exit before any cross-lane step, the
    others match the 16-lane kernel as in the full batch (CH4 transient at
    rtol 1e-8, t_end 1e2 s; the DMTM DRC on n // 4 + 1 temperatures)."""
    s, _ = _ch4(P, inputs)
    net = s.device()
    kw = dict(T=np.linspace(473.0, 573.0, n), t0=0.0, t_end=1e2, rtol=1e-8, atol=1e-12)
    monkeypatch.setenv('PCK_GRP_QUAD', '2')
    a = s.solve_batch(**kw)
    assert net.group_kernel() == 3
    monkeypatch.setenv('PCK_GRP_QUAD', '0')
    b = s.solve_batch(**kw)
    np.testing.assert_array_equal(a['status'], b['status'])
    assert np.all(a['status'] == 0), _counts(a['status'])
    assert a['y'].shape == (len(s.plan().dyn), n)
    assert close(a['y'], b['y'], rtol=1e-7, floor=1e-14), np.abs(a['y'] - b['y']).max()
    d = _dmtm(P, inputs)
    m = n // 4 + 1
    monkeypatch.setenv('PCK_GRP_QUAD', '2')
    c = d.drc_batch(('r5', 'r9'), T=np.linspace(450.0, 750.0, m), eps=5.0e-2)
    assert d.device(('r5', 'r9')).group_kernel() == 3
    monkeypatch.setenv('PCK_GRP_QUAD', '0')
    e = d.drc_batch(('r5', 'r9'), T=np.linspace(450.0, 750.0, m), eps=5.0e-2)
    monkeypatch.delenv('PCK_GRP_QUAD')
    np.testing.assert_array_equal(c['status'], e['status'])
    for name in d.reactions:
        assert c[name].shape == (m,)
        np.testing.assert_allclose(c[name], e[name], rtol=0, atol=1e-5)


def test_quad_newton_matches_lane_group_steady(P, inputs, monkeypatch):
    """Steady solves on the quad-group kernel (mk_quad.h: q_newton, the
    Newton polish with the refinement, balance test and steady rule of
    mk_group.h: grp_newton) against the 16-lane kernel
    (PCK_GRP_QUAD_NEWTON=0): DMTM steady states over a T x p grid -- the same
    statuses, the same roots to the refinement's rounding, the same TOFs."""
    s = _dmtm(P, inputs)
    net = s.device(('r5', 'r9'))
    TT, pp = np.meshgrid(np.linspace(450.0, 750.0, 16), np.logspace(4.0, 6.0, 16), indexing='ij')
    kw = dict(T=TT.ravel(), p=pp.ravel(), tof_terms=('r5', 'r9'), steady=True)
    a = s.solve_batch(**kw)
    assert net.group_kernel() == 3
    monkeypatch.setenv('PCK_GRP_QUAD_NEWTON', '0')
    b = s.solve_batch(**kw)
    assert net.group_kernel() == 2
    monkeypatch.delenv('PCK_GRP_QUAD_NEWTON')
    pairs = _counts(np.array(['%d->%d' % (u, v) for u, v in zip(b['status'], a['status'])]))
    assert np.array_equal(a['status'], b['status']), pairs
    ok = a['status'] == 0
    assert ok.mean() > 0.5, pairs
    assert close(a['y'][:, ok], b['y'][:, ok], rtol=1e-8, floor=1e-14), np.abs(a['y'] - b['y']).max()
    np.testing.assert_allclose(a['tof'][ok], b['tof'][ok], rtol=1e-8)


def test_quad_trajectories_match_lane_group(P, inputs, monkeypatch):
    """Trajectory samples (System.solve_odes / solve_batch(t_out=...)) from
    the quad kernel's dense output against the 16-lane kernel's
    (PCK_GRP_QUAD=0): DMTM over 32 temperatures, 41 log-spaced samples from
    0 to 1e4 s (and one sample past t_end by rounding) at rtol 1e-10."""
    s = _dmtm(P, inputs)
    net = s.device()
    t_out = np.concatenate([[0.0], np.logspace(-8.0, 4.0, 40), [1e4 * (1.0 + 4e-16)]])
    kw = dict(T=np.linspace(450.0, 750.0, 32), t0=0.0, t_end=1e4, rtol=1e-10, atol=1e-14, t_out=t_out)
    a = s.solve_batch(**kw)
    assert net.group_kernel() == 3
    monkeypatch.setenv('PCK_GRP_QUAD', '0')
    b = s.solve_batch(**kw)
    monkeypatch.delenv('PCK_GRP_QUAD')
    np.testing.assert_array_equal(a['status'], b['status'])
    assert np.all(np.isfinite(a['traj']))
    assert close(a['traj'], b['traj'], rtol=1e-6, floor=1e-12), np.abs(a['traj'] - b['traj']).max()
    np.testing.assert_allclose(a['traj'][-1], a['y'], rtol=1e-12, atol=1e-300)
