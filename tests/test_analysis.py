"""Descriptor-grid post-processing (pycatkin/functions/analysis.py:27-266)
and the batched C x O grid (pycatkin_amd/functions/analysis.py).

CPU: the host logic of check_convergence / average_neighborhood / the maps,
with the reference's quirks (analysis.py:64, :116), and the deep copy of a
System that already holds plans.
GPU: solve_descriptor_grid over a 4 x 4 E_C x E_O grid of test/CH4_input.json
at 523 K against tests/golden/ch4_grid_fixture.npz (make_ch4_grid_fixture.py:
the oracle at lsoda 1e-13 / 1e-20) and against the reference's per-point loop
run on the device (one System with constant energies per point); then
check_convergence's printed diagnosis against the same per-point loop."""
import copy
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GRID = os.path.join(HERE, 'golden', 'ch4_grid_fixture.npz')


def _A():
    from pycatkin_amd.functions import analysis
    return analysis


def _log(success, n=4, m=4, ns=3):
    from pycatkin_amd import SteadyStateResults
    return {(i, j): SteadyStateResults(np.full(ns, 10.0 * i + j), bool(success[i][j]))
            for i in range(n) for j in range(m)}


# ---------------------------------------------------------------- CPU (no GPU)
def test_average_neighborhood_first_point_only():
    """analysis.py:94-116: the return sits inside the loop -- only the first
    misfit with >= 2 worked neighbours is averaged."""
    A = _A()
    ok = [[1, 1, 1, 1], [1, 0, 1, 1], [1, 1, 0, 1], [1, 1, 1, 1]]
    log = _log(ok)
    mis = [k for k, v in log.items() if not v.success]
    wk = [k for k, v in log.items() if v.success]
    new = A.average_neighborhood(mis, wk, log)
    nb = [(0, 0), (0, 1), (0, 2), (1, 0), (1, 2), (2, 0), (2, 1)]       # (2, 2) failed
    np.testing.assert_array_equal(new[(1, 1)].x, np.mean([log[k].x for k in nb], axis=0))
    assert new[(1, 1)].success is False
    np.testing.assert_array_equal(new[(2, 2)].x, log[(2, 2)].x)          # not reached
    assert log[(1, 1)].x[0] == 11.0                                       # the input log is untouched
    allp = A.average_neighborhood(mis, wk, log, all_points=True)
    nb2 = [(1, 2), (1, 3), (2, 1), (2, 3), (3, 1), (3, 2), (3, 3)]
    np.testing.assert_array_equal(allp[(2, 2)].x, np.mean([log[k].x for k in nb2], axis=0))


def test_average_neighborhood_skips_and_returns_none(capsys):
    """Fewer than 2 worked neighbours: a message and the point is skipped;
    nothing averaged -> None (the reference falls off the loop)."""
    A = _A()
    ok = [[0, 0, 1], [0, 0, 0], [1, 0, 0]]
    log = _log(ok, 3, 3)
    mis = [k for k, v in log.items() if not v.success]
    wk = [k for k, v in log.items() if v.success]
    assert A.average_neighborhood([(0, 0)], wk, log) is None
    assert 'FAILED FINDING SURROUNDINGS FOR (0, 0)' in capsys.readouterr().out
    assert A.average_neighborhood([], wk, log) is None
    new = A.average_neighborhood(mis, wk, log, all_points=True)
    np.testing.assert_array_equal(new[(1, 1)].x, np.mean([log[(0, 2)].x, log[(2, 0)].x], axis=0))


def test_check_convergence_partition_without_failures():
    """analysis.py:47-76: all points converged -> no rebuild, no device call."""
    A = _A()
    log = _log([[1, 1], [1, 1]], 2, 2)
    mis, wk = A.check_convergence(log, object(), [0.0, 1.0], [0.0, 1.0])
    assert mis == [] and wk == list(log)


def test_maps_and_scores():
    """analysis.py:131-136 and 206-235: the convergence map and the heatmap
    scores (log|v|, clipped at -25; colour range rounded to 2 decimals)."""
    A = _A()
    wm = A.convergence_map([0, 1, 2], [0, 1], [(1, 0), (2, 1)])
    np.testing.assert_array_equal(wm, [[1, 1], [0, 1], [1, 0]])
    res = {(i, j): {'CH3OH': 10.0 ** (-5 * (i + j)), 'CO2': 2.0} for i in range(3) for j in range(2)}
    sc, (vmin, vmax) = A.heatmap_scores(['CH3OH', 'CO2'], res, [0, 1, 2], [0, 1])
    assert sc.shape == (2, 3, 2)
    assert sc[0, 2, 1] == -25.0 and sc[0, 1, 1] == pytest.approx(np.log(1e-10))
    assert vmin == -25.0 and vmax == round(np.log(2.0), 2)
    with pytest.warns(UserWarning):
        sc2, _ = A.make_heatmap('CO2', res, [0, 1, 2], [0, 1], use_log=False)
    assert np.all(sc2 == 2.0)


def test_deepcopy_drops_plans(inputs):
    """A deep copy of a System with compiled plans (analysis.py:40,
    butadiene_mkm.py:47) starts with an empty plan cache; the descriptor
    forms compile to a plan over ('EC', 'EO')."""
    import pycatkin_amd as P
    s = P.read_from_input_file(os.path.join(inputs, 'CH4', 'input.json'), formulation='patched')
    for r, st in (('C_ads', 'sC'), ('O_ads', 'sO')):
        s.reactions[r].dErxn_user = 1.0
        s.states[st].Gelec = 1.0
    s.plan()
    assert s._plans
    c = copy.deepcopy(s)
    assert c._plans == {} and s._plans
    assert _A().set_descriptor_energies(c) == ('EC', 'EO')
    assert c.plan().descriptors == ['EC', 'EO']
    assert s.plan().descriptors == []


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope='module')
def P():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    import pycatkin_amd
    return pycatkin_amd


def close(a, b, rtol=1e-6, floor=1e-12):
    a, b = np.asarray(a), np.asarray(b)
    return np.all(np.abs(a - b) <= rtol * np.abs(b) + floor)


def _ch4_point(P, inputs, EC, EO):
    s = P.read_from_input_file(os.path.join(inputs, 'CH4', 'input.json'), formulation='patched')
    s.reactions['C_ads'].dErxn_user = EC
    s.reactions['O_ads'].dErxn_user = EO
    s.states['sC'].Gelec = EC
    s.states['sO'].Gelec = EO
    s.T = 523.0
    s.build()
    return s


@pytest.fixture(scope='module')
def grid(P, inputs):
    fx = dict(np.load(GRID))
    s = _ch4_point(P, inputs, 1.0, 1.0)
    log = _A().solve_descriptor_grid(s, fx['C_range'], fx['O_range'], T=float(fx['T']))
    return s, fx, log


@pytest.mark.gpu
def test_descriptor_grid_vs_fixture(P, inputs, grid):
    """Every grid point the oracle integrates to 1e4 s: the batched device
    transient against lsoda at 1e-13 / 1e-20 at 1e-6 relative, with an
    absolute floor of 10 x the solve's atol 1e-12 (a component below ~1e-6
    is held to atol per step, not to rtol; its global error at 1e4 s is a few
    atol: 1.2e-12 at E_C = 1.0, E_O = 0.6) -- or, where the transient end is
    ill-conditioned, no further off than scipy's lsoda at the solve's own
    tolerances lands (`lsoda_err` in the fixture; E_C = 1.5, E_O = 0.6 has
    not settled by 1e4 s, max|f| 5.6e-9: lsoda at 1e-10 is 7.8e-6 off, BDF
    fails, the device 4.7e-7).  The oracle's surface order is index_map's."""
    s, fx, log = grid
    names = [str(x) for x in fx['names']]
    assert names == s._surface_order()
    excess = {}
    for (i, j), v in log.items():
        if fx['status'][i, j] != 0:
            continue
        d = np.abs(v.x - fx['y'][i, j])
        bound = max(1e-11, np.nan_to_num(fx['lsoda_err'][i, j], nan=0.0))
        excess[(i, j)] = (float(np.max(d - 1e-6 * np.abs(fx['y'][i, j])) / bound), float(np.max(d)))
    assert len(excess) == int((fx['status'] == 0).sum()) == 15
    worst = sorted(excess.items(), key=lambda kv: -kv[1][0])
    assert worst[0][1][0] <= 1.0, str(worst[:6])
    # the settled points (max|f| < 1e-11) are held to the plain bound
    settled = [(i, j) for (i, j) in excess if fx['max_f'][i, j] < 1e-11]
    assert len(settled) >= 7
    for k in settled:
        assert close(log[k].x, fx['y'][k], rtol=1e-6, floor=1e-11), (k, excess[k])


@pytest.mark.gpu
def test_descriptor_grid_matches_per_point_loop(P, inputs, grid, capsys):
    """The reference's loop, per point (descriptor energies as constants,
    build(), SteadyStateSolver.solve_ode(), solver.py:374-418) on the device:
    the same success flags, x within 1e-9 (one launch with descriptor forms
    against 16 launches with constant energies).  check_convergence then
    prints, for the failed points, what analysis.py:47-73 prints from the
    per-point rebuild (composition initial_system[len(gas):] ++ x)."""
    s, fx, log = grid
    A = _A()
    C, Oe = fx['C_range'], fx['O_range']
    ref_lines = []
    for (i, j), v in log.items():
        sp = _ch4_point(P, inputs, float(C[i]), float(Oe[j]))
        r = P.SteadyStateSolver(sp).solve_ode(tmax=1e4)
        assert r.success == v.success, ((i, j), r.success, v.success)
        if fx['status'][i, j] == 0:
            assert close(v.x, r.x, rtol=1e-9, floor=1e-20), ((i, j), np.abs(v.x - r.x).max())
        if not v.success:
            y = np.concatenate((sp.initial_system[len(sp.gas_indices):], v.x))
            surf = [sum(y[list(idx)]) for idx in sp.coverage_map.values()]
            if np.any(np.abs(np.array(surf) - 1) > 0.05):
                ref_lines.append(f"{(i, j)} : SURF SUM FAILED: {' , '.join(str(x)[:8] for x in surf)}")
            elif np.any(np.abs(sp.get_dydt(y)) > 1e-6):
                ref_lines.append(f"{(i, j)} : RATE FAILED: {max(sp.get_dydt(y)):.4e}")
    capsys.readouterr()
    mis, wk = A.check_convergence(log, s, C, Oe)
    out = capsys.readouterr().out.strip().splitlines()
    assert mis == [k for k, v in log.items() if not v.success] and len(mis) >= 3
    assert wk == [k for k, v in log.items() if v.success]
    assert out == ref_lines
    # the failed points include the oracle's non-converged corners
    for k in ((0, 2), (0, 3), (1, 3)):
        assert k in mis
    new = A.average_neighborhood(mis, wk, log, all_points=True)
    for k in mis:
        nb = [(k[0] + a, k[1] + b) for a in (-1, 0, 1) for b in (-1, 0, 1) if (a, b) != (0, 0) and (k[0] + a, k[1] + b) in wk]
        if len(nb) >= 2:
            np.testing.assert_allclose(new[k].x, np.mean([log[q].x for q in nb], axis=0), rtol=1e-15)


@pytest.mark.gpu
def test_convergence_batch_matches_test_convergence(P, inputs, grid):
    """SteadyStateSolver.test_convergence_batch (two launches, batched
    eigenvalues) against test_convergence per column (solver.py:69-120), at
    the grid's own states with per-point descriptor energies and at one
    temperature sweep."""
    s, fx, log = grid
    for (i, j), v in list(log.items())[::3]:
        sp = _ch4_point(P, inputs, float(fx['C_range'][i]), float(fx['O_range'][j]))
        sol = P.SteadyStateSolver(sp)
        assert sol.test_convergence_batch(v.x[:, None])[0] == sol.test_convergence(v.x)
    sp = _ch4_point(P, inputs, 1.0, 1.0)
    sol = P.SteadyStateSolver(sp)
    T = np.array([480.0, 523.0, 560.0])
    Y, _ = sol.solve_ode_batch(T=T)
    ok = sol.test_convergence_batch(Y, T=T)
    for c in range(T.size):
        sp.T = float(T[c])
        assert ok[c] == sol.test_convergence(Y[:, c]), c
