"""Random stiff networks on every group kernel: the synthetic generator
(pycatkin_amd/functions/synthetic.py, the BASELINE configs[4] family) at 40
species / 120 reactions (64-lane kernel, its Newton polish included), 24 /
72 (32-lane) and 12 / 36 (quad), 64
random-descriptor conditions each, steady-state rule to t_end = 1e8 s,
against tests/golden/synthetic_sizes_fixture.npz (make_synthetic_sizes_fixture.py:
the oracle's steady rule, lsoda at rtol 1e-11 / atol 1e-20).

Bounds as test_synthetic_fixture_parity: where both sides report the steady
state reached, coverages and the TOF of R0 at 1e-6 relative (coverage floor
1e-20, the oracle's atol); where neither does (the transient end), 1e-5 --
the two integrators' accuracy on a state still moving at t_end; the
classification may differ only where the oracle's criterion lies within a
factor 2 of ROOT_DIST."""
import os
import sys

import numpy as np
import pytest

from oracle import mk_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, 'golden'))
from make_synthetic_sizes_fixture import NETS, ROOT_DIST, SEED_NET, STEADY_ATOL, T, T_END  # noqa: E402

FIXTURE = os.path.join(HERE, 'golden', 'synthetic_sizes_fixture.npz')


@pytest.fixture(scope='module')
def fx():
    return dict(np.load(FIXTURE))


def _net(key):
    from pycatkin_amd.functions.synthetic import synthetic_network
    ns, nr = NETS[key]
    return synthetic_network(n_species=ns, n_reactions=nr, seed=SEED_NET)


# ---------------------------------------------------------------- CPU (no GPU)
@pytest.mark.parametrize('key', sorted(NETS))
def test_synthetic_sizes_fixture_reproduces(fx, key):
    """The fixture's oracle rows re-run here (two conditions) and the
    product's plan over the same species: the fixture is what the oracle
    computes for the network the product builds."""
    from _synth import spec_of
    from pycatkin_amd.functions.synthetic import synthetic_system
    net = _net(key)
    sim, _ = synthetic_system(net, t_end=T_END)
    plan = sim.plan(('R0',))
    assert sorted(plan.dyn) == sorted(str(x) for x in fx[key + '_dyn'])
    assert len(plan.dyn) == NETS[key][0]
    # (syn40: the oracle's transient exceeds its budget at 2 of 64 conditions)
    assert fx[key + '_ok'].sum() >= 62
    for k in [k for k in range(8) if fx[key + '_ok'][k]][:2]:
        m = O.ClassicModel(spec_of(net, fx['desc'][k], float(T)), T=float(T))
        r = O.steady_rule(m, dist=ROOT_DIST, dist_atol=STEADY_ATOL, budget=400000, t_end=T_END)
        assert bool(r['regular']) == bool(fx[key + '_regular'][k])
        np.testing.assert_allclose(r['y'][m.dyn], fx[key + '_y'][k], rtol=1e-9, atol=1e-25)


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope='module')
def P():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    import pycatkin_amd
    return pycatkin_amd


@pytest.mark.gpu
@pytest.mark.parametrize('key,lanes', [('syn40', 64), ('syn24', 32), ('syn12', 4)])
def test_synthetic_sizes_steady_vs_oracle(P, fx, key, lanes):
    """One steady solve of the 64 conditions (System.solve_batch(steady=True),
    the default STEADY_TRANSIENT tolerances) on the kernel the network's size
    selects -- asserted through pck_network_group_lanes -- against the
    oracle's rule."""
    from pycatkin_amd.functions.synthetic import synthetic_system
    sim, _ = synthetic_system(_net(key), t_end=T_END)
    plan = sim.plan(('R0',))
    D = fx['desc']
    n = D.shape[0]
    r = sim.solve_batch(T=np.full(n, float(T)), desc={'D%d' % k: D[:, k] for k in range(4)}, tof_terms=('R0',),
                        steady=True)
    assert sim.device(('R0',)).group_lanes() == lanes
    st = r['status']
    assert set(np.unique(st).tolist()) <= {0, 4}, np.unique(st, return_counts=True)
    names = [str(x) for x in fx[key + '_dyn']]
    y = r['y'][[plan.dyn.index(nm) for nm in names]].T
    ok = fx[key + '_ok']                    # conditions the oracle answered
    reg, dev = fx[key + '_regular'], st == 0
    flips = np.nonzero((dev != reg) & ok)[0]
    for f in flips:
        assert 0.5 * ROOT_DIST <= fx[key + '_crit'][f] <= 2.0 * ROOT_DIST, (key, int(f), st[f], fx[key + '_crit'][f])
    assert len(flips) <= 2, flips
    ref = fx[key + '_y']
    both = dev & reg & ok
    neither = ~dev & ~reg & ok
    assert both.sum() >= 50, both.sum()
    err = np.abs(y - ref) / (np.abs(ref) + 1e-300)
    ok_root = np.abs(y - ref) <= 1e-6 * np.abs(ref) + 1e-20
    assert np.all(ok_root[both]), (key, np.nonzero(both & ~np.all(ok_root, axis=1))[0][:5], err[both].max())
    ok_tr = np.abs(y - ref) <= 1e-5 * np.abs(ref) + 1e-20
    assert np.all(ok_tr[neither]), (key, np.nonzero(neither & ~np.all(ok_tr, axis=1))[0][:5])
    tof, tref = r['tof'], fx[key + '_tof']
    assert np.all(np.abs(tof[both] - tref[both]) <= 1e-6 * np.abs(tref[both])), \
        (key, np.max(np.abs(tof[both] - tref[both]) / np.abs(tref[both])))
    # the site balance holds on every condition
    C = plan.conservation
    np.testing.assert_allclose(C @ r['y'], np.repeat((C @ plan.y0_default)[:, None], n, axis=1), rtol=0, atol=1e-10)


@pytest.mark.gpu
def test_synthetic_drc_on_32_lane_groups(P, fx):
    """The steady degree of rate control (old_system.py:490-515,
    System.drc_batch(steady=True): 2 R + 1 = 145 group solves per condition)
    of the 24-species network at two conditions, against
    tests/golden/synthetic_drc_fixture.npz (make_synthetic_drc_fixture.py: the
    oracle's steady rule for every perturbed system) at 1e-6 on every xi;
    the sum rule (sum_j xi_j = 1) holds to 1e-6."""
    from pycatkin_amd.functions.synthetic import synthetic_system
    dfx = dict(np.load(os.path.join(HERE, 'golden', 'synthetic_drc_fixture.npz')))
    assert dfx['all_regular'].all()
    sim, _ = synthetic_system(_net('syn24'), t_end=T_END)
    plan = sim.plan(('R0',))
    rows = dfx['rows']
    D = fx['desc'][rows]
    out = sim.drc_batch(('R0',), T=np.full(rows.size, float(T)), desc={'D%d' % k: D[:, k] for k in range(4)},
                        eps=float(dfx['eps']), steady=True)
    assert sim.device(('R0',)).group_lanes() == 32
    assert np.all(out['status'] == 0), out['status']
    np.testing.assert_allclose(out['tof0'], dfx['tof0'], rtol=1e-6)
    xi = np.array([out['R%d' % j] for j in range(len(plan.reactions))]).T
    err = np.abs(xi - dfx['xi'])
    assert err.max() <= 1e-6, (err.max(), np.unravel_index(np.argmax(err), err.shape))
    np.testing.assert_allclose(xi.sum(axis=1), 1.0, atol=1e-6)


@pytest.mark.gpu
def test_synthetic_trajectory_on_32_lane_groups(P, fx):
    """Trajectory samples (solve_batch(t_out=...), the RODAS4P dense output
    of the 32-lane kernel) of the 24-species network at four conditions, 31
    log-spaced samples 0 .. 1e4 s at rtol 1e-10 / atol 1e-14, against
    tests/golden/synthetic_traj_fixture.npz (the oracle's model, LSODA at
    1e-12 / 1e-20 with t_eval; BDF agrees to 2.5e-8) at 1e-6 relative with
    a 1e-12 floor."""
    from pycatkin_amd.functions.synthetic import synthetic_system
    tfx = dict(np.load(os.path.join(HERE, 'golden', 'synthetic_traj_fixture.npz')))
    sim, _ = synthetic_system(_net('syn24'))
    plan = sim.plan()
    rows = tfx['rows']
    D = fx['desc'][rows]
    r = sim.solve_batch(T=np.full(rows.size, float(T)), desc={'D%d' % k: D[:, k] for k in range(4)}, t0=0.0,
                        t_end=float(tfx['t_out'][-1]), rtol=1e-10, atol=1e-14, t_out=tfx['t_out'])
    assert sim.device().group_lanes() == 32
    assert np.all(r['status'] == 0), r['status']
    pos = [plan.dyn.index(str(nm)) for nm in tfx['dyn']]
    traj = r['traj'][:, pos, :]                          # [n_out, NS, n]
    ref = np.transpose(tfx['traj'], (1, 2, 0))           # [n_out, NS, n]
    bad = ~(np.abs(traj - ref) <= 1e-6 * np.abs(ref) + 1e-12)
    assert not bad.any(), (np.argwhere(bad)[:6].tolist(), np.abs(traj - ref).max())
