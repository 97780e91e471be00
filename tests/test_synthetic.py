"""Synthetic stress network (pycatkin_amd.functions.synthetic): structure and
plan on the host (no device)."""
import numpy as np

from pycatkin_amd.functions.synthetic import synthetic_energies, synthetic_network, synthetic_system


def test_network_shape_and_site_balance():
    net = synthetic_network()
    assert len(net['adsorbates']) == 49 and len(net['reactions']) == 150
    used = set()
    for kind, reac, prod in net['reactions']:
        used.update(reac + prod)
        sites = lambda side: sum(1 for s in side if s == 's' or s.startswith('A'))  # noqa: E731
        if kind == 'surf':
            assert sites(reac) == sites(prod)                  # every surface step conserves sites
        else:
            assert sites(reac) == sites(prod)                  # gas + n s -> n adsorbates
    assert set(net['adsorbates']) <= used
    assert synthetic_network(seed=0)['E0'].tolist() == net['E0'].tolist()   # deterministic


def test_plan_dimensions_and_conservation():
    sim, net = synthetic_system()
    plan = sim.plan(('R0',))
    assert len(plan.dyn) == 50 and len(plan.fix) == 6 and len(plan.reactions) == 150
    C = plan.conservation
    assert C.shape[0] == 1
    np.testing.assert_allclose(C[0] / C[0][np.nonzero(C[0])[0][0]], np.ones(50))


def test_ts_energies_are_above_both_ends():
    net = synthetic_network()
    E, ts = synthetic_energies(net, np.array([0.3, -0.2, 0.1, 0.4]))
    for j, (kind, reac, prod) in enumerate(net['reactions']):
        if kind == 'surf':
            e = ts['TS%d' % j]
            assert e >= sum(E[s] for s in reac) + 0.4 - 1e-12
            assert e >= sum(E[s] for s in prod) + 0.4 - 1e-12


def test_presets_accept_every_reported_steady_status():
    """presets.run_temperatures / run_parameters accept statuses 0 (steady
    state reached), 4 (transient end reported) and 5 (the same after a failed
    retry pass) and flag only the integrator failures 1-3."""
    from pycatkin_amd.functions.presets import _failed
    st = np.array([0, 4, 5, 1, 2, 3, 0, 5], np.int32)
    assert _failed(st).tolist() == [3, 4, 5]
    assert _failed(np.array([0, 4, 5])).size == 0
