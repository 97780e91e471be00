"""Synthetic stress network (BASELINE.json configs[4]): 50 dynamic species /
150 reactions on one site type, with random descriptor-dependent energies.

Not a reference example -- the reference has no network this size; this is
the stiffness / LDS-capacity stress case of the batched solver.  It is built
from the same classes as every reference input (State, Reaction with
transition states, InfiniteDilutionReactor), so it exercises the same
thermochemistry and the same mass-action formulation (old_system.py):

  * 6 gases (fixed partial pressures; translational + rotational free
    energies from mass / inertia / symmetry number, state.py:320-365),
  * the free site 's' and 49 adsorbates A0..A48 (electronic energy affine in
    the per-condition descriptors D0..D{n_desc-1}),
  * 6 molecular + 4 dissociative adsorptions (collision theory, classic
    reverse rate), and surface steps (association X+Y <-> Z+s, isomerisation
    X <-> Y, exchange X+Y <-> Z+W) through transition states with
    E_TS = E_IS + max(E_FS - E_IS, 0) + beta  (Arrhenius, reaction.py:121).

`synthetic_network` returns the structure and coefficients as plain data;
`synthetic_system` turns it into a System whose energies are LinearForms of
the descriptors, so one plan serves a batch of random-energy conditions.
"""
from __future__ import annotations

import numpy as np

GASES = [  # name, mass (amu), sigma, principal moments (amu A^2), pressure (bar)
    ('G0', 28.010, 1, (0.0, 8.7, 8.7), 0.20),
    ('G1', 31.998, 2, (0.0, 11.7, 11.7), 0.10),
    ('G2', 44.009, 2, (0.0, 43.1, 43.1), 0.05),
    ('G3', 16.043, 12, (3.2, 3.2, 3.2), 0.30),
    ('G4', 2.016, 2, (0.0, 0.28, 0.28), 0.20),
    ('G5', 18.015, 2, (0.6, 1.2, 1.8), 0.15),
]


def synthetic_network(n_species=50, n_reactions=150, n_desc=4, seed=0):
    """Structure + energy coefficients of the synthetic network (plain data).

    Returns dict(gases, adsorbates, reactions, E0, Ed, beta, n_desc) where
    reactions[j] = (kind, reactants, products) with kind 'ads' or 'surf',
    adsorbate energy E_a(D) = E0[a] + Ed[a] . D, and beta[j] is the intrinsic
    barrier of surface step j (eV)."""
    rng = np.random.default_rng(seed)
    n_ads = n_species - 1
    ads = ['A%d' % i for i in range(n_ads)]
    gas = [g[0] for g in GASES]
    rx = []
    for g in range(len(gas)):                                   # molecular adsorption
        rx.append(('ads', [gas[g], 's'], [ads[g]]))
    for g in range(4):                                          # dissociative adsorption
        i, j = rng.choice(np.arange(6, n_ads), 2, replace=False)
        rx.append(('ads', [gas[g], 's', 's'], [ads[i], ads[j]]))
    # connect every adsorbate: species k is made from two earlier ones or one earlier one
    for k in range(6, n_ads):
        if rng.random() < 0.5:
            i, j = rng.choice(k, 2, replace=False)
            rx.append(('surf', [ads[i], ads[j]], [ads[k], 's']))
        else:
            i = int(rng.integers(k))
            rx.append(('surf', [ads[i]], [ads[k]]))
    while len(rx) < n_reactions:
        kind = rng.integers(3)
        if kind == 0:
            i, j, k = rng.choice(n_ads, 3, replace=False)
            rx.append(('surf', [ads[i], ads[j]], [ads[k], 's']))
        elif kind == 1:
            i, j = rng.choice(n_ads, 2, replace=False)
            rx.append(('surf', [ads[i]], [ads[j]]))
        else:
            i, j, k, l = rng.choice(n_ads, 4, replace=False)
            rx.append(('surf', [ads[i], ads[j]], [ads[k], ads[l]]))
    rx = rx[:n_reactions]
    E0 = np.empty(n_ads)
    E0[:6] = rng.uniform(-1.6, -0.8, 6)                         # adsorbed gases: ~ -1 eV vs. the gas
    E0[6:] = rng.uniform(-1.2, 0.2, n_ads - 6)
    Ed = np.zeros((n_ads, n_desc))
    for a in range(n_ads):                                      # 1-2 descriptors per adsorbate
        for k in rng.choice(n_desc, int(rng.integers(1, 3)), replace=False):
            Ed[a, k] = rng.uniform(0.3, 1.0)
    beta = rng.uniform(0.4, 1.1, len(rx))
    return dict(gases=GASES, adsorbates=ads, reactions=rx, E0=E0, Ed=Ed, beta=beta, n_desc=n_desc)


def synthetic_system(net=None, T=500.0, p=1.0e5, t_end=1.0e4, rtol=1e-8, atol=1e-10, **kw):
    """System (classic formulation, InfiniteDilutionReactor) for the network;
    descriptors 'D0'.. are per-condition inputs of solve_batch(desc=...)."""
    from ..classes.reaction import Reaction
    from ..classes.reactor import InfiniteDilutionReactor
    from ..classes.state import State
    from ..classes.system import System
    from ..energy import Descriptor, clamp0
    net = net or synthetic_network(**kw)
    D = [Descriptor('D%d' % k) for k in range(net['n_desc'])]
    start = {g[0]: g[4] for g in net['gases']}
    start['s'] = 1.0
    sim = System(times=[0.0, t_end], start_state=start, T=T, p=p, rtol=rtol, atol=atol)
    for name, mass, sigma, inertia, _ in net['gases']:
        sim.add_state(State(state_type='gas', name=name, mass=mass, sigma=sigma, inertia=list(inertia), Gelec=0.0))
    sim.add_state(State(state_type='surface', name='s', Gelec=0.0))
    E = {}
    for a, name in enumerate(net['adsorbates']):
        e = float(net['E0'][a])
        for k in range(net['n_desc']):
            if net['Ed'][a, k] != 0.0:
                e = e + float(net['Ed'][a, k]) * D[k]
        E[name] = e
        sim.add_state(State(state_type='adsorbate', name=name, Gelec=e))
    E['s'] = 0.0
    st = sim.states
    for j, (kind, reac, prod) in enumerate(net['reactions']):
        name = 'R%d' % j
        if kind == 'ads':
            sim.add_reaction(Reaction(name=name, reac_type='adsorption', reactants=[st[s] for s in reac],
                                      products=[st[s] for s in prod], area=1.0e-19))
            continue
        eis = sum((E[s] for s in reac), 0.0)
        efs = sum((E[s] for s in prod), 0.0)
        ets = eis + clamp0(efs - eis) + float(net['beta'][j])
        ts = State(state_type='TS', name='TS%d' % j, Gelec=ets)
        sim.add_state(ts)
        sim.add_reaction(Reaction(name=name, reac_type='Arrhenius', reactants=[st[s] for s in reac],
                                  products=[st[s] for s in prod], TS=[ts], area=1.0e-19))
    sim.add_reactor(InfiniteDilutionReactor())
    sim.names_to_indices()
    return sim, net


def synthetic_energies(net, desc):
    """Numeric adsorbate / TS electronic energies at one descriptor vector
    (eV) -- the same affine model, for building a CPU check of one condition."""
    desc = np.asarray(desc, float)
    E = {name: float(net['E0'][a] + net['Ed'][a] @ desc) for a, name in enumerate(net['adsorbates'])}
    E['s'] = 0.0
    ts = {}
    for j, (kind, reac, prod) in enumerate(net['reactions']):
        if kind == 'surf':
            eis = sum(E[s] for s in reac)
            efs = sum(E[s] for s in prod)
            ts['TS%d' % j] = eis + max(efs - eis, 0.0) + float(net['beta'][j])
    return E, ts
