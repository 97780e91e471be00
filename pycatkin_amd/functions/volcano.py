"""The CO-oxidation volcano driver (examples/COOxVolcano/cooxvolcano.py) as
one batched device launch over a descriptor grid.

The reference mutates the user-defined reaction energies in a Python double
loop and calls System.activity() per grid point (cooxvolcano.py:22-47).  Here
the same assignments are made ONCE with Descriptor forms, and the grid is a
batch of conditions.
"""
from __future__ import annotations

import numpy as np

from ..energy import TSYM, Descriptor, clamp0

# standard entropies (Atkins, eV/K) -- cooxvolcano.py:13-14
SCOg = 2.0487e-3
SO2g = 2.1261e-3


def set_volcano_energies(sim_system, SCO=SCOg, SO2=SO2g):
    """cooxvolcano.py:28-44 with ECO / EO as per-condition descriptors."""
    eco, eo = Descriptor('ECO'), Descriptor('EO')
    R = sim_system.reactions
    R['CO_ads'].dErxn_user = eco                                   # (a)
    R['CO_ads'].dGrxn_user = eco + SCO * TSYM
    R['2O_ads'].dErxn_user = 2.0 * eo                              # (b)
    R['2O_ads'].dGrxn_user = 2.0 * eo + SO2 * TSYM
    EO2 = sim_system.states['sO2'].get_potential_energy()          # (c)
    R['O2_ads'].dErxn_user = EO2
    R['O2_ads'].dGrxn_user = EO2 + SO2 * TSYM
    ETS_CO_ox = sim_system.states['SRTS_ox'].get_potential_energy()  # (d)
    R['CO_ox'].dEa_fwd_user = clamp0(ETS_CO_ox - (eco + eo))
    ETS_O2_2O = sim_system.states['SRTS_O2'].get_potential_energy()  # (e)
    R['O2_2O'].dEa_fwd_user = clamp0(ETS_O2_2O - EO2)
    sim_system._plans.clear()
    return ('ECO', 'EO')


def volcano_grid(be_co, be_o):
    """Flattened (ECO, EO) pairs in activity[iCO, iO] order."""
    ECO, EO = np.meshgrid(np.asarray(be_co, float), np.asarray(be_o, float), indexing='ij')
    return ECO.ravel(), EO.ravel()


def tile_order(shape, tile=(16, 4)):
    """Permutation of a row-major (n0, n1) grid that puts each t0 x t1 patch
    (t0 * t1 = 64) on consecutive conditions: one wavefront per grid patch.

    Step counts, Newton iterations and the LU's row-swap pattern vary smoothly
    over the descriptor grid and jump across the volcano's regime boundaries.
    Lanes of a wave that share a patch take the same branches and finish
    together.  Measured on the 1024 x 1024 COOx grid (profiles/r1/tile_order):
    row-major 64-point segments 94 M solves/s, 8x8 137 M, 16x4 / 32x2 / 64x1
    ~140 M -- the swap pattern follows E_O, so narrow-in-E_O patches win.
    Ragged edges (dimensions not divisible by the patch) stay a permutation.
    """
    n0, n1 = int(shape[0]), int(shape[1])
    t0, t1 = (tile, tile) if np.ndim(tile) == 0 else (int(tile[0]), int(tile[1]))
    i, j = np.meshgrid(np.arange(n0), np.arange(n1), indexing='ij')
    key = ((i // t0) * ((n1 + t1 - 1) // t1) + (j // t1)) * (t0 * t1) + (i % t0) * t1 + (j % t1)
    return np.argsort(key.ravel(), kind='stable')


def volcano_activity(sim_system, be_co, be_o, tof_terms=('CO_ox',), steady=False, T=None, **kw):
    """activity[iCO, iO] (eV) like cooxvolcano.py:47, for the whole grid at once."""
    set_volcano_energies(sim_system)
    eco, eo = volcano_grid(be_co, be_o)
    shape = (np.size(be_co), np.size(be_o))
    perm = tile_order(shape)                # device order: 16x4 patches per wave
    T = sim_system.params['temperature'] if T is None else T
    r = sim_system.solve_batch(T=np.full(eco.size, float(T)), desc={'ECO': eco[perm], 'EO': eo[perm]},
                               tof_terms=tuple(tof_terms), steady=steady, activity=True, **kw)
    inv = np.empty_like(perm)
    inv[perm] = np.arange(perm.size)
    for key, v in list(r.items()):          # back to activity[iCO, iO] order
        if isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[-1] == perm.size:
            r[key] = v[..., inv]
        elif hasattr(v, 'device') and v.ndim >= 1 and v.shape[-1] == perm.size:    # to_numpy=False
            import torch
            r[key] = v[..., torch.from_numpy(inv).to(v.device)]
    return r['tof'].reshape(shape), r
