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


def volcano_activity(sim_system, be_co, be_o, tof_terms=('CO_ox',), steady=False, T=None, **kw):
    """activity[iCO, iO] (eV) like cooxvolcano.py:47, for the whole grid at once."""
    set_volcano_energies(sim_system)
    eco, eo = volcano_grid(be_co, be_o)
    T = sim_system.params['temperature'] if T is None else T
    r = sim_system.solve_batch(T=np.full(eco.size, float(T)), desc={'ECO': eco, 'EO': eo},
                               tof_terms=tuple(tof_terms), steady=steady, activity=True, **kw)
    shape = (np.size(be_co), np.size(be_o))
    return r['tof'].reshape(shape), r
