"""Reactor classes with the reference's constructors (pycatkin/classes/reactor.py).

On the device a reactor is three per-species coefficients of the dynamic
rows: rowscale = rs0 + rs_T*T, a flow rate and a concentration factor
(pycatkin_amd/network.py builds them).  These classes only carry the inputs.
"""
from ..constants.physical_constants import bartoPa, kB


class Reactor:
    """reactor.py:8-86"""

    def __init__(self, name='reactor', volume=None, catalyst_area=None, residence_time=None, flow_rate=None,
                 path_to_pickle=None):
        if path_to_pickle:
            raise NotImplementedError('pickled reactors are not loaded (no unpickling of external files)')
        self.name = name
        self.volume = volume
        self.catalyst_area = catalyst_area
        self.residence_time = residence_time
        self.flow_rate = flow_rate
        self.scaling = None
        self.is_adsorbate = None
        self.is_gas = None
        self.dynamic_indices = None

    def set_scaling(self, T):
        """reactor.py:34-41"""
        self.scaling = kB * T * self.catalyst_area / self.volume

    def set_indices(self, is_adsorbate, is_gas):
        self.is_adsorbate = list(is_adsorbate)
        self.is_gas = list(is_gas)

    def get_dynamic_indices(self, adsorbate_indices, gas_indices):
        self.dynamic_indices = list(adsorbate_indices)
        return self.dynamic_indices

    # device coefficients for a dynamic species: (rowscale0, rowscale_T, flow_rate)
    def row_coefficients(self, is_adsorbate):
        return (1.0, 0.0, 0.0) if is_adsorbate else (0.0, 0.0, 0.0)


class InfiniteDilutionReactor(Reactor):
    """reactor.py:89-122: gas pressures are boundary conditions."""


class CSTReactor(Reactor):
    """reactor.py:125-189: gas rows scaled by kB*T*A/V/bartoPa plus flow."""

    def __init__(self, name='reactor', volume=None, catalyst_area=None, residence_time=None, flow_rate=None):
        super().__init__(residence_time=residence_time, flow_rate=flow_rate, volume=volume,
                         catalyst_area=catalyst_area, name=name)
        if self.residence_time is None:
            assert self.flow_rate is not None and self.volume is not None
            self.residence_time = self.volume / self.flow_rate

    def get_dynamic_indices(self, adsorbate_indices, gas_indices):
        self.dynamic_indices = list(adsorbate_indices) + list(gas_indices)
        return self.dynamic_indices

    def row_coefficients(self, is_adsorbate):
        if is_adsorbate:
            return (1.0, 0.0, 0.0)
        return (0.0, kB * self.catalyst_area / self.volume / bartoPa, 1.0 / self.residence_time)
