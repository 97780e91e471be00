"""Reaction classes with the reference's constructors
(pycatkin/classes/reaction.py).  Energies are LinearForms in eV; the device
turns them into J/mol (x eVtokJ*1e3) and into rate constants per condition.
"""
from __future__ import annotations

from ..energy import as_form, tkeyed


def _lin(x):
    """User energies may be floats, LinearForms (descriptor expressions) or
    dicts keyed by temperature (reaction.py:228-262: ``self.dErxn_user[T]``).
    A dict becomes a per-condition input filled from each condition's T at
    solve time (energy.tkeyed; a temperature missing from the dict raises
    KeyError, as the reference's lookup does)."""
    if isinstance(x, dict):
        return tkeyed(x)
    return as_form(x)


class Reaction:
    """Mirror of pycatkin.classes.reaction.Reaction (reaction.py:6-200)."""

    def __init__(self, name='reaction', reac_type=None, reversible=True, reactants=None, products=None,
                 TS=None, area=1.0e-19, scaling=1.0, path_to_pickle=None):
        if path_to_pickle:
            raise NotImplementedError('pickled reactions are not loaded (no unpickling of external files)')
        self.reac_type = reac_type
        self.reversible = reversible
        self.reactants = reactants
        self.products = products
        self.TS = TS
        self.area = area
        self.name = name
        self.scaling = scaling
        self.kfwd = None
        self.krev = None
        self.Keq = None
        self.dGrxn = self.dGa_fwd = self.dGa_rev = None
        self.dErxn = self.dEa_fwd = self.dEa_rev = None

    def _source(self):
        return self

    def energy_forms(self):
        """calc_reaction_energy (reaction.py:43-69) -> {key: LinearForm (eV) or None}."""
        src = self._source()
        out = dict(dGrxn=None, dErxn=None, dGa_fwd=None, dEa_fwd=None, dGa_rev=None, dEa_rev=None)
        Greac = sum((s.free_form() for s in src.reactants), as_form(0.0))
        Ereac = sum((s.elec_form() for s in src.reactants), as_form(0.0))
        Gprod = Eprod = None
        if src.reversible:
            Gprod = sum((s.free_form() for s in src.products), as_form(0.0))
            Eprod = sum((s.elec_form() for s in src.products), as_form(0.0))
            out['dGrxn'] = Gprod - Greac
            out['dErxn'] = Eprod - Ereac
        if src.TS is not None:
            GTS = sum((s.free_form() for s in src.TS), as_form(0.0))
            ETS = sum((s.elec_form() for s in src.TS), as_form(0.0))
            out['dGa_fwd'] = GTS - Greac
            out['dEa_fwd'] = ETS - Ereac
            if src.reversible:
                out['dGa_rev'] = GTS - Gprod
                out['dEa_rev'] = ETS - Eprod
        else:
            z = as_form(0.0)
            out.update(dGa_fwd=z, dGa_rev=z, dEa_fwd=z, dEa_rev=z)
        return out

    # numeric getters (J/mol, like the reference) -- evaluated on the device
    def get_reaction_energy(self, T, p, verbose=False, etype='free'):
        from ..engine import evaluate_forms
        f = self.energy_forms()['dErxn' if etype == 'electronic' else 'dGrxn']
        return None if f is None else evaluate_forms([f], T, p)[0] * 1.0e3 * 96.485

    def get_reaction_barriers(self, T, p, verbose=False, etype='free'):
        from ..engine import evaluate_forms
        e = self.energy_forms()
        keys = ('dEa_fwd', 'dEa_rev') if etype == 'electronic' else ('dGa_fwd', 'dGa_rev')
        forms = [e[k] for k in keys]
        vals = evaluate_forms([f for f in forms if f is not None], T, p)
        it = iter(vals)
        return tuple(None if f is None else next(it) * 1.0e3 * 96.485 for f in forms)

    def calc_rate_constants(self, T, p, verbose=False):
        """reaction.py:94-168 for one condition (device kernel (1))."""
        from ..engine import single_reaction_rate_constants
        self.kfwd, self.krev = single_reaction_rate_constants(self, T, p)


class UserDefinedReaction(Reaction):
    """Mirror of reaction.py:202-295: energies given by the user (eV), as
    numbers or as LinearForms in Descriptor(...) / TSYM."""

    def __init__(self, reac_type, reversible=True, reactants=None, products=None, TS=None,
                 area=1.0e-19, name='reaction', scaling=1.0,
                 dErxn_user=None, dEa_fwd_user=None, dEa_rev_user=None,
                 dGrxn_user=None, dGa_fwd_user=None, dGa_rev_user=None):
        super().__init__(reac_type=reac_type, reversible=reversible, reactants=reactants, products=products,
                         TS=TS, area=area, name=name, scaling=scaling)
        self.dErxn_user = dErxn_user
        self.dEa_fwd_user = dEa_fwd_user
        self.dEa_rev_user = dEa_rev_user
        self.dGrxn_user = dGrxn_user
        self.dGa_fwd_user = dGa_fwd_user
        self.dGa_rev_user = dGa_rev_user

    def energy_forms(self):
        """reaction.py:222-274"""
        out = dict(dGrxn=None, dErxn=None, dGa_fwd=None, dEa_fwd=None, dGa_rev=None, dEa_rev=None)
        if self.reversible:
            if self.dErxn_user is not None:
                out['dErxn'] = _lin(self.dErxn_user)
            if self.dGrxn_user is not None:
                out['dGrxn'] = _lin(self.dGrxn_user)
            if out['dErxn'] is None:
                assert out['dGrxn'] is not None
                out['dErxn'] = out['dGrxn']
            if out['dGrxn'] is None:
                out['dGrxn'] = out['dErxn']
        if self.dEa_fwd_user is not None:
            out['dEa_fwd'] = _lin(self.dEa_fwd_user)
            if self.reversible:
                out['dEa_rev'] = out['dEa_fwd'] - out['dErxn']
        if self.dGa_fwd_user is not None:
            out['dGa_fwd'] = _lin(self.dGa_fwd_user)
            if self.reversible:
                out['dGa_rev'] = out['dGa_fwd'] - out['dGrxn']
        if out['dEa_fwd'] is None and out['dGa_fwd'] is not None:
            out['dEa_fwd'], out['dEa_rev'] = out['dGa_fwd'], out['dGa_rev']
        elif out['dEa_fwd'] is not None and out['dGa_fwd'] is None:
            out['dGa_fwd'], out['dGa_rev'] = out['dEa_fwd'], out['dEa_rev']
        elif out['dEa_fwd'] is None and out['dGa_fwd'] is None:
            z = as_form(0.0)
            out.update(dEa_fwd=z, dEa_rev=z, dGa_fwd=z, dGa_rev=z)
        return out


class ReactionDerivedReaction(Reaction):
    """Mirror of reaction.py:298-360: energies from a base reaction's states."""

    def __init__(self, reac_type, reversible=True, reactants=None, products=None, TS=None,
                 area=1.0e-19, name='reaction', scaling=1.0, base_reaction=None):
        super().__init__(reac_type=reac_type, reversible=reversible, reactants=reactants, products=products,
                         TS=TS, area=area, name=name, scaling=scaling)
        assert base_reaction is not None
        self.base_reaction = base_reaction

    def _source(self):
        return self.base_reaction
