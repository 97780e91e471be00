"""Generate golden vectors by running the REFERENCE PyCatKin code in this
container (it is importable here from /root/reference; not on the GPU box).

What runs from the reference, unmodified:
  pycatkin/functions/rate_constants.py   karr / kads / kdes / keq_therm
  pycatkin/classes/reaction.py           Reaction / UserDefinedReaction
                                         calc_reaction_energy, calc_rate_constants
  pycatkin/classes/old_system.py         System.species_odes / species_jacobian /
                                         solve_odes / find_steady / run_and_return_tof /
                                         activity / degree_of_rate_control
  pycatkin/classes/reactor.py            InfiniteDilutionReactor / CSTReactor
What is supplied here: the State objects (pycatkin/classes/state.py imports
`ase`, which this image lacks), as small duck-typed objects whose free energies
come from oracle.mk_oracle.Thermo -- itself pinned separately by
test/test_1.py's energy goldens.  For the "classic" rate model (the one the
reference's own test goldens pin) a Reaction subclass below overrides only the
non-activated adsorption/desorption branch of calc_rate_constants.

Output: tests/golden/ref_vectors.json (small; committed).
Run:    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, ROOT)
sys.path.insert(0, REF)

from oracle import mk_oracle as O  # noqa: E402
from pycatkin.classes import old_system as RS  # noqa: E402
from pycatkin.classes import reaction as RR  # noqa: E402
from pycatkin.classes import reactor as RX  # noqa: E402
from pycatkin.functions import rate_constants as RC  # noqa: E402


class DuckState:
    """Stands in for pycatkin.classes.state.State as a reaction input."""

    def __init__(self, spec, name):
        st = spec['states'][name]
        self.spec, self.name = spec, name
        self.state_type, self.mass, self.sigma = st['type'], st['mass'], st['sigma']
        self.inertia = None if st['inertia'] is None else list(st['inertia'])
        self.Gelec = None

    def get_free_energy(self, T, p, verbose=False):
        th = O.Thermo(self.spec, T, p)
        self.Gelec = th.elec(self.name)
        return th.free(self.name)

    def get_potential_energy(self, verbose=False):
        return O.Thermo(self.spec, 300.0, 1e5).elec(self.name)


def classic_reaction(base):
    class Classic(base):
        """calc_rate_constants with the thermodynamic reverse rate for
        non-activated adsorption / desorption (the semantics the reference's
        own goldens pin); every other branch defers to the reference."""

        def calc_rate_constants(self, T, p, verbose=False):
            typ = str(self.reac_type).upper()
            self.calc_reaction_energy(T=T, p=p, verbose=verbose)
            if typ == 'GHOST':
                # scaling-0 ghost steps never move a species; a unit kfwd keeps
                # old_system.reaction_terms' krev*(1+pert/kfwd) finite
                self.kfwd, self.krev = 1.0, 0.0
                return
            if typ in ('ADSORPTION', 'DESORPTION') and not self.dGa_fwd:
                side = self.reactants if typ == 'ADSORPTION' else self.products
                gas = [s for s in side if s.state_type == 'gas'][0]
                ka = RC.kads(T=T, mass=gas.mass, area=self.area)
                if typ == 'ADSORPTION':
                    self.kfwd = ka
                    self.krev = RC.k_from_eq_rel(ka, RC.keq_therm(T, self.dGrxn), 'forward') if self.reversible else 0.0
                else:
                    self.krev = ka if self.reversible else 0.0
                    self.kfwd = RC.k_from_eq_rel(ka, RC.keq_therm(T, self.dGrxn), 'reverse')
                return
            super().calc_rate_constants(T=T, p=p, verbose=verbose)
            if self.kfwd is None:
                self.kfwd = 0.0
            if self.krev is None:
                self.krev = 0.0
    return Classic


def build_reference_system(spec, mode):
    states = {n: DuckState(spec, n) for n in spec['states']}
    sysd = spec['system']
    s = RS.System()
    s.set_parameters(times=list(sysd['times']), start_state=dict(sysd.get('start_state') or {}),
                     inflow_state=dict(sysd.get('inflow_state') or {}), T=sysd['T'], p=sysd['p'],
                     use_jacobian=sysd.get('use_jacobian', True), ode_solver='solve_ivp',
                     nsteps=sysd.get('nsteps', 1e4), rtol=sysd.get('rtol', 1e-8), atol=sysd.get('atol', 1e-10),
                     xtol=sysd.get('xtol', 1e-8), ftol=sysd.get('ftol', 1e-8))
    for st in states.values():
        s.add_state(st)
    for name, r in spec['reactions'].items():
        kw = dict(reac_type=r['reac_type'], reversible=r['reversible'],
                  reactants=[states[x] for x in r['reactants']], products=[states[x] for x in r['products']],
                  TS=None if r['TS'] is None else [states[x] for x in r['TS']], area=r['area'],
                  name=name, scaling=r['scaling'])
        if r['kind'] == 'user':
            cls = RR.UserDefinedReaction
            kw.update({k: v for k, v in r['user'].items()})
        else:
            cls = RR.Reaction
        if mode == 'classic':
            cls = classic_reaction(cls)
        s.add_reaction(cls(**kw))
    rx = spec['reactor']
    if rx['kind'] == 'CSTR':
        s.add_reactor(RX.CSTReactor(residence_time=rx['residence_time'], volume=rx['volume'],
                                    catalyst_area=rx['catalyst_area']))
    else:
        s.add_reactor(RX.InfiniteDilutionReactor())
    s.names_to_indices()
    return s


def dmtm_vectors(mode):
    spec = O.load_spec(os.path.join(REF, 'examples/DMTM/input.json'))
    out = dict(temperatures=[400.0, 600.0, 800.0], mode=mode, kf=[], kr=[], y_end=[], y_steady=[],
               tof=[], drc=[], odes_y=[], odes=[], snames=None, reactions=list(spec['reactions']))
    rng = np.random.default_rng(7)
    for T in out['temperatures']:
        s = build_reference_system(spec, mode)
        s.params['temperature'] = T
        s.check_rate_constants()
        out['kf'].append([s.rate_constants[r]['kfwd'] for r in out['reactions']])
        out['kr'].append([s.rate_constants[r]['krev'] for r in out['reactions']])
        y = rng.uniform(0.0, 1.0, len(s.snames))
        out['odes_y'].append(y.tolist())
        out['odes'].append(s.species_odes(y).tolist())
        s.solve_odes()
        out['y_end'].append(s.solution[-1].tolist())
        out['y_steady'].append(s.find_steady(store_steady=True).tolist())
        out['tof'].append(s.run_and_return_tof(['r5', 'r9']))
        xi = s.degree_of_rate_control(['r5', 'r9'], eps=5.0e-2)
        out['drc'].append([xi[r] for r in out['reactions']])
        out['snames'] = list(s.snames)
    return out


def volcano_vectors():
    spec = O.load_spec(os.path.join(REF, 'examples/COOxVolcano/input.json'))
    be = [-2.5, -1.5, -1.0, -0.5, 0.5]
    SCOg, SO2g = 2.0487e-3, 2.1261e-3
    T = spec['system']['T']
    s = build_reference_system(spec, 'classic')
    # examples/COOxVolcano/input.json asks for ode_solver 'ode' (lsoda)
    s.params['ode_solver'] = 'ode'
    s.params['nsteps'] = int(1e4)
    act = []
    for ECO in be:
        row = []
        for EO in be:
            # examples/COOxVolcano/cooxvolcano.py:28-47
            s.reactions['CO_ads'].dErxn_user = ECO
            s.reactions['CO_ads'].dGrxn_user = ECO + SCOg * T
            s.reactions['2O_ads'].dErxn_user = 2.0 * EO
            s.reactions['2O_ads'].dGrxn_user = 2.0 * EO + SO2g * T
            spec['reactions']['CO_ads']['user'].update(dErxn_user=ECO, dGrxn_user=ECO + SCOg * T)
            spec['reactions']['2O_ads']['user'].update(dErxn_user=2.0 * EO, dGrxn_user=2.0 * EO + SO2g * T)
            th = O.Thermo(spec, T, spec['system']['p'])
            EO2 = th.elec('sO2')
            s.reactions['O2_ads'].dErxn_user = EO2
            s.reactions['O2_ads'].dGrxn_user = EO2 + SO2g * T
            s.reactions['CO_ox'].dEa_fwd_user = np.max((th.elec('SRTS_ox') - (ECO + EO), 0.0))
            s.reactions['O2_2O'].dEa_fwd_user = np.max((th.elec('SRTS_O2') - EO2, 0.0))
            row.append(float(s.activity(tof_terms=['CO_ox'])))
        act.append(row)
    return dict(binding_energies=be, activity=act)


def main():
    out = dict(generator='tests/golden/make_golden.py (reference code at /root/reference)',
               dmtm_classic=dmtm_vectors('classic'), dmtm_patched=dmtm_vectors('patched'),
               volcano=volcano_vectors())
    with open(os.path.join(HERE, 'ref_vectors.json'), 'w') as fh:
        json.dump(out, fh, indent=1)
    print('wrote', os.path.join(HERE, 'ref_vectors.json'))


if __name__ == '__main__':
    main()
