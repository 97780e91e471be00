"""read_from_input_file: the reference's JSON input format
(pycatkin/functions/load_input.py:9-167) -> a pycatkin_amd System."""
from __future__ import annotations

import json
import os

from ..classes.reaction import Reaction, ReactionDerivedReaction, UserDefinedReaction
from ..classes.reactor import CSTReactor, InfiniteDilutionReactor
from ..classes.state import ScalingState, State
from ..classes.system import System
from ..constants.physical_constants import bartoPa


def _resolve(d, base_dir):
    d = dict(d)
    for k in ('path', 'vibs_path'):
        if d.get(k) and base_dir and not os.path.isabs(d[k]):
            d[k] = os.path.join(base_dir, d[k])
    return d


def read_from_input_file(input_path='input.json', base_system=None, base_dir=None, formulation='classic',
                         rate_model='classic', verbose=False):
    """Build a System from a reference input file.  Relative data paths are
    resolved against `base_dir` (default: the input file's directory)."""
    if verbose:
        print('Loading input file: %s.' % input_path)
    with open(input_path) as fh:
        pck = json.load(fh)
    base_dir = base_dir or os.path.dirname(os.path.abspath(input_path))
    if 'states' not in pck:
        raise RuntimeError('Input file contains no states.')
    states = {s: State(name=s, **_resolve(d, base_dir)) for s, d in pck['states'].items()}
    for s, d in pck.get('scaling relation states', {}).items():
        states[s] = ScalingState(name=s, **_resolve(d, base_dir))
    if 'system' not in pck:
        raise RuntimeError('Input file contains no system details.')
    sp = json.loads(json.dumps(pck['system']))
    p = sp['p']
    startsites = 0.0
    for s in list((sp.get('start_state') or {})):                  # load_input.py:46-54
        if states[s].state_type == 'gas':
            sp['start_state'][s] = sp['start_state'][s] * p / bartoPa
        elif states[s].state_type in ('surface', 'adsorbate'):
            startsites += sp['start_state'][s]
    if 'start_state' in sp and startsites == 0.0:
        raise ValueError('Initial surface coverage cannot be zero for all states!')
    for s in list((sp.get('inflow_state') or {})):                 # load_input.py:55-60
        if states[s].state_type == 'gas':
            sp['inflow_state'][s] = sp['inflow_state'][s] * p / bartoPa
        else:
            raise TypeError('Only gas states can comprise the inflow!')
    sim = System(formulation=formulation, rate_model=rate_model, **sp)
    for s in states.values():
        if s.gasdata is not None:
            s.gasdata = dict(s.gasdata)
            s.gasdata['state'] = [states[i] if isinstance(i, str) else i for i in s.gasdata['state']]
        sim.add_state(s)
    reactions = {}
    for group, cls in (('reactions', Reaction), ('manual reactions', UserDefinedReaction)):
        for r, d in pck.get(group, {}).items():
            d = dict(d)
            d['reactants'] = [sim.states[s] for s in d['reactants']]
            d['products'] = [sim.states[s] for s in d['products']]
            if d.get('TS') is not None:
                d['TS'] = [sim.states[s] for s in d['TS']]
            reactions[r] = cls(name=r, **d)
    for r, d in pck.get('reaction derived reactions', {}).items():
        if base_system is None and not reactions:
            raise RuntimeError('Base reactions not defined.')
        d = dict(d)
        base = d.pop('base_reaction')
        d['reactants'] = [sim.states[s] for s in d['reactants']]
        d['products'] = [sim.states[s] for s in d['products']]
        if d.get('TS') is not None:
            d['TS'] = [sim.states[s] for s in d['TS']]
        src = base_system.reactions if base_system is not None else reactions
        reactions[r] = ReactionDerivedReaction(name=r, base_reaction=src[base], **d)
    for r in reactions.values():                                   # load_input.py:116-129
        for s in r.reactants + r.products + (r.TS or []):
            if isinstance(s, ScalingState):
                for sr in s.scaling_reactions.values():
                    if isinstance(sr['reaction'], str):
                        sr['reaction'] = reactions[sr['reaction']]
        sim.add_reaction(r)
    rx = pck.get('reactor')
    if rx is not None:
        if not isinstance(rx, dict):
            if rx != 'InfiniteDilutionReactor':
                raise TypeError('Only InfiniteDilutionReactor can be specified without reactor parameters.')
            sim.add_reactor(InfiniteDilutionReactor())
        elif 'InfiniteDilutionReactor' in rx:
            sim.add_reactor(InfiniteDilutionReactor())
        elif 'CSTReactor' in rx:
            sim.add_reactor(CSTReactor(**rx['CSTReactor']))
        else:
            raise TypeError('Unknown reactor option, please choose InfiniteDilutionReactor or CSTReactor.')
    elif sim.reactions:
        raise RuntimeError('Cannot consider reactions without reactor. To use constant boundary conditions, '
                           'please specify InfiniteDilutionReactor.')
    sim.names_to_indices()
    return sim
