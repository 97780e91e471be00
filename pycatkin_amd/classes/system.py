"""System: the reference's System API on top of the batched device solver.

Reference-API methods (pycatkin/classes/old_system.py -- the API every example
driver uses -- and the steady-state helpers of the patched
pycatkin/classes/system.py) are kept with their names and argument meaning.
Each of them is a batch of one through the same C-ABI the batched methods
(`*_batch`) use; there is no CPU compute path.
"""
from __future__ import annotations

import copy
from typing import NamedTuple

import numpy as np

from ..constants.physical_constants import R, bartoPa, eVtokJ, h, kB
from ..energy import TKEYED, LinearForm
from .reaction import Reaction
from .reactor import InfiniteDilutionReactor, Reactor
from .state import State


# Steady-state solves (steady=True; DESIGN.md "Steady state").  The transient
# to t_end is integrated at STEADY_TRANSIENT = (rtol, atol), Newton polishes
# its end state, and the root is the answer only if the transient has reached
# it: every dynamic species within ROOT_DIST * |root| + atol of it
# (pck_solve_params.root_dist).  Otherwise (status 4) the answer is the
# transient end at t_end -- the reference's System.activity semantics
# (old_system.py:517-529, what examples/COOxVolcano/cooxvolcano.py:47 reports).
# The tiny atol makes the error control relative on every coverage, down to
# the 1e-16 free sites of an O-poisoned surface whose product the TOF is, so
# that the distance test compares two well-resolved states; the rtol is what
# the 1e-6 bound on log10(TOF) needs with margin: measured on the 89 043
# degenerate points of the 1024 x 1024 volcano grid against a 1e-12 / 1e-24
# run (tools/retry_probe.py, profiles/r3/retry_probe.json), 1e-6 / 1e-22 is
# within 2.7e-8 relative.  On that grid one transient at these tolerances
# costs less than round 3's input-tolerance pass plus a tight retry of the
# degenerate points (6.1 ms against 7.5 ms per step, profiles/r4/tolerance_ab).
STEADY_TRANSIENT = (1.0e-6, 1.0e-22)
ROOT_DIST = 1.0e-6
# round-3 name of the tight tolerances (the retry pass, now optional)
DEGENERATE_RETRY = STEADY_TRANSIENT
# Screening pass of steady solves (round 5, pck_solve_params.screen_rtol;
# DESIGN.md "Screening pass"): the rule first at rtol SCREEN_RTOL (atol scaled
# alike), a root accepted there only within SCREEN_MARGIN * ROOT_DIST * |root|
# + atol (the caller's, round 6) of the screening transient's end.  With that
# absolute term a margin of 0.1 sent ~15 % of the CSTR sweep's trips to a full
# solve (2.8 vs 1.4 ms); 0.5 accepts all of them and 2 % more of the volcano
# grid (2.32 vs 2.37 ms), with 0 status changes on both against the single
# pass (profiles/r6/ab_screen_acceptance, screen_check_*_m0.5.json); every other condition is solved again at
# STEADY_TRANSIENT exactly as without screening.  A transient that has settled
# on its root ends on it at any tolerance, so the accepted conditions report
# the same root.
SCREEN_RTOL = 3.0e-2
SCREEN_MARGIN = 0.5
# 'auto' screens the one-lane networks (<= 8 dynamic species: the volcano and
# CSTR configs); the lane-group kernels screen too when asked (screen=rtol),
# but a network that rarely reaches its root by t_end (the synthetic one
# never does) would then solve most conditions twice
SCREEN_MAX_LANE_SPECIES = 8


def _retry_tolerances(retry):
    """solve_batch's `retry`: None -> no second pass, 'auto' -> STEADY_TRANSIENT,
    else a positive (rtol, atol) pair (any sequence or array of two)."""
    if isinstance(retry, str):
        if retry != 'auto':
            raise ValueError("retry must be 'auto', None or an (rtol, atol) pair, not %r" % retry)
        return DEGENERATE_RETRY
    if retry is None:
        return None
    r = np.asarray(retry, float).ravel()
    if r.size != 2 or not np.all(r > 0.0):
        raise ValueError('retry must be a positive (rtol, atol) pair, not %r' % (retry,))
    return float(r[0]), float(r[1])


class SteadyStateResults(NamedTuple):
    """system.py:20-30"""
    x: np.ndarray
    success: bool


class System:
    """Holds states, reactions and a reactor; solves batches of MK models.

    formulation: 'classic' (old_system.py, default) or 'patched' (system.py).
    rate_model:  'classic' (thermodynamic reverse rate for non-activated
                 adsorption/desorption -- what the reference's goldens pin) or
                 'patched' (kads/kdes, reaction.py:135-162)."""

    def __init__(self, times=None, start_state=None, inflow_state=None, T=293.15, p=101325.0,
                 use_jacobian=True, ode_solver='solve_ivp', nsteps=1e4, rtol=1e-8, atol=1e-10,
                 xtol=1e-8, ftol=1e-8, verbose=False, y0=None, min_tol=1e-32,
                 formulation='classic', rate_model='classic', path_to_pickle=None):
        if path_to_pickle:
            raise NotImplementedError('pickled systems are not loaded (no unpickling of external files)')
        self.states = dict()
        self.unique_states = set()
        self.reactions = dict()
        self.reactor = None
        self.energy_landscapes = None
        self.formulation = formulation
        self.rate_model = rate_model
        self.min_tol = min_tol
        self.snames = None
        self.solution = None
        self.times = None
        self.full_steady = None
        self.rates = None
        self.rate_constants = None
        self._plans = {}
        self.set_parameters(times=times, start_state=start_state, inflow_state=inflow_state, T=T, p=p,
                            use_jacobian=use_jacobian, ode_solver=ode_solver, nsteps=nsteps, rtol=rtol, atol=atol,
                            xtol=xtol, ftol=ftol, verbose=verbose)

    # -- setup (old_system.py:49-175, system.py:90-187) ------------------------
    def set_parameters(self, times=None, start_state=None, inflow_state=None, T=293.15, p=101325.0,
                       use_jacobian=True, ode_solver='solve_ivp', nsteps=1e4, rtol=1e-8, atol=1e-10,
                       xtol=1e-8, ftol=1e-8, verbose=False):
        self.params = dict(times=copy.deepcopy(times), start_state=copy.deepcopy(start_state),
                           inflow_state=copy.deepcopy(inflow_state), temperature=T, pressure=p, rtol=rtol,
                           atol=atol, xtol=xtol, ftol=ftol, jacobian=use_jacobian, nsteps=int(nsteps),
                           ode_solver=ode_solver, verbose=verbose)

    def __deepcopy__(self, memo):
        """A deep copy (butadiene_mkm.py:47, analysis.py:40) starts with an
        empty plan cache: device networks are not copied."""
        out = self.__class__.__new__(self.__class__)
        memo[id(self)] = out
        for k, v in self.__dict__.items():
            setattr(out, k, {} if k == '_plans' else copy.deepcopy(v, memo))
        return out

    # patched-API attribute names
    @property
    def T(self):
        return self.params['temperature']

    @T.setter
    def T(self, v):
        self.params['temperature'] = v

    @property
    def p(self):
        return self.params['pressure']

    @p.setter
    def p(self, v):
        self.params['pressure'] = v

    @property
    def start_state(self):
        return self.params['start_state'] or {}

    @property
    def inflow_state(self):
        return self.params['inflow_state'] or {}

    def add_state(self, state):
        assert isinstance(state, State), 'state %s MUST be an instance of State' % state
        if state.name in self.unique_states:
            raise ValueError('Found two copies of state %s. State names must be unique!' % state.name)
        self.unique_states.add(state.name)
        self.states[state.name] = state
        self.snames = sorted(self.states)
        self._plans.clear()

    def add_reaction(self, reaction):
        assert isinstance(reaction, Reaction), 'reaction %s MUST be an instance of Reaction' % reaction
        self.reactions[reaction.name] = reaction
        self._plans.clear()

    def add_reactor(self, reactor):
        assert isinstance(reactor, Reactor)
        self.reactor = reactor
        self._plans.clear()

    def add_energy_landscape(self, energy_landscape):
        if self.energy_landscapes is None:
            self.energy_landscapes = dict()
        self.energy_landscapes[energy_landscape.name] = energy_landscape

    def names_to_indices(self):
        """old_system.py:99-152 index bookkeeping (kept for API compatibility)."""
        self.snames = sorted(self.states)
        ads, gas = set(), set()
        for r in self.reactions.values():
            for s in r.reactants + r.products:
                if s.state_type in ('adsorbate', 'surface'):
                    ads.add(self.snames.index(s.name))
                elif s.state_type == 'gas':
                    gas.add(self.snames.index(s.name))
        self.adsorbate_indices = sorted(ads)
        self.gas_indices = sorted(gas)
        n = len(self.snames)
        if self.reactor is not None:
            self.reactor.set_indices([1 if i in ads else 0 for i in range(n)], [1 if i in gas else 0 for i in range(n)])
            self.dynamic_indices = self.reactor.get_dynamic_indices(self.adsorbate_indices, self.gas_indices)

    def build(self):
        """Index bookkeeping: old_system.py:99-152 (classic) or system.py:167-187
        (patched: coverage_map, gas_indices, index_map, rate_map,
        initial_system, reaction_matrix)."""
        if self.formulation == 'patched':
            return self._build_patched()
        return self.names_to_indices()

    # -- patched-formulation API (pycatkin/classes/system.py) --------------------
    def _build_patched(self):
        """system.py:191-394: index_map (gas first, then each surface followed by
        its adsorbates), coverage_map {surface: set of indices}, gas_indices,
        rate_map, initial_system (normalised, capped at min_tol) and the +-1
        reaction_matrix (species x non-ghost reactions, products win)."""
        order = self.index_map_ordered()
        self.index_map = {s: i for i, s in enumerate(order)}
        self.gas_indices = {i for i, s in enumerate(order) if self.states[s].state_type == 'gas'}
        self.coverage_map = {sf: {self.index_map[x] for x in grp} for sf, grp in self._coverage_names.items()}
        self.rate_map = {}
        for name, rx in self.reactions.items():
            if str(rx.reac_type).upper() == 'GHOST':
                continue
            self.rate_map[name] = {'reac': [self.index_map[x.name] for x in rx.reactants],
                                   'prod': [self.index_map[x.name] for x in rx.products],
                                   'site_density': 1.0 / rx.area if rx.area else 0.0, 'scaling': rx.scaling}
        self.initial_system = self.initial_vector()
        M = np.zeros((len(order), len(self.rate_map)))
        for j, rm in enumerate(self.rate_map.values()):
            M[rm['reac'], j] = -1.0
            M[rm['prod'], j] = 1.0
        self.reaction_matrix = M
        return self

    def _patched_eval(self):
        if self.formulation != 'patched':
            raise RuntimeError('the System._fun_ss / get_dydt family belongs to the patched formulation '
                               '(System(formulation="patched"), pycatkin/classes/system.py)')
        if getattr(self, 'initial_system', None) is None:
            self._build_patched()
        plan = self.plan()
        net = self.device()
        ngas = len(self.gas_indices)
        return plan, net, ngas

    def _device_state(self, plan, y_full):
        """(surface part in plan.dyn order, gas concentrations x p in plan.fix order)."""
        y_full = np.asarray(y_full, float).ravel()
        idx = self.index_map
        yd = np.array([y_full[idx[s]] for s in plan.dyn])
        fx = np.array([y_full[idx[s]] for s in plan.fix]) * float(self.p)
        return yd, fx

    def _rates_batch(self, Y, desc=None):
        """forward / backward rates [n_reactions, m] (rate_map order) at full
        compositions Y [n_species, m] (gas fractions x p), one device launch;
        `desc` {name: [m]} for a network with descriptor energies."""
        plan, net, ngas = self._patched_eval()
        Y = np.asarray(Y, float)
        m = Y.shape[1]
        idx = self.index_map
        yd = Y[[idx[s] for s in plan.dyn]]
        fx = Y[[idx[s] for s in plan.fix]] * float(self.p)
        T, p, d, _, _, _ = self._inputs(net, plan, m, np.full(m, float(self.T)), float(self.p), desc,
                                        None, None, None)
        kf, kr = net.rate_constants(m, T, p, d)
        rf, rr = net.reaction_rates(m, T, p, yd, kf, kr, d, fx)
        rf, rr = rf.cpu().numpy(), rr.cpu().numpy()
        names = list(self.rate_map)
        order = [plan.reactions.index(name) for name in names]
        return rf[order], rr[order]

    def _calc_rates(self, y):
        """system.py:345-376: (n_reactions, 2) forward / backward rates at the
        full composition y (gas fractions x p), on the device."""
        rf, rr = self._rates_batch(np.asarray(y, float).reshape(-1, 1))
        return np.stack([rf[:, 0], rr[:, 0]], axis=1)

    def get_dydt(self, y):
        """system.py:396-416: reaction_matrix @ (r_fwd - r_rev) for every tracked species."""
        rates = self._calc_rates(y)
        return self.reaction_matrix @ (rates[:, 0] - rates[:, 1])

    def get_dydt_batch(self, Y, desc=None):
        """get_dydt for compositions Y [n_species, m] in one launch."""
        rf, rr = self._rates_batch(Y, desc)
        return self.reaction_matrix @ (rf - rr)

    def get_forward_only(self, y):
        """system.py:418-433 (the reference multiplies by the backward column)."""
        return self.reaction_matrix @ self._calc_rates(y)[:, 1]

    def _jac(self, y):
        """system.py:437-491: d r_j / d y_k (n_reactions x n_species).  Every
        species enters a side of a reaction with exponent 1 (a repeated species
        with its count), so d(k prod c)/d y_k = k prod(others) (x p for a gas):
        the rate of that side with y_k set to 1 -- one device launch evaluates
        the rates at all n_species such compositions.  The reference's P_term
        (system.py:478-484) multiplies by p only when ANOTHER species of the
        side is a gas, so the column of a gas species itself carries no p:
        that column is divided by p here to return the reference's matrix
        (the device integrators use the exact derivative)."""
        self._patched_eval()
        y = np.asarray(y, float).ravel()
        n = len(y)
        Y = np.repeat(y[:, None], n, axis=1)
        Y[np.arange(n), np.arange(n)] = 1.0
        rf, rr = self._rates_batch(Y)
        out = np.zeros((len(self.rate_map), n))
        for j, (name, rm) in enumerate(self.rate_map.items()):
            for lst, other, sgn, r in ((rm['reac'], rm['prod'], 1.0, rf), (rm['prod'], rm['reac'], -1.0, rr)):
                for i in set(lst):
                    if i in other:
                        raise RuntimeError('Species %d appreas on both sides of reaction %s' % (i, name))
                    cnt = lst.count(i)
                    # side rate at y_i = 1 is k prod(others) y_i^0 -> times cnt y_i^(cnt-1)
                    out[j, i] = sgn * r[j, i] * (cnt * y[i] ** (cnt - 1) if cnt > 1 else 1.0)
                    if i in self.gas_indices:
                        out[j, i] /= float(self.p)
        return out

    def get_jacobian(self, y):
        """system.py:493-508: reaction_matrix @ _jac(y)."""
        return self.reaction_matrix @ self._jac(y)

    def _ss_pre(self, y_surf):
        """system.py:512-526"""
        self._patched_eval()
        y_gas = self.initial_system[sorted(self.gas_indices)]
        return np.concatenate([y_gas, np.asarray(y_surf, float)])

    def _fun_ss(self, y_surf):
        """system.py:528-545: surface rates at the invariant gas composition (device pck_species_rates)."""
        return self._fun_ss_batch(np.asarray(y_surf, float)[:, None])[:, 0]

    def _jac_ss(self, y_surf):
        """system.py:547-564: surface block of the Jacobian (device pck_jacobian)."""
        return self._jac_ss_batch(np.asarray(y_surf, float)[:, None])[:, :, 0]

    def _fun_ss_batch(self, Y, desc=None, T=None):
        """_fun_ss for a batch of surface states Y [n_surface, n] in one launch
        (`desc` / `T`: per-condition descriptor energies / temperatures)."""
        plan, net, ngas = self._patched_eval()
        n = Y.shape[1]
        T = float(self.T) if T is None else T
        T, p, d, fx, y0, inflow = self._inputs(net, plan, n, T, None, desc, None, None, None)
        kf, kr = net.rate_constants(n, T, p, d)
        return net.species_rates(n, T, p, self._to_plan(plan, Y), kf, kr, d, fx, inflow).cpu().numpy()[self._from_plan(plan)]

    def _jac_ss_batch(self, Y, desc=None, T=None):
        plan, net, ngas = self._patched_eval()
        n = Y.shape[1]
        T = float(self.T) if T is None else T
        T, p, d, fx, y0, inflow = self._inputs(net, plan, n, T, None, desc, None, None, None)
        kf, kr = net.rate_constants(n, T, p, d)
        J = net.jacobian(n, T, p, self._to_plan(plan, Y), kf, kr, d, fx, inflow).cpu().numpy()
        inv = self._from_plan(plan)
        return J[np.ix_(inv, inv)]

    def _surface_order(self):
        return [s for s in sorted(self.index_map, key=self.index_map.get) if self.index_map[s] not in self.gas_indices]

    def _to_plan(self, plan, Y):
        """surface states in index_map order -> plan.dyn order"""
        order = self._surface_order()
        return np.asarray(Y, float)[[order.index(s) for s in plan.dyn]]

    def _from_plan(self, plan):
        """permutation taking plan.dyn order back to index_map order"""
        return [plan.dyn.index(s) for s in self._surface_order()]

    # -- patched-formulation bookkeeping (system.py:191-328) -------------------
    def index_map_ordered(self):
        ads = [n for n, s in self.states.items() if s.state_type == 'adsorbate']
        gas = sorted(n for n, s in self.states.items() if s.state_type == 'gas')
        surf = sorted(n for n, s in self.states.items() if s.state_type == 'surface')
        order = list(gas)
        self._coverage_names = {}
        for sf in surf:
            grp = [sf] + [a for a in ads if a[0] == sf]
            self._coverage_names[sf] = grp
            order += grp
        return order

    def initial_vector(self):
        """system.py:282-328: normalised gas fractions and site coverages, capped at min_tol."""
        order = self.index_map_ordered()
        pos = {s: i for i, s in enumerate(order)}
        y = np.zeros(len(order))
        for d in (self.start_state, self.inflow_state):
            for k, v in d.items():
                y[pos[k]] = v
        gi = [pos[s] for s in order if self.states[s].state_type == 'gas']
        if gi:
            y[gi] /= np.sum(y[gi])
        for grp in self._coverage_names.values():
            ii = [pos[s] for s in grp]
            y[ii] /= np.sum(y[ii])
        return np.where(y < self.min_tol, self.min_tol, y)

    def start_state_values(self):
        return dict(self.start_state)

    def inflow_state_values(self):
        return dict(self.inflow_state)

    # -- compilation -------------------------------------------------------------
    def plan(self, tof_terms=(), descriptors=None):
        from ..network import compile_system
        key = (tuple(tof_terms), tuple(descriptors) if descriptors else None, self.formulation, self.rate_model,
               self._energy_key())
        if key not in self._plans:
            if self.snames is None:
                self.snames = sorted(self.states)
            plan = compile_system(self, tof_terms=tof_terms, descriptors=descriptors, rate_model=self.rate_model)
            self._plans[key] = [plan, None]
        return self._plans[key][0]

    def device(self, tof_terms=(), descriptors=None):
        from ..engine import DeviceNetwork
        plan = self.plan(tof_terms, descriptors)
        key = [k for k, v in self._plans.items() if v[0] is plan][0]
        if self._plans[key][1] is None:
            self._plans[key][1] = DeviceNetwork.from_plan(plan)
        return self._plans[key][1]

    def _energy_key(self):
        """User energies may be mutated between calls (volcano drivers): key the cache on them."""
        out = []
        for r in self.reactions.values():
            for a in ('dErxn_user', 'dEa_fwd_user', 'dEa_rev_user', 'dGrxn_user', 'dGa_fwd_user', 'dGa_rev_user'):
                v = getattr(r, a, None)
                if isinstance(v, dict):             # temperature-keyed (energy.tkeyed)
                    v = tuple(sorted((float(k), float(x)) for k, x in v.items()))
                out.append(repr(v) if isinstance(v, LinearForm) else v)
        return tuple(out)

    # -- batch inputs --------------------------------------------------------------
    def _inputs(self, net, plan, n, T, p, desc, y0, fix, inflow):
        T = self.params['temperature'] if T is None else T
        p = self.params['pressure'] if p is None else p
        d = None
        if plan.descriptors:
            given = [k for k in plan.descriptors if not k.startswith('@T:')]
            if given and desc is None:
                raise ValueError('network depends on descriptors %s' % given)
            Tn = np.broadcast_to(np.asarray(T, float), (n,))
            cols = []
            for k in plan.descriptors:
                if k.startswith('@T:'):             # temperature-keyed user energy (energy.tkeyed)
                    table = TKEYED[k]
                    cols.append(np.array([table[float(t)] for t in Tn]))
                else:
                    cols.append(np.broadcast_to(np.asarray(desc[k], float), (n,)))
            d = np.stack(cols)
        if fix is None:
            if plan.formulation == 'patched':
                pp = np.broadcast_to(np.asarray(p, float), (n,))
                fix = plan.fix_default[:, None] * pp[None, :] if len(plan.fix) else None
            else:
                fix = plan.fix_default * plan.fix_conc_factor
        else:
            fix = np.asarray(fix, float) * (plan.fix_conc_factor[:, None] if np.ndim(fix) == 2 else plan.fix_conc_factor)
        y0 = plan.y0_default if y0 is None else y0
        inflow = plan.inflow_default if inflow is None else inflow
        return T, p, d, fix, y0, inflow

    @staticmethod
    def _n(*xs):
        sizes = [int(np.size(x)) for x in xs if x is not None and np.ndim(x) > 0]
        return max(sizes) if sizes else 1

    # -- batched entry points ------------------------------------------------------
    def rate_constants_batch(self, T=None, p=None, desc=None):
        """kf, kr [active reactions, n] (reaction.py:94 for every condition)."""
        plan = self.plan((), None)
        net = self.device((), None)
        n = self._n(T, p, *(desc or {}).values()) if desc else self._n(T, p)
        T, p, d, _, _, _ = self._inputs(net, plan, n, T, p, desc, None, None, None)
        kf, kr = net.rate_constants(n, T, p, d)
        return kf.cpu().numpy(), kr.cpu().numpy()

    def solve_batch(self, T=None, p=None, desc=None, y0=None, fix=None, inflow=None, tof_terms=(),
                    steady=False, activity=False, t_end=None, t0=None, rtol=None, atol=None, max_steps=200000,
                    newton_iters=60, to_numpy=True, t_out=None, retry=None, root_dist='auto', screen='auto',
                    wave_order='auto'):
        """Transient solve to t_end (solve_odes), optionally polished to the
        steady state (find_steady), with TOF or activity per condition; with
        t_out, also the dynamic state at those times ('traj' [n_out, NS, n],
        RODAS4P dense output).

        steady=True: the transient runs at STEADY_TRANSIENT (1e-6 / 1e-22)
        unless rtol / atol are given here -- the System's params['rtol'] /
        ['atol'] (the input file's) are NOT used for steady solves, since the
        rule's distance test needs relative error control on every coverage
         -- and the Newton root of its end state is reported (status
        0) where the transient has reached it to `root_dist` ('auto':
        ROOT_DIST when t_end > t0, else 0 -- a polish of the given state, as
        find_steady); elsewhere the transient end (status 4).  `retry` =
        (rtol, atol) integrates the status-4 conditions again at those
        tolerances in a second launch (None: no second pass).  `screen`
        ('auto': SCREEN_RTOL for steady solves with root_dist > 0, no retry
        and no t_out; None: off; a number: the screening rtol) runs the rule
        at that loose tolerance first and solves only the conditions it does
        not accept at the transient tolerances ('auto' on one-lane networks
        only; a number screens the 16- / 32-lane group networks too, a network
        of at most 16 species then running on the 16-lane kernel instead of
        the quad one; networks of more than 32 species refuse it).
        `wave_order` ('auto', 'on', 'off'; pck_solve_params.wave_order): the
        one-lane solver's cost-ordered dispatch, a preview of 4 samples per
        wavefront that puts the costliest wavefronts first ('auto': from
        131 072 conditions).  It pays where costs vary a lot across the batch
        (the volcano grid) and is overhead where they do not: a 262 144-
        temperature CSTR sweep takes 1.71 ms with it off against 2.36 ms
        (DESIGN.md "Round 6")."""
        plan = self.plan(tuple(tof_terms), None)
        net = self.device(tuple(tof_terms), None)
        sizes = [T, p] + (list(desc.values()) if desc else [])
        n = self._n(*sizes)
        if y0 is not None and np.ndim(y0) == 2:
            n = max(n, np.shape(y0)[1])
        T, p, d, fx, y0, inflow = self._inputs(net, plan, n, T, p, desc, y0, fix, inflow)
        times = self.params['times'] or [0.0, 1.0e4]
        t0 = times[0] if t0 is None else t0
        t_end = times[-1] if t_end is None else t_end
        if steady:
            rtol = STEADY_TRANSIENT[0] if rtol is None else rtol
            atol = STEADY_TRANSIENT[1] if atol is None else atol
        if isinstance(root_dist, str):
            if root_dist != 'auto':
                raise ValueError("root_dist must be 'auto' or a number in [0, 1)")
            root_dist = ROOT_DIST if (steady and t_end > t0) else 0.0
        if isinstance(screen, str):
            if screen != 'auto':
                raise ValueError("screen must be 'auto', None or an rtol")
            screen = SCREEN_RTOL if (steady and root_dist > 0.0 and retry is None and t_out is None
                                     and net.NDYN <= SCREEN_MAX_LANE_SPECIES) else None
        out = net.solve(n, T, p, y0, d, fx, inflow, t0=t0, t_end=t_end,
                        rtol=self.params['rtol'] if rtol is None else rtol,
                        atol=self.params['atol'] if atol is None else atol,
                        max_steps=max_steps, newton=steady, newton_iters=newton_iters, activity=activity,
                        t_out=t_out, retry=_retry_tolerances(retry) if steady else None,
                        root_dist=float(root_dist) if steady else 0.0,
                        screen=(float(screen), SCREEN_MARGIN) if (steady and screen) else None,
                        wave_order={'auto': 0, 'on': 1, 'off': -1}[wave_order])
        if to_numpy:
            return {k: v.cpu().numpy() for k, v in out.items()}
        return out

    def drc_batch(self, tof_terms, T=None, p=None, desc=None, eps=1.0e-3, steady=False, t_end=None, rtol=None,
                  atol=None, max_steps=200000, y0=None, fix=None, inflow=None, screen='auto'):
        """Degree of rate control of every reaction (old_system.py:490-515) for a batch.
        steady=True: each of the 2R+1 solves is a steady-state solve with
        solve_batch's rule (STEADY_TRANSIENT unless rtol / atol are given;
        the root where the transient has reached it to ROOT_DIST, else the
        transient end: the condition's status is then 4).  `screen`: as in
        solve_batch (each of the 2R+1 solves screened on its own).

        Returns {reaction name: xi [n]} (ghost reactions: 0) plus 'tof0' and 'status'."""
        plan = self.plan(tuple(tof_terms), None)
        net = self.device(tuple(tof_terms), None)
        n = self._n(T, p, *(desc.values() if desc else []))
        for a in (y0, fix, inflow):
            if a is not None and np.ndim(a) == 2:
                n = max(n, np.shape(a)[1])
        T, p, d, fx, y0, inflow = self._inputs(net, plan, n, T, p, desc, y0, fix, inflow)
        times = self.params['times'] or [0.0, 1.0e4]
        if steady:
            rtol = STEADY_TRANSIENT[0] if rtol is None else rtol
            atol = STEADY_TRANSIENT[1] if atol is None else atol
        if isinstance(screen, str):
            if screen != 'auto':
                raise ValueError("screen must be 'auto', None or an rtol")
            screen = SCREEN_RTOL if (steady and net.NDYN <= SCREEN_MAX_LANE_SPECIES) else None
        r = net.drc(n, T, p, y0, d, fx, inflow, t0=times[0], t_end=times[-1] if t_end is None else t_end,
                    rtol=self.params['rtol'] if rtol is None else rtol,
                    atol=self.params['atol'] if atol is None else atol, max_steps=max_steps, newton=steady,
                    drc_eps=eps, root_dist=ROOT_DIST if steady else 0.0,
                    screen=(float(screen), SCREEN_MARGIN) if (steady and screen) else None)
        xi = r['xi'].cpu().numpy()
        out = {name: (xi[plan.reactions.index(name)] if name in plan.reactions else np.zeros(n))
               for name in plan.all_reactions}
        out['tof0'] = r['tof0'].cpu().numpy()
        out['status'] = r['status'].cpu().numpy()
        out['nsteps'] = r['nsteps'].cpu().numpy()
        return out

    # -- reference API (one condition) -------------------------------------------------
    def _full(self, plan, ydyn):
        """Dynamic state -> vector over all states in reference order."""
        order = plan.species
        y = np.zeros(len(order))
        pos = {s: i for i, s in enumerate(order)}
        if plan.formulation == 'patched':
            y[:] = self.initial_vector()
        else:
            for s, v in (self.start_state or {}).items():
                y[pos[s]] = v
        for i, s in enumerate(plan.dyn):
            y[pos[s]] = ydyn[i]
        return y

    def output_times(self):
        """old_system.py:363-368: [0] + nsteps log-spaced times from times[0]
        (1e-8 if 0) to times[-1] -- the reference's `ode` path output grid.
        The `solve_ivp` path stores every BDF step instead (old_system.py:350-358),
        which no other integrator reproduces; it gets the same grid here."""
        t0, t1 = float(self.params['times'][0]), float(self.params['times'][-1])
        n = int(self.params['nsteps'])
        out = np.concatenate((np.zeros(1), np.logspace(np.log10(t0 if t0 else 1.0e-8), np.log10(t1), num=n,
                                                        endpoint=True)))
        # 10**log10(t1) can land one ulp above t1 (7200 -> 7200.000000000001):
        # the last sample is the end of the integration, exactly
        out[-1] = t1
        return out

    def solve_odes(self):
        """old_system.py:315-383: integrate params['times'][0] -> [-1]; self.times /
        self.solution hold the state at output_times() (device dense output)."""
        plan = self.plan()
        times = self.output_times()
        inside = times[times >= float(self.params['times'][0])]
        r = self.solve_batch(T=[self.params['temperature']], t_out=inside)
        self._check(r['status'][0], 'solve_odes')
        traj = r['traj'][:, :, 0]
        sol = np.empty((times.size, len(plan.species)))
        sol[:times.size - inside.size] = self._full(plan, plan.y0_default)
        for k in range(inside.size):
            sol[times.size - inside.size + k] = self._full(plan, traj[k])
        self.times = times
        self.solution = sol
        return self.solution

    def write_results(self, path=''):
        """old_system.py:531-568: rates_/coverages_/pressures_<T>K_<p>bar.csv over
        self.times (forward and reverse rate of every reaction at each sample
        from one device launch of pck_reaction_rates)."""
        import os
        import pandas as pd
        if path != '' and not os.path.isdir(path):
            os.makedirs(path, exist_ok=True)
        plan = self.plan()
        T = self.params['temperature']
        p = self.params['pressure']
        tag = ('%1.1f' % T) + 'K_' + ('%1.1f' % (p / bartoPa)) + 'bar.csv'
        names = list(plan.species)
        st = self.states
        ads = [i for i, s in enumerate(names) if st[s].state_type in ('adsorbate', 'surface') and s in plan.dyn + plan.fix]
        gas = [i for i, s in enumerate(names) if st[s].state_type == 'gas' and s in plan.dyn + plan.fix]
        rates = self._rates_at(plan, self.solution)
        rheader = ['Time (s)'] + [x for r in self.reactions.values() for x in (r.name + '_fwd', r.name + '_rev')]
        times = self.times.reshape(-1, 1)
        pd.DataFrame(np.concatenate((times, rates), axis=1), columns=rheader).to_csv(path + 'rates_' + tag,
                                                                                     index=False)
        pd.DataFrame(np.concatenate((times, self.solution[:, ads]), axis=1),
                     columns=['Time (s)'] + [names[i] for i in ads]).to_csv(path + 'coverages_' + tag, index=False)
        pd.DataFrame(np.concatenate((times, self.solution[:, gas]), axis=1),
                     columns=['Time (s)'] + [names[i] for i in gas]).to_csv(path + 'pressures_' + tag, index=False)

    def _rates_at(self, plan, full_states):
        """[n_samples, 2 * n_reactions] (fwd, rev interleaved, reference order) at
        full state vectors (classic units), one pck_reaction_rates launch."""
        net = self.device()
        m = full_states.shape[0]
        pos = {s: i for i, s in enumerate(plan.species)}
        yd = np.stack([full_states[:, pos[s]] for s in plan.dyn]) if plan.dyn else np.zeros((0, m))
        fx = (np.stack([full_states[:, pos[s]] for s in plan.fix]) * plan.fix_conc_factor[:, None]
              if plan.fix else None)
        T = np.full(m, float(self.params['temperature']))
        Tt, p, d, _, _, _ = self._inputs(net, plan, m, T, None, None, None, None, None)
        kf, kr = net.rate_constants(m, Tt, p, d)
        rf, rr = net.reaction_rates(m, Tt, p, yd, kf, kr, d, fx)
        rf, rr = rf.cpu().numpy(), rr.cpu().numpy()
        out = np.zeros((m, 2 * len(plan.all_reactions)))
        for j, name in enumerate(plan.all_reactions):
            if name in plan.reactions:
                a = plan.reactions.index(name)
                out[:, 2 * j], out[:, 2 * j + 1] = rf[a], rr[a]
        return out

    def find_steady(self, *args, **kw):
        """old_system.py:385-468 find_steady(store_steady, plot_comparison, path) for
        formulation 'classic'; system.py:566-639 find_steady(max_iters, y0, method)
        -> SteadyStateResults for formulation 'patched'."""
        if self.formulation == 'patched':
            return self.find_steady_state(*args, **kw)
        return self._find_steady_classic(*args, **kw)

    def _find_steady_classic(self, store_steady=False, plot_comparison=False, path=None):
        plan = self.plan()
        if self.solution is not None:
            pos = {s: i for i, s in enumerate(plan.species)}
            y0 = np.array([self.solution[-1][pos[s]] for s in plan.dyn])
        else:
            y0 = plan.y0_default
        r = self.solve_batch(T=[self.params['temperature']], y0=y0[:, None], t_end=self.params['times'][0],
                             t0=self.params['times'][0], steady=True)
        # status 4: a degenerate root; the reference's least_squares returns
        # wherever xtol stops it (old_system.py:426-433), the device returns
        # the transient end it started from -- never an error
        self._check(r['status'][0], 'find_steady', degenerate_ok=True)
        full = self._full(plan, r['y'][:, 0])
        if store_steady:
            self.full_steady = full
        return full

    @staticmethod
    def _check(st, what, degenerate_ok=False):
        """Raise on a failed solve (1 max steps, 2 step failure, 3 non-finite);
        status 4 (no steady state reached by t_end: the transient end is
        reported) and 5 (the same after a failed `retry` pass: the first
        pass's transient) are results where the reference's steady-state path
        would return one."""
        if st != 0 and not (degenerate_ok and st in (4, 5, 6)):
            raise RuntimeError('%s: device solver status %d (1 max steps, 2 step failure, 3 non-finite, '
                               '4 no steady state reached: transient end, 5 the same with the first-pass '
                               'transient, 6 a DRC mixing reached roots and transient ends)' % (what, st))

    def reaction_terms(self, y):
        """old_system.py:202-225: rates (n_reactions, 2) at the full state y."""
        plan = self.plan()
        kf, kr = self.rate_constants_batch(T=[self.params['temperature']])
        pos = {s: i for i, s in enumerate(plan.species)}
        y = np.asarray(y, float).ravel()
        self.rates = np.zeros((len(plan.all_reactions), 2))
        for j, name in enumerate(plan.all_reactions):
            if name not in plan.reactions:
                continue
            a = plan.reactions.index(name)
            rx = self.reactions[name]
            rf, rr = kf[a, 0], kr[a, 0]
            for side, acc in ((rx.reactants, 0), (rx.products, 1)):
                v = rf if acc == 0 else rr
                for s in side:
                    if s.name in pos:
                        c = y[pos[s.name]]
                        if s.state_type == 'gas':
                            c = c * (bartoPa if plan.formulation == 'classic' else self.params['pressure'])
                        v *= c
                if acc == 0:
                    rf = v
                else:
                    rr = v
            self.rates[j] = (rf, rr)
        return self.rates

    def run_and_return_tof(self, tof_terms, ss_solve=False):
        """old_system.py:470-488"""
        r = self.solve_batch(T=[self.params['temperature']], tof_terms=tuple(tof_terms), steady=ss_solve)
        self._check(r['status'][0], 'run_and_return_tof', degenerate_ok=True)
        return float(r['tof'][0])

    def activity(self, tof_terms, ss_solve=False):
        """old_system.py:517-529 (eV)"""
        r = self.solve_batch(T=[self.params['temperature']], tof_terms=tuple(tof_terms), steady=ss_solve,
                             activity=True)
        self._check(r['status'][0], 'activity', degenerate_ok=True)
        return float(r['tof'][0])

    def degree_of_rate_control(self, tof_terms, ss_solve=False, eps=1.0e-3):
        """old_system.py:490-515.  As the reference's (whose ss_solve path
        returns wherever least_squares stops), a condition whose transient has
        not reached a steady state (status 4) still returns its xi: every TOF
        of the central difference is then that solve's answer by
        solve_batch's rule (a root reached, or the transient end at t_end)."""
        r = self.drc_batch(tof_terms, T=[self.params['temperature']], eps=eps, steady=ss_solve)
        self._check(r['status'][0], 'degree_of_rate_control', degenerate_ok=True)
        if r['status'][0] == 6:
            import warnings
            warnings.warn('degree_of_rate_control: the perturbed solves fall on both sides of the steady rule '
                          '(some reached a root, some report the transient end at t_end): the central '
                          'differences mix the two and xi measures the rule switching (status 6)')
        return {k: float(r[k][0]) for k in self.reactions}

    # patched-API steady state (system.py:566-639)
    def find_steady_state(self, max_iters=30, y0=None, method=None):
        """system.py:566-639.  The reference restarts scipy `root` from a random
        guess until the surface rates vanish and the sites sum to one; here the
        guess (y0, or the start state: deterministic) is first integrated to
        params['times'][-1] (1e6 s when no times are set) so that Newton
        starts in the basin of the stable root, then polished."""
        plan = self.plan()
        yd = plan.y0_default if y0 is None else np.asarray(y0, float)[len(plan.fix):]
        times = self.params.get('times')
        t_end = float(times[-1]) if times is not None and len(times) else 1.0e6
        r = self.solve_batch(T=[self.params['temperature']], y0=np.asarray(yd)[:, None],
                             t0=0.0, t_end=t_end, steady=True, newton_iters=max(int(max_iters), 60))
        x = np.concatenate([plan.fix_default, r['y'][:, 0]])
        return SteadyStateResults(x, bool(r['status'][0] == 0))
