"""Compile a System into the flat device plan of include/pycatkin_amd.h.

Two ODE formulations of the reference are supported, selected by
System.formulation:

  'classic'  pycatkin/classes/old_system.py:99-313 + reactor.py -- sorted state
             names, gas pressures in bar (x bartoPa in the rates), stoichiometric
             weights scaling (x 1/area for gas rows), Reactor row scaling / flow.
  'patched'  pycatkin/classes/system.py:191-508 -- gas first then each surface
             followed by its adsorbates, gas mole fractions x p, a +-1
             reaction_matrix built by index assignment (no accumulation).

Ghost reactions (reac_type 'ghost') only carry descriptor energies and are
left out of the rate network, as system.py:260 does.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L
from .constants.physical_constants import amutokg, bartoPa, h, kB
from .energy import LinearForm, as_form


@dataclass
class NetworkPlan:
    ip: np.ndarray
    dp: np.ndarray
    formulation: str
    rate_model: str
    species: list            # all tracked species names in reference order
    dyn: list                # dynamic species names (solver state order)
    fix: list                # fixed species names (folded into k)
    reactions: list          # active reaction names (device order)
    all_reactions: list      # every reaction name (reference order)
    descriptors: list        # descriptor names (device order)
    tof_terms: list
    conc_factor: np.ndarray  # per dynamic species
    fix_conc_factor: np.ndarray
    y0_default: np.ndarray   # dynamic initial state
    fix_default: np.ndarray  # fixed-species values in the reference's units (bar / fraction)
    inflow_default: np.ndarray
    conservation: np.ndarray
    extra: dict = field(default_factory=dict)

    @property
    def digest(self):
        return hashlib.sha1(self.ip.tobytes() + self.dp.tobytes()).hexdigest()[:16]


def _rref_pivots(C, tol=1e-10):
    """Reduced row echelon form of C with the pivot column of every row."""
    A = np.array(C, dtype=float)
    m, n = A.shape
    piv = []
    r = 0
    for c in range(n):
        if r >= m:
            break
        p = r + int(np.argmax(np.abs(A[r:, c])))
        if abs(A[p, c]) <= tol:
            continue
        A[[r, p]] = A[[p, r]]
        A[r] /= A[r, c]
        for q in range(m):
            if q != r:
                A[q] -= A[q, c] * A[r]
        piv.append(c)
        r += 1
    A = A[:r]
    A[np.abs(A) < tol] = 0.0
    near = np.abs(A - np.round(A)) < 1e-9          # site balances are integer rows
    A[near] = np.round(A[near])
    return A, piv


def conservation_laws(S_dyn, rs0, flow):
    """Left null space of the dynamic rate matrix (rows with a flow term excluded)."""
    n = S_dyn.shape[0]
    keep = [i for i in range(n) if flow[i] == 0.0]
    if not keep:
        return np.zeros((0, n)), []
    M = (S_dyn[keep] * np.asarray(rs0)[keep, None])
    cols = [j for j in range(M.shape[1]) if np.any(M[:, j] != 0.0)]
    if not cols:
        basis = np.eye(len(keep))
    else:
        u, sv, vt = np.linalg.svd(M[:, cols].T)
        rank = int(np.sum(sv > 1e-10 * max(float(sv.max()), 1.0)))
        basis = vt[rank:]
    if basis.shape[0] == 0:
        return np.zeros((0, n)), []
    R, piv = _rref_pivots(basis)
    C = np.zeros((R.shape[0], n))
    C[:, keep] = R
    return C, [keep[p] for p in piv]


def _rx_type(rxn, states_by_name, rate_model):
    typ = str(rxn.reac_type).upper()
    if typ == 'ARRHENIUS':
        return L.RX_ARRHENIUS, None
    if typ in ('ADSORPTION', 'DESORPTION'):
        side = rxn.reactants if typ == 'ADSORPTION' else rxn.products
        gas = [s for s in side if s.state_type == 'gas']
        if len(gas) != 1:
            raise ValueError('reaction %s: must have ONLY one gas-phase species adsorbing or desorbing '
                             '(reaction.py:137)' % rxn.name)
        g = gas[0]
        if g.mass is None:
            g.get_atoms()
        kads_c = rxn.area / np.sqrt(2.0 * np.pi * (g.mass * amutokg) * kB)
        if rate_model == 'patched' and g.inertia is not None:
            inertia = list(g.inertia)
            if len(inertia) == 3 and all(abs(k) > 0.001 for k in inertia):   # rate_constants.py:40-47
                from .constants.physical_constants import amuA2tokgm2
                theta = [h ** 2 / (8 * np.pi ** 2 * (I * amuA2tokgm2) * kB) for I in inertia]
                c0 = (kB ** 2 * rxn.area * 2 * np.pi ** 1.5 * (g.mass * amutokg)) / (h ** 3 * g.sigma * np.prod(theta))
                e = 3.5
            else:
                from .constants.physical_constants import amuA2tokgm2
                theta = h ** 2 / (8 * np.pi ** 2 * (max(inertia) * amuA2tokgm2) * kB)
                c0 = (kB ** 2 * rxn.area * 2 * np.pi * (g.mass * amutokg)) / (h ** 3 * g.sigma * theta)
                e = 3.0
            t = L.RX_ADS_KDES if typ == 'ADSORPTION' else L.RX_DES_KDES
            return t, (kads_c, c0, e)
        t = L.RX_ADS_KEQ if typ == 'ADSORPTION' else L.RX_DES_KEQ
        return t, (kads_c, 0.0, 0.0)
    # any other reac_type (e.g. 'scaling' in examples/COOxReactor/input_AuPd.json)
    # takes the Arrhenius branch whenever dGa_fwd != 0 (reaction.py:121); with no
    # barrier at all the reference raises, and so does this.
    ga = rxn.energy_forms().get('dGa_fwd')
    if typ != 'GHOST' and ga is not None and not (ga.is_constant() and float(ga) == 0.0):
        return L.RX_ARRHENIUS, None
    raise RuntimeError('Reaction with id %s has invalid `reaction.reac_type`, must be one of `arrhenius`, '
                       '`adsorption`, `desorption`, `ghost`' % rxn.name)


def _collect_clamps(form, acc):
    for cid, inner in form.clamps.items():
        if cid not in acc:
            _collect_clamps(inner, acc)
            acc[cid] = inner


def compile_system(system, tof_terms=(), descriptors=None, rate_model=None):
    """Build the device plan for `system` (a pycatkin_amd System)."""
    formulation = getattr(system, 'formulation', 'classic')
    rate_model = rate_model or getattr(system, 'rate_model', 'classic')
    states = system.states
    all_rxn = list(system.reactions)
    active = [r for r in all_rxn if str(system.reactions[r].reac_type).upper() != 'GHOST']
    if formulation == 'classic':
        species = sorted(states)
        ads, gas = set(), set()
        for r in all_rxn:
            rx = system.reactions[r]
            for s in rx.reactants + rx.products:
                if s.state_type in ('adsorbate', 'surface'):
                    ads.add(s.name)
                elif s.state_type == 'gas':
                    gas.add(s.name)
        ads_l = [s for s in species if s in ads]
        gas_l = [s for s in species if s in gas]
        cstr = system.reactor is not None and type(system.reactor).__name__ == 'CSTReactor'
        dyn = ads_l + (gas_l if cstr else [])
        fix = [] if cstr else gas_l
    elif formulation == 'patched':
        idx = system.index_map_ordered()
        species = idx
        gas_l = [s for s in idx if states[s].state_type == 'gas']
        dyn = [s for s in idx if states[s].state_type != 'gas']
        fix = gas_l
        cstr = False
    else:
        raise ValueError('unknown formulation %r' % formulation)
    NS, NF, R = len(dyn), len(fix), len(active)
    if NS < 1 or NS > 64:
        raise ValueError('network has %d dynamic species; plans hold 1..64 (solver kernels: 1..%d)'
                         % (NS, L.MAX_DYN))
    if R > L.MAX_RXN:
        raise ValueError('network has %d active reactions (max %d)' % (R, L.MAX_RXN))
    di = {s: i for i, s in enumerate(dyn)}
    fi = {s: i for i, s in enumerate(fix)}
    expf = np.zeros((R, NS), np.int32)
    expr = np.zeros((R, NS), np.int32)
    foldf = np.zeros((R, max(NF, 0)), np.int32)
    foldr = np.zeros((R, max(NF, 0)), np.int32)
    S = np.zeros((NS, R))
    for j, r in enumerate(active):
        rx = system.reactions[r]
        for side, e_dyn, e_fix, sgn in ((rx.reactants, expf, foldf, -1.0), (rx.products, expr, foldr, 1.0)):
            for s in side:
                if formulation == 'classic' and s.state_type not in ('adsorbate', 'surface', 'gas'):
                    continue                       # old_system.py:107-114 tracks only these types
                if s.name in di:
                    e_dyn[j, di[s.name]] += 1
                    if formulation == 'classic':
                        w = rx.scaling * ((1.0 / rx.area if rx.area else 0.0) if s.state_type == 'gas' else 1.0)
                        S[di[s.name], j] += sgn * w
                elif s.name in fi:
                    e_fix[j, fi[s.name]] += 1
        if formulation == 'patched':            # system.py:388-392 (assignment, products win)
            for s in rx.reactants:
                if s.name in di:
                    S[di[s.name], j] = -1.0
            for s in rx.products:
                if s.name in di:
                    S[di[s.name], j] = 1.0
    # dynamic-row coefficients
    dyn_blk = np.zeros((NS, 4))
    for i, s in enumerate(dyn):
        g = states[s].state_type == 'gas'
        cf = bartoPa if (g and formulation == 'classic') else 1.0
        if formulation == 'classic' and system.reactor is not None:
            rs0, rsT, fl = system.reactor.row_coefficients(not g)
        else:
            rs0, rsT, fl = 1.0, 0.0, 0.0
        dyn_blk[i] = (cf, rs0, rsT, fl)
    fix_cf = np.array([bartoPa if formulation == 'classic' else 1.0 for _ in fix])
    C, cpiv = conservation_laws(S, dyn_blk[:, 1], dyn_blk[:, 3])
    if C.shape[0] > L.MAX_CONS:
        raise ValueError('too many conservation laws (%d)' % C.shape[0])
    tof_idx = []
    for t in tof_terms:
        if t not in active:
            raise KeyError('TOF term %r is not an active reaction' % t)
        tof_idx.append(active.index(t))
    if len(tof_idx) > L.MAX_TOF:
        raise ValueError('too many TOF terms')

    # ---- energy program -----------------------------------------------------
    rx_int = np.zeros((R, 6), np.int32)
    rx_dbl = np.zeros((R, 3))
    forms = []
    for j, r in enumerate(active):
        rx = system.reactions[r]
        t, consts = _rx_type(rx, states, rate_model)
        rx_int[j, 0] = t
        rx_int[j, 1] = 1 if rx.reversible else 0
        rx_int[j, 5] = 0 if t == L.RX_ARRHENIUS else 1
        if consts is not None:
            rx_dbl[j] = consts
        en = rx.energy_forms()
        forms.append((en['dGa_fwd'], en['dGrxn'] if rx.reversible else None, en['dErxn']))
    prog = energy_program(forms, states, descriptors)
    if R:
        rx_int[:, 2:5] = prog["slots"]
    descriptors, D, NTH = prog['descriptors'], len(prog['descriptors']), prog['NTH']
    th_int, th_dbl, freqs = prog['th_int'], prog['th_dbl'], prog['freqs']
    reg_ptr, reg_clamp, reg_feat, reg_coef = prog['reg_ptr'], prog['reg_clamp'], prog['reg_feat'], prog['reg_coef']
    regs = prog['regs']
    th_found = prog['th_found']
    return _pack(system, formulation, rate_model, species, dyn, fix, active, all_rxn, descriptors, tof_terms,
                 th_int, reg_ptr, reg_clamp, reg_feat, rx_int, expf, expr, foldf, foldr, cpiv, tof_idx,
                 th_dbl, freqs, reg_coef, rx_dbl, S, dyn_blk, C, D, NTH, regs, R, NS, NF, fix_cf, th_found)


def energy_program(forms, states, descriptors=None):
    """Registers for a list of tuples of LinearForms (None = absent slot).

    Returns the packed program pieces and, in 'slots', the register index of
    every form (-1 for None)."""
    clamps = {}
    for tri in forms:
        for f in tri:
            if f is not None:
                _collect_clamps(f, clamps)
    desc_found, th_found = set(), []

    def scan(f):
        for k in f.terms:
            if k[0] == 'desc':
                desc_found.add(k[1])
            elif k[0] in ('vib', 'tran', 'rot') and k[1] not in th_found:
                th_found.append(k[1])
    for inner in clamps.values():
        scan(inner)
    for tri in forms:
        for f in tri:
            if f is not None:
                scan(f)
    if descriptors is None:
        descriptors = sorted(desc_found)
    else:
        descriptors = list(descriptors)
        missing = desc_found - set(descriptors)
        if missing:
            raise KeyError('energies use descriptors %s not given' % sorted(missing))
    D = len(descriptors)
    NTH = len(th_found)
    feat_base = 2 + D + 3 * NTH
    clamp_ids = sorted(clamps)
    reg_of_clamp = {cid: k for k, cid in enumerate(clamp_ids)}
    regs = [(clamps[cid], 1) for cid in clamp_ids]
    width = max((len(t) for t in forms), default=0)
    slots = np.full((len(forms), width), -1, np.int32)
    for j, tri in enumerate(forms):
        for q, f in enumerate(tri):
            if f is not None:
                slots[j, q] = len(regs)
                regs.append((f, 0))
    kind_off = {'vib': 0, 'tran': 1, 'rot': 2}
    reg_ptr, reg_clamp, reg_feat, reg_coef = [0], [], [], []
    for r_i, (f, cl) in enumerate(regs):
        for key, coef in f.terms.items():
            if coef == 0.0:
                continue
            if key == ('1',):
                fidx = 0
            elif key == ('T',):
                fidx = 1
            elif key[0] == 'desc':
                fidx = 2 + descriptors.index(key[1])
            elif key[0] in kind_off:
                fidx = 2 + D + 3 * th_found.index(key[1]) + kind_off[key[0]]
            elif key[0] == 'clamp':
                fidx = feat_base + reg_of_clamp[key[1]]
                if reg_of_clamp[key[1]] >= r_i:
                    raise RuntimeError('clamp register ordering')
            else:
                raise KeyError(key)
            reg_feat.append(fidx)
            reg_coef.append(float(coef))
        reg_ptr.append(len(reg_feat))
        reg_clamp.append(cl)
    refs = {}
    for f, _ in regs:
        refs.update(f.refs)
    th_int = np.zeros((NTH, 4), np.int32)
    th_dbl = np.zeros((NTH, 5))
    freqs = []
    for s_i, sname in enumerate(th_found):
        # the State object the form was built from: a reaction-derived
        # reaction's energies come from its base system's states
        # (reaction.py:312-339), which may share names with this system's own
        # (Butadiene: the DFT base's 'H2' vs the MKM's mass-only 'H2')
        st = refs[sname] if sname in refs else states[sname]
        kind = 0
        uf = np.zeros(0)
        if st.Gvibr is None:
            uf = st.use_freq()
            if np.sum(uf) != 0.0:
                kind |= L.TH_VIB
        st.calc_zpe()
        if st.state_type == 'gas':
            kind |= L.TH_GAS
            if st.mass is None or st.inertia is None:
                st.get_atoms()
        th_int[s_i] = (kind, len(freqs), len(uf) if kind & L.TH_VIB else 0, st.shape or 0)
        if kind & L.TH_VIB:
            freqs.extend(float(x) for x in uf)
        th_dbl[s_i] = (st.Gzpe or 0.0, st.mass or 0.0, st.sigma or 1.0,
                       st.rot_inertia() if kind & L.TH_GAS else 1.0, np.nan)
    return dict(slots=slots, descriptors=descriptors, NTH=NTH, th_int=th_int, th_dbl=th_dbl, freqs=freqs,
                reg_ptr=reg_ptr, reg_clamp=reg_clamp, reg_feat=reg_feat, reg_coef=reg_coef, regs=regs,
                th_found=th_found)


def _blobs(D, NTH, NREG, R, NS, NF, NCONS, iblocks, dblocks, NTOF):
    hdr = np.zeros(L.IP_MIN, np.int32)
    hdr[L.I_VERSION] = L.ABI_VERSION
    hdr[L.I_NDESC], hdr[L.I_NTH], hdr[L.I_NREG], hdr[L.I_NRXN] = D, NTH, NREG, R
    hdr[L.I_NDYN], hdr[L.I_NFIX], hdr[L.I_NCONS], hdr[L.I_NTOF] = NS, NF, NCONS, NTOF
    off = L.IP_MIN
    for k, b in enumerate(iblocks):
        hdr[L.I_OFF_TH + k] = off
        off += b.size
    doff = 0
    for k, b in enumerate(dblocks):
        hdr[L.I_HDR + k] = doff
        doff += b.size
    ip = np.concatenate([hdr] + [np.asarray(b, np.int32).ravel() for b in iblocks]).astype(np.int32)
    dp = np.concatenate([np.asarray(b, np.float64).ravel() for b in dblocks]) if doff else np.zeros(1)
    return ip, dp


def _pack(system, formulation, rate_model, species, dyn, fix, active, all_rxn, descriptors, tof_terms,
          th_int, reg_ptr, reg_clamp, reg_feat, rx_int, expf, expr, foldf, foldr, cpiv, tof_idx,
          th_dbl, freqs, reg_coef, rx_dbl, S, dyn_blk, C, D, NTH, regs, R, NS, NF, fix_cf, th_found):
    iblocks = [th_int.ravel(), np.array(reg_ptr + reg_clamp + reg_feat, np.int32), rx_int.ravel(),
               expf.ravel(), expr.ravel(), foldf.ravel(), foldr.ravel(), np.array(cpiv, np.int32),
               np.array(tof_idx, np.int32)]
    dblocks = [th_dbl.ravel(), np.array(freqs, float), np.array(reg_coef, float), rx_dbl.ravel(), S.ravel(),
               dyn_blk.ravel(), C.ravel()]
    ip, dp = _blobs(D, NTH, len(regs), R, NS, NF, C.shape[0], iblocks, dblocks, len(tof_idx))
    # defaults from the system's start / inflow states
    start = dict(system.start_state_values())
    inflow = dict(system.inflow_state_values())
    if formulation == 'patched':
        y_all = system.initial_vector()
        pos = {s: i for i, s in enumerate(species)}
        y0 = np.array([y_all[pos[s]] for s in dyn])
        fixd = np.array([y_all[pos[s]] for s in fix])
    else:
        y0 = np.array([float(start.get(s, 0.0)) for s in dyn])
        fixd = np.array([float(start.get(s, 0.0)) for s in fix])
    inflow_d = np.array([float(inflow.get(s, 0.0)) for s in dyn])
    return NetworkPlan(ip=ip, dp=dp, formulation=formulation, rate_model=rate_model, species=species, dyn=dyn,
                       fix=fix, reactions=active, all_reactions=all_rxn, descriptors=descriptors,
                       tof_terms=list(tof_terms), conc_factor=dyn_blk[:, 0].copy(), fix_conc_factor=fix_cf,
                       y0_default=y0, fix_default=fixd, inflow_default=inflow_d, conservation=C,
                       extra=dict(cpiv=cpiv, S=S, thermo_states=th_found, nreg=len(regs)))


def compile_forms(forms, states, descriptors=None):
    """Energy-only plan (NDYN = NRXN = 0) whose registers end with `forms`;
    returns (ip, dp, register index of each form, descriptor names)."""
    prog = energy_program([(f,) for f in forms], states, descriptors)
    iblocks = [prog['th_int'].ravel(), np.array(prog['reg_ptr'] + prog['reg_clamp'] + prog['reg_feat'], np.int32),
               np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int32),
               np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int32)]
    dblocks = [prog['th_dbl'].ravel(), np.array(prog['freqs'], float), np.array(prog['reg_coef'], float),
               np.zeros(0), np.zeros(0), np.zeros(0), np.zeros(0)]
    ip, dp = _blobs(len(prog['descriptors']), prog['NTH'], len(prog['regs']), 0, 0, 0, 0, iblocks, dblocks, 0)
    return ip, dp, [int(s[0]) for s in prog['slots']], prog['descriptors']


def structural_digest(ip, dp):
    """FNV-1a 64 of the solver-side structure of a plan (NS, R, NCONS,
    exponents, stoichiometry, dynamic-row coefficients, conservation rows and
    pivots) -- the key pck_network_create matches against the compiled-in
    networks of csrc/networks.h (same byte order as mk_kernels.hip)."""
    ip = np.asarray(ip, np.int32)
    dp = np.asarray(dp, np.float64)
    NS, R, NC = int(ip[L.I_NDYN]), int(ip[L.I_NRXN]), int(ip[L.I_NCONS])
    parts = [np.array([NS, R, NC], np.int32),
             ip[ip[L.I_OFF_EXPF]: ip[L.I_OFF_EXPF] + R * NS],
             ip[ip[L.I_OFF_EXPR]: ip[L.I_OFF_EXPR] + R * NS],
             dp[ip[L.I_HDR + L.D_STOICH]: ip[L.I_HDR + L.D_STOICH] + NS * R],
             dp[ip[L.I_HDR + L.D_DYN]: ip[L.I_HDR + L.D_DYN] + NS * 4],
             dp[ip[L.I_HDR + L.D_CONS]: ip[L.I_HDR + L.D_CONS] + NC * NS],
             ip[ip[L.I_OFF_CPIV]: ip[L.I_OFF_CPIV] + NC]]
    h = 0xcbf29ce484222325
    for part in parts:
        for byte in np.ascontiguousarray(part).tobytes():
            h ^= byte
            h = (h * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h
