"""Device execution of a compiled network through the C-ABI.

PyTorch-ROCm is used for device buffers and the current HIP stream only;
every number is computed by the HIP kernels of libpycatkin_amd.so.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib as L
from .constants.physical_constants import bartoPa


_POISON = os.environ.get('PCK_DEBUG_POISON') == '1'


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError('pycatkin_amd needs a HIP device (MI355X); torch.cuda.is_available() is False '
                           'and there is no CPU fallback')
    return torch


def _stream(torch):
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


class DeviceNetwork:
    """A NetworkPlan uploaded to the current device (pck_network_create)."""

    def __init__(self, ip, dp, plan=None):
        self.lib = L.load()
        self.torch = _torch()
        self.plan = plan
        self._ip = np.ascontiguousarray(ip, np.int32)
        self._dp = np.ascontiguousarray(dp, np.float64)
        h = C.c_void_p()
        L.check(self.lib.pck_network_create(self._ip.ctypes.data_as(C.c_void_p), self._ip.size,
                                            self._dp.ctypes.data_as(C.c_void_p), self._dp.size, C.byref(h)))
        self.h = h
        dims = (C.c_int32 * 11)()
        L.check(self.lib.pck_network_dims(self.h, dims))
        (self.D, self.NTH, self.NREG, self.NRXN, self.NDYN, self.NFIX, self.NCONS, self.NTOF,
         self.nfeat, self.compiled_plan) = list(dims)[:10]

    def plan_id(self):
        """Solver plan of the last lane solve: a compiled-in id (csrc/networks.h),
        100 = hipRTC-specialised at run time (csrc/mk_jit.h), 0 = runtime plan."""
        dims = (C.c_int32 * 11)()
        L.check(self.lib.pck_network_dims(self.h, dims))
        return int(dims[9])

    def group_kernel(self):
        """Kernel of the last lane-group solve: 0 compiled-in record tables,
        1 hipRTC exact-size record tables, 2 hipRTC with the network compiled
        in (mk_group.h: ct_rhs / ct_jac)."""
        dims = (C.c_int32 * 11)()
        L.check(self.lib.pck_network_dims(self.h, dims))
        return int(dims[10])

    def group_lanes(self):
        """Lanes per condition of the last lane-group solve: 4 (quad-group
        kernel), 16, 32 or 64 (group width G); 0 before any group solve."""
        g = C.c_int32(0)
        L.check(self.lib.pck_network_group_lanes(self.h, C.byref(g)))
        return int(g.value)

    def set_plan_mode(self, mode):
        """A/B switch: 0 / False = auto, 1 / True = runtime plan (never the
        compiled-in one), 2 = lane-group solver."""
        L.check(self.lib.pck_network_set_plan_mode(self.h, int(mode)))

    @classmethod
    def from_plan(cls, plan):
        return cls(plan.ip, plan.dp, plan)

    def __del__(self):
        try:
            if getattr(self, 'h', None) is not None and self.h.value:
                self.lib.pck_network_destroy(self.h)
                self.h = None
        except Exception:
            pass

    # -- inputs -----------------------------------------------------------------
    def _col(self, x, n, name):
        """(tensor, stride): a scalar broadcasts with stride 0."""
        torch = self.torch
        t = torch.as_tensor(x, dtype=torch.float64, device='cuda')
        if t.dim() == 0 or t.numel() == 1:
            return t.reshape(1).contiguous(), 0
        t = t.reshape(-1).contiguous()
        if t.numel() != n:
            raise ValueError('%s has %d entries for %d conditions' % (name, t.numel(), n))
        return t, 1

    def _mat(self, x, rows, n, name):
        """[rows, n] matrix or a [rows] column broadcast to every condition."""
        torch = self.torch
        if rows == 0 or x is None:
            return torch.zeros(1, dtype=torch.float64, device='cuda'), 0, 0
        t = torch.as_tensor(x, dtype=torch.float64, device='cuda')
        if t.dim() == 1:
            if t.numel() != rows:
                raise ValueError('%s: expected %d rows' % (name, rows))
            return t.contiguous(), 1, 0
        if tuple(t.shape) != (rows, n):
            raise ValueError('%s: expected shape (%d, %d), got %s' % (name, rows, n, tuple(t.shape)))
        t = t.contiguous()
        return t, n, 1

    def conditions(self, n, T, p, desc=None, fixc=None, y0=None, inflow=None):
        keep = []
        c = L.Conditions()
        c.n = int(n)
        tT, c.sT = self._col(T, n, 'T')
        tp, c.sp = self._col(p, n, 'p')
        keep += [tT, tp]
        c.T, c.p = _ptr(tT), _ptr(tp)
        td, c.ld_desc, c.s_desc = self._mat(desc, self.D, n, 'descriptors')
        tf, c.ld_fix, c.s_fix = self._mat(fixc, self.NFIX, n, 'fixed species')
        keep += [td, tf]
        c.desc, c.fixc = _ptr(td), _ptr(tf)
        if y0 is not None:
            ty, c.ld_y0, c.s_y0 = self._mat(y0, self.NDYN, n, 'y0')
            keep.append(ty)
            c.y0 = _ptr(ty)
        if inflow is not None:
            ti, c.ld_in, c.s_in = self._mat(inflow, self.NDYN, n, 'inflow')
            keep.append(ti)
            c.inflow = _ptr(ti)
        return c, keep

    # -- kernels ------------------------------------------------------------------
    def energies(self, n, T, p, desc=None):
        torch = self.torch
        c, keep = self.conditions(n, T, p, desc)
        out = torch.empty((max(self.NREG, 1), max(n, 1)), dtype=torch.float64, device='cuda')
        L.check(self.lib.pck_energies(self.h, C.byref(c), _ptr(out), out.shape[1], _stream(torch)))
        return out[:self.NREG, :n]

    def rate_constants(self, n, T, p, desc=None):
        torch = self.torch
        c, keep = self.conditions(n, T, p, desc)
        kf = torch.empty((max(self.NRXN, 1), max(n, 1)), dtype=torch.float64, device='cuda')
        kr = torch.empty_like(kf)
        L.check(self.lib.pck_rate_constants(self.h, C.byref(c), _ptr(kf), _ptr(kr), kf.shape[1], _stream(torch)))
        return kf[:self.NRXN, :n], kr[:self.NRXN, :n]

    def species_rates(self, n, T, p, y, kf, kr, desc=None, fixc=None, inflow=None):
        torch = self.torch
        c, keep = self.conditions(n, T, p, desc, fixc, None, inflow)
        y = torch.as_tensor(y, dtype=torch.float64, device='cuda').reshape(self.NDYN, n).contiguous()
        kf, kr = kf.contiguous(), kr.contiguous()
        out = torch.empty_like(y)
        L.check(self.lib.pck_species_rates(self.h, C.byref(c), _ptr(kf), _ptr(kr), kf.shape[1], _ptr(y), n,
                                           _ptr(out), _stream(torch)))
        return out

    def reaction_rates(self, n, T, p, y, kf, kr, desc=None, fixc=None):
        """pck_reaction_rates: (rf, rr) [NRXN, n] at states y [NDYN, n]."""
        torch = self.torch
        c, keep = self.conditions(n, T, p, desc, fixc, None, None)
        y = torch.as_tensor(y, dtype=torch.float64, device='cuda').reshape(self.NDYN, n).contiguous()
        kf, kr = kf.contiguous(), kr.contiguous()
        rf = torch.empty((max(self.NRXN, 1), n), dtype=torch.float64, device='cuda')
        rr = torch.empty_like(rf)
        L.check(self.lib.pck_reaction_rates(self.h, C.byref(c), _ptr(kf), _ptr(kr), kf.shape[1], _ptr(y), n, _ptr(rf),
                                            _ptr(rr), n, _stream(torch)))
        return rf[:self.NRXN], rr[:self.NRXN]

    def jacobian(self, n, T, p, y, kf, kr, desc=None, fixc=None, inflow=None):
        torch = self.torch
        c, keep = self.conditions(n, T, p, desc, fixc, None, inflow)
        y = torch.as_tensor(y, dtype=torch.float64, device='cuda').reshape(self.NDYN, n).contiguous()
        kf, kr = kf.contiguous(), kr.contiguous()
        out = torch.empty((self.NDYN * self.NDYN, n), dtype=torch.float64, device='cuda')
        L.check(self.lib.pck_jacobian(self.h, C.byref(c), _ptr(kf), _ptr(kr), kf.shape[1], _ptr(y), n,
                                      _ptr(out), _stream(torch)))
        return out.reshape(self.NDYN, self.NDYN, n)

    @staticmethod
    def params(t_end, t0=0.0, rtol=1e-8, atol=1e-10, max_steps=100000, newton=False, newton_iters=60,
               activity=False, drc_eps=1e-3, retry=None, wave_order=0, root_dist=0.0, screen=None):
        """retry = (rtol, atol): with newton, the conditions whose polish meets a
        degenerate root (status 4) are integrated again at these tolerances
        and report that transient end (pck_solve_params.retry_rtol).
        screen = (rtol, margin): the screening pass of steady solves
        (pck_solve_params.screen_rtol / screen_margin)."""
        p = L.SolveParams()
        p.t0, p.t_end, p.rtol, p.atol = float(t0), float(t_end), float(rtol), float(atol)
        p.max_steps, p.newton, p.newton_iters = int(max_steps), int(bool(newton)), int(newton_iters)
        p.want_activity, p.drc_eps = int(bool(activity)), float(drc_eps)
        if retry is not None:
            p.retry_rtol, p.retry_atol = float(retry[0]), float(retry[1])
        p.wave_order = int(wave_order)     # 0 auto, 1 on, -1 off (pck_solve_params.wave_order)
        p.root_dist = float(root_dist)     # newton: the root only if the transient reached it
        if screen is not None:
            p.screen_rtol, p.screen_margin = float(screen[0]), float(screen[1])
        return p

    def solve(self, n, T, p, y0, desc=None, fixc=None, inflow=None, want_k=False, out=None, t_out=None, **kw):
        """pck_solve: returns dict(y [NS,n], tof [n] (or activity), status, nsteps)
        and, with t_out (ascending sample times), traj [n_out, NS, n]."""
        torch = self.torch
        c, keep = self.conditions(n, T, p, desc, fixc, y0, inflow)
        prm = self.params(**kw)
        tt = None
        if t_out is not None:
            tt = torch.as_tensor(np.asarray(t_out, float).ravel(), dtype=torch.float64, device='cuda').contiguous()
            if tt.numel() and bool((tt[1:] < tt[:-1]).any()):
                raise ValueError('t_out must be ascending')
            prm.t_out, prm.n_out = _ptr(tt).value, int(tt.numel())
        if out is None:
            out = dict(y=torch.empty((self.NDYN, n), dtype=torch.float64, device='cuda'),
                       tof=torch.empty(n, dtype=torch.float64, device='cuda'),
                       status=torch.empty(n, dtype=torch.int32, device='cuda'),
                       nsteps=torch.empty(n, dtype=torch.int32, device='cuda'))
            if want_k:
                out['kf'] = torch.empty((self.NRXN, n), dtype=torch.float64, device='cuda')
                out['kr'] = torch.empty_like(out['kf'])
        if _POISON:
            # diagnostics (PCK_DEBUG_POISON=1): every output starts as NaN / -7,
            # so an element the kernels never write shows in the result
            for k, v in out.items():
                v.fill_(float('nan') if v.is_floating_point() else -7)
        o = L.Outputs()
        o.y, o.ld_y = _ptr(out['y']), n
        o.tof, o.status, o.nsteps = _ptr(out['tof']), _ptr(out['status']), _ptr(out['nsteps'])
        if 'kf' in out:
            o.kf, o.kr, o.ld_k = _ptr(out['kf']), _ptr(out['kr']), n
        if tt is not None and tt.numel():
            # samples a failed solve never reaches stay NaN
            out['traj'] = torch.full((tt.numel(), self.NDYN, n), float('nan'), dtype=torch.float64, device='cuda')
            o.traj, o.ld_traj = _ptr(out['traj']), n
        L.check(self.lib.pck_solve(self.h, C.byref(c), C.byref(prm), C.byref(o), _stream(torch)))
        return out

    def drc(self, n, T, p, y0, desc=None, fixc=None, inflow=None, **kw):
        torch = self.torch
        c, keep = self.conditions(n, T, p, desc, fixc, y0, inflow)
        prm = self.params(**kw)
        xi = torch.zeros((max(self.NRXN, 1), n), dtype=torch.float64, device='cuda')
        tof0 = torch.empty(n, dtype=torch.float64, device='cuda')
        st = torch.empty(n, dtype=torch.int32, device='cuda')
        ns = torch.empty(n, dtype=torch.int32, device='cuda')
        L.check(self.lib.pck_drc(self.h, C.byref(c), C.byref(prm), _ptr(xi), n, _ptr(tof0), _ptr(st), _ptr(ns),
                                 _stream(torch)))
        return dict(xi=xi[:self.NRXN], tof0=tof0, status=st, nsteps=ns)


_form_cache = {}


def descriptor_values(dnames, T, desc=None):
    """The descriptor column of one condition at temperature T: a
    temperature-keyed user energy ('@T:' descriptor, energy.tkeyed) is looked
    up in its table at T (KeyError on a missing T, like the reference's
    dErxn_user[T], reaction.py:228-262); any other descriptor comes from
    `desc` (ValueError if it is not given)."""
    from .energy import TKEYED
    given = [k for k in dnames if not k.startswith('@T:')]
    if given and desc is None:
        raise ValueError('forms depend on descriptors %s; pass desc=' % given)
    return np.array([TKEYED[k][float(T)] if k.startswith('@T:') else desc[k] for k in dnames], float)


def evaluate_forms(forms, T, p, states=None, desc=None):
    """Evaluate LinearForms (eV) for one condition on the device (kernel 1)."""
    from .network import compile_forms
    states_map = {s.name: s for s in (states or [])}
    ip, dp, regs, dnames = compile_forms(forms, states_map)
    d = None if not dnames else descriptor_values(dnames, T, desc)
    net = DeviceNetwork(ip, dp)
    vals = net.energies(1, float(T), float(p), d).cpu().numpy()[:, 0]
    return [float(vals[r]) for r in regs]


def single_reaction_rate_constants(rxn, T, p):
    """Reaction.calc_rate_constants for one condition through kernel (1)."""
    from .network import NetworkPlan  # noqa: F401
    from .classes.system import System
    from .classes.reactor import InfiniteDilutionReactor
    s = System()
    seen = {}
    for st in list(rxn.reactants) + list(rxn.products) + list(rxn.TS or []):
        seen[st.name] = st
    for st in seen.values():
        s.add_state(st)
    s.add_reaction(rxn)
    s.add_reactor(InfiniteDilutionReactor())
    kf, kr = s.rate_constants_batch(T=[float(T)], p=float(p))
    return float(kf[0, 0]), float(kr[0, 0])
