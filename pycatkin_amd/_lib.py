"""ctypes binding of the C-ABI in include/pycatkin_amd.h (libpycatkin_amd.so).

This is the ONLY compute path of the package: there is no CPU fallback.  If
the shared library is missing or the process has no HIP device the calls
raise instead of silently computing something else.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PCK_LIB selects an alternative in-tree build (A/B experiments of tools/ab_variants.sh)
LIB_PATH = os.environ.get('PCK_LIB') or os.path.join(_HERE, 'libpycatkin_amd.so')

# symbols declared in include/pycatkin_amd.h (checked by tests/test_capi.py)
EXPORTED = ('pck_abi_version', 'pck_last_error', 'pck_network_create', 'pck_network_destroy',
            'pck_network_dims', 'pck_network_group_lanes', 'pck_network_set_plan_mode', 'pck_energies', 'pck_rate_constants', 'pck_species_rates',
            'pck_reaction_rates', 'pck_jacobian', 'pck_solve', 'pck_drc')

ABI_VERSION = 6

# header slot indices (must match the enums of include/pycatkin_amd.h)
I_VERSION, I_NDESC, I_NTH, I_NREG, I_NRXN, I_NDYN, I_NFIX, I_NCONS, I_NTOF = range(9)
I_OFF_TH, I_OFF_REG, I_OFF_RX, I_OFF_EXPF, I_OFF_EXPR, I_OFF_FOLDF, I_OFF_FOLDR, I_OFF_CPIV, I_OFF_TOF = range(9, 18)
I_HDR = 18
D_TH, D_FREQ, D_REGCOEF, D_RX, D_STOICH, D_DYN, D_CONS = range(7)
D_NBLK = 7
IP_MIN = I_HDR + D_NBLK

RX_ARRHENIUS, RX_ADS_KEQ, RX_DES_KEQ, RX_ADS_KDES, RX_DES_KDES = range(5)
TH_VIB, TH_GAS = 1, 2
MAX_DYN, MAX_DYN_LANE, MAX_RXN, MAX_CONS, MAX_TOF = 64, 8, 256, 4, 16
PLAN_AUTO, PLAN_RUNTIME, PLAN_GROUP = 0, 1, 2
ST_OK, ST_MAXSTEPS, ST_STEPFAIL, ST_NONFINITE, ST_NEWTON, ST_NEWTON_LOOSE, ST_DRC_MIXED = range(7)
E_ARG, E_HIP, E_SIZE = -1, -2, -3


class Conditions(C.Structure):
    _fields_ = [('n', C.c_int64),
                ('T', C.c_void_p), ('sT', C.c_int64),
                ('p', C.c_void_p), ('sp', C.c_int64),
                ('desc', C.c_void_p), ('ld_desc', C.c_int64), ('s_desc', C.c_int64),
                ('fixc', C.c_void_p), ('ld_fix', C.c_int64), ('s_fix', C.c_int64),
                ('y0', C.c_void_p), ('ld_y0', C.c_int64), ('s_y0', C.c_int64),
                ('inflow', C.c_void_p), ('ld_in', C.c_int64), ('s_in', C.c_int64)]


class SolveParams(C.Structure):
    _fields_ = [('t0', C.c_double), ('t_end', C.c_double), ('rtol', C.c_double), ('atol', C.c_double),
                ('max_steps', C.c_int32), ('newton', C.c_int32), ('newton_iters', C.c_int32),
                ('want_activity', C.c_int32), ('drc_eps', C.c_double), ('t_out', C.c_void_p), ('n_out', C.c_int64),
                ('retry_rtol', C.c_double), ('retry_atol', C.c_double), ('wave_order', C.c_int32),
                ('root_dist', C.c_double), ('screen_rtol', C.c_double), ('screen_margin', C.c_double)]


class Outputs(C.Structure):
    _fields_ = [('y', C.c_void_p), ('ld_y', C.c_int64), ('tof', C.c_void_p), ('status', C.c_void_p),
                ('nsteps', C.c_void_p), ('kf', C.c_void_p), ('kr', C.c_void_p), ('ld_k', C.c_int64),
                ('traj', C.c_void_p), ('ld_traj', C.c_int64)]


_lib = None


def load():
    """Load libpycatkin_amd.so (built by __graft_entry__.build()); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(LIB_PATH):
        raise RuntimeError('pycatkin_amd: %s not found -- run `python -c "import __graft_entry__ as g; g.build()"` '
                           '(hipcc --offload-arch=gfx950); there is no CPU fallback' % LIB_PATH)
    # torch first: its HIP runtime (libamdhip64.so.7, bundled with the wheel) is
    # then the one our library's libamdhip64.so.7 dependency binds to, so the
    # process has a single HIP/HSA runtime and device buffers are shared.
    import torch  # noqa: F401
    lib = C.CDLL(LIB_PATH)
    vp, i64, i32p = C.c_void_p, C.c_int64, C.POINTER(C.c_int32)
    lib.pck_abi_version.restype = C.c_int
    lib.pck_last_error.restype = C.c_char_p
    lib.pck_network_create.argtypes = [vp, i64, vp, i64, C.POINTER(vp)]
    lib.pck_network_destroy.argtypes = [vp]
    lib.pck_network_dims.argtypes = [vp, i32p]
    lib.pck_network_group_lanes.argtypes = [vp, i32p]
    lib.pck_network_set_plan_mode.argtypes = [vp, C.c_int]
    lib.pck_energies.argtypes = [vp, C.POINTER(Conditions), vp, i64, vp]
    lib.pck_rate_constants.argtypes = [vp, C.POINTER(Conditions), vp, vp, i64, vp]
    lib.pck_species_rates.argtypes = [vp, C.POINTER(Conditions), vp, vp, i64, vp, i64, vp, vp]
    lib.pck_jacobian.argtypes = [vp, C.POINTER(Conditions), vp, vp, i64, vp, i64, vp, vp]
    lib.pck_reaction_rates.argtypes = [vp, C.POINTER(Conditions), vp, vp, i64, vp, i64, vp, vp, i64, vp]
    lib.pck_solve.argtypes = [vp, C.POINTER(Conditions), C.POINTER(SolveParams), C.POINTER(Outputs), vp]
    lib.pck_drc.argtypes = [vp, C.POINTER(Conditions), C.POINTER(SolveParams), vp, i64, vp, vp, vp, vp]
    for name in EXPORTED:
        if name not in ('pck_last_error',):
            getattr(lib, name).restype = C.c_int
    if lib.pck_abi_version() != ABI_VERSION:
        raise RuntimeError('pycatkin_amd: ABI mismatch (library %d, python %d)' % (lib.pck_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        msg = load().pck_last_error().decode(errors='replace')
        raise RuntimeError('pycatkin_amd C-ABI error %d: %s' % (rc, msg))
