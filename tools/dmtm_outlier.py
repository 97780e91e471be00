"""Diagnostic (GPU): the DMTM DRC bench grid's slowest condition (index 2297,
T 622.22 K, p 644 947 Pa) and two neighbours as plain solves at the input
tolerances; with a PCK_TRACE build (PCK_LIB=...) the step trace of the first
into gpurun_out/r4v_trace.npy.  Run per variant: PCK_GRP_CT=0, PCK_JIT=0."""
import ctypes as C, os, sys, numpy as np
sys.path.insert(0, '/root/repo')
import pycatkin_amd as P
from pycatkin_amd import _lib as L
s = P.read_from_input_file('/root/repo/tests/golden/inputs/DMTM/input.json')
TT, pp = np.meshgrid(np.linspace(400.0, 800.0, 64), np.logspace(4.0, 6.0, 64), indexing='ij')
T, p = TT.ravel(), pp.ravel()
ks = [2297, 2296, 2298]
lib = L.load()
tr = hasattr(lib, 'pck_trace_set')
if tr:
    lib.pck_trace_set.argtypes = [C.c_longlong]
    lib.pck_trace_get.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    L.check(lib.pck_trace_set(0))
b = s.solve_batch(T=T[ks], p=p[ks], tof_terms=('r5', 'r9'))
net = s.device(('r5', 'r9'))
print(os.environ.get('PCK_GRP_CT'), os.environ.get('PCK_JIT'), 'base nsteps', b['nsteps'], b['status'], 'group kernel', net.group_kernel() if hasattr(net, 'group_kernel') else None, flush=True)
if tr:
    buf = np.zeros(8192 * 8); pos = C.c_int()
    L.check(lib.pck_trace_get(buf.ctypes.data_as(C.c_void_p), C.byref(pos)))
    rec = buf.reshape(8192, 8)[:min(pos.value, 8192)]
    np.save('gpurun_out/r4v_trace.npy', rec)
    print('trace records', pos.value)
