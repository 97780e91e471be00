"""Diagnostic: per-iteration trace of the lane solver's Newton polish on
volcano fixture nodes (needs the PCK_TRACE build: tools/ab_build.sh trace
-DPCK_TRACE; run as `python tools/trace_newton.py --lib
pycatkin_amd/_ab/lib_trace.so K [K ...]` with K fixture node indices).

For each node: the device transient (STEADY_TRANSIENT, to t_end), then
Newton alone from that state (t_end = t0) with one record per iteration
[it, rel, alpha, z...] and an exit record [-1, converged, min z, resolved].
Writes gpurun_out/trace_newton.json; compare with a numpy restatement of
the same iteration from the same start (the transient end is stored too).
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    args = sys.argv[1:]
    if '--lib' in args:
        i = args.index('--lib')
        os.environ['PCK_LIB'] = os.path.abspath(args[i + 1])
        del args[i:i + 2]
    import torch  # noqa: F401
    import pycatkin_amd as P
    from pycatkin_amd import _lib as L
    from pycatkin_amd.classes.system import STEADY_TRANSIENT
    from pycatkin_amd.functions.volcano import set_volcano_energies
    lib = L.load()
    lib.pck_trace_set.argtypes = [C.c_longlong]
    lib.pck_trace_get.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    split = '--split' in args          # K index the split fixture (tests/golden/split_fixture.npz) instead
    if split:
        args.remove('--split')
        sf = np.load(os.path.join(ROOT, 'tests', 'golden', 'split_fixture.npz'))
    fx = dict(np.load(os.path.join(ROOT, 'tests', 'golden', 'volcano_fixture.npz')))
    lo, hi, G = fx['grid']
    be = np.linspace(lo, hi, int(G))
    s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    plan = s.plan(('CO_ox',))
    out = {'dyn': list(plan.dyn)}
    for k in (int(a) for a in args):
        if split:
            desc = {'ECO': sf['ECO'][k:k + 1], 'EO': sf['EO'][k:k + 1]}
        else:
            desc = {'ECO': be[fx['i'][k:k + 1]], 'EO': be[fx['j'][k:k + 1]]}
        kw = dict(T=np.full(1, 600.0), desc=desc, tof_terms=('CO_ox',))
        a = s.solve_batch(steady=False, rtol=STEADY_TRANSIENT[0], atol=STEADY_TRANSIENT[1], **kw)
        L.check(lib.pck_trace_set(0))
        d = s.solve_batch(steady=True, retry=None, y0=a['y'], t0=0.0, t_end=0.0, **kw)
        buf = np.zeros(8192 * 8)
        pos = C.c_int()
        L.check(lib.pck_trace_get(buf.ctypes.data_as(C.c_void_p), C.byref(pos)))
        rec = buf.reshape(8192, 8)[:min(pos.value, 8192)]
        out[k] = dict(yT=a['y'][:, 0].tolist(), status=int(d['status'][0]), y=d['y'][:, 0].tolist(),
                      records=rec.tolist())
        print(k, 'status', int(d['status'][0]), flush=True)
        for r in rec:
            print('   ' + ' '.join('%.6e' % v for v in r), flush=True)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, 'gpurun_out', 'trace_newton.json'), 'w'))


if __name__ == '__main__':
    main()
