"""Diagnostic: per-step trace of the lane-group integrator for a few
conditions of the synthetic config (needs the PCK_TRACE build:
tools/ab_build.sh trace -DPCK_TRACE; run with PCK_LIB=pycatkin_amd/_ab/lib_trace.so).

    python tools/trace_group.py IDX [IDX ...]      (indices of the bench's 65536-condition synthetic set)
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401
    from pycatkin_amd import _lib as L
    from pycatkin_amd.functions.synthetic import synthetic_system
    lib = L.load()
    lib.pck_trace_set.argtypes = [C.c_longlong]
    lib.pck_trace_get.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    out = {}
    if sys.argv[1] == 'dmtm':                    # tools/trace_group.py dmtm T rtol atol
        import pycatkin_amd as P
        sim = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'DMTM', 'input.json'))
        jobs = [(float(sys.argv[2]), dict(T=np.array([float(sys.argv[2])]), tof_terms=('r5', 'r9'), steady=True,
                                          rtol=float(sys.argv[3]), atol=float(sys.argv[4])))]
    else:
        sim, _ = synthetic_system()
        D = np.random.default_rng(0).uniform(-0.5, 0.5, (65536, 4))     # the bench's synthetic set
        jobs = [(int(a), dict(T=np.full(1, 500.0), desc={'D%d' % k: D[int(a):int(a) + 1, k] for k in range(4)},
                              tof_terms=('R0',), steady=True)) for a in sys.argv[1:]]
    for idx, kw in jobs:
        L.check(lib.pck_trace_set(0))           # the in-call index of the one condition solved
        r = sim.solve_batch(max_steps=int(os.environ.get('MAXSTEPS', 20000)), **kw)
        buf = np.zeros(8192 * 8)
        pos = C.c_int()
        L.check(lib.pck_trace_get(buf.ctypes.data_as(C.c_void_p), C.byref(pos)))
        rec = buf.reshape(8192, 8)
        k = pos.value
        order = np.arange(k)[-8192:] % 8192
        rec = rec[order]
        acc = rec[:, 3] <= 1.0
        out[idx] = dict(status=int(r['status'][0]), nsteps=int(r['nsteps'][0]), records=int(k),
                        accepted=int(acc.sum()), lu_fail=int((rec[:, 4] == 0).sum()),
                        first=rec[:40].tolist(), last=rec[-60:].tolist())
        print(idx, 'status', r['status'][0], 'nsteps', r['nsteps'][0], 'records', k, 'lu fails',
              int((rec[:, 4] == 0).sum()), flush=True)
        for row in rec[:: max(1, len(rec) // 40)]:
            print('   n %6d t %.6e h %.3e q %.3e lu %d pivmin %.3e F0[0] %.3e y0 %.3e' % tuple(row), flush=True)
        print('  last:')
        for row in rec[-25:]:
            print('   n %6d t %.6e h %.3e q %.3e lu %d pivmin %.3e F0[0] %.3e y0 %.3e' % tuple(row), flush=True)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, 'gpurun_out', 'trace_group.json'), 'w'))


if __name__ == '__main__':
    main()
