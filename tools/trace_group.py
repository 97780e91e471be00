"""Diagnostic: per-step trace of the lane-group integrator for a few
conditions of the synthetic config (needs the PCK_TRACE build:
tools/ab_build.sh trace -DPCK_TRACE; run with PCK_LIB=pycatkin_amd/_ab/lib_trace.so).

    python tools/trace_group.py IDX [IDX ...]      (indices of the 16384-condition synthetic set)
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
    sim, _ = synthetic_system()
    n = 16384
    D = np.random.default_rng(0).uniform(-0.5, 0.5, (n, 4))
    out = {}
    for idx in (int(a) for a in sys.argv[1:]):
        L.check(lib.pck_trace_set(idx))
        d = D[idx:idx + 1]
        r = sim.solve_batch(T=np.full(1, 500.0), desc={'D%d' % k: d[:, k] for k in range(4)}, tof_terms=('R0',),
                            steady=True, max_steps=int(os.environ.get('MAXSTEPS', 20000)))
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
        for row in rec[-25:]:
            print('   n %6d t %.6e h %.3e q %.3e lu %d pivmin %.3e F0[0] %.3e y0 %.3e' % tuple(row), flush=True)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, 'gpurun_out', 'trace_group.json'), 'w'))


if __name__ == '__main__':
    main()
