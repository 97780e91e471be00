"""Diagnostic: shader-clock cycles per integrator phase (Jacobian, LU,
triangular solves, rate evaluations) of one lane-group condition solved
alone (needs the PCK_TRACE build: tools/ab_build.sh trace -DPCK_TRACE, run
with PCK_LIB=pycatkin_amd/_ab/lib_trace.so PCK_JIT=0).

    python tools/phase_group.py synthetic IDX [MAXSTEPS]
    python tools/phase_group.py dmtm T
    python tools/phase_group.py ch4 T
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    # --lib PATH (the PCK_TRACE build); the compiled-in kernels carry the
    # phase counters, so the hipRTC path is switched off here
    if '--lib' in sys.argv:
        i = sys.argv.index('--lib')
        os.environ['PCK_LIB'] = os.path.abspath(sys.argv[i + 1])
        del sys.argv[i:i + 2]
    os.environ['PCK_JIT'] = '0'
    import torch
    import pycatkin_amd as P
    from pycatkin_amd import _lib as L
    lib = L.load()
    lib.pck_trace_set.argtypes = [C.c_longlong]
    lib.pck_phase_get.argtypes = [C.c_void_p]
    which = sys.argv[1]
    ms = 200000
    if which == 'synthetic':
        from pycatkin_amd.functions.synthetic import synthetic_system
        sim, _ = synthetic_system()
        D = np.random.default_rng(0).uniform(-0.5, 0.5, (16384, 4))
        i = int(sys.argv[2])
        ms = int(sys.argv[3]) if len(sys.argv) > 3 else 200000
        kw = dict(T=np.full(1, 500.0), desc={'D%d' % k: D[i:i + 1, k] for k in range(4)}, tof_terms=('R0',),
                  steady=True)
    elif which == 'dmtm':
        sim = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'DMTM', 'input.json'))
        kw = dict(T=np.array([float(sys.argv[2])]), tof_terms=('r5', 'r9'), steady=True)
    else:
        sim = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'CH4', 'input.json'),
                                     formulation='patched')
        # the descriptor energies of bench.py: ch4_workload (unset, the
        # reaction energies are None)
        for r, s in (('C_ads', 'sC'), ('O_ads', 'sO')):
            sim.reactions[r].dErxn_user = 1.0
            sim.states[s].Gelec = 1.0
        kw = dict(T=np.array([float(sys.argv[2])]), steady=False, t_end=1e4, rtol=1e-10, atol=1e-12)
    sim.solve_batch(max_steps=100, **kw)        # warm (hipRTC / module load)
    L.check(lib.pck_trace_set(0))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = sim.solve_batch(max_steps=ms, **kw)
    wall = time.perf_counter() - t0
    ph = np.zeros(8)
    L.check(lib.pck_phase_get(ph.ctypes.data_as(C.c_void_p)))
    steps = max(ph[5], 1.0)
    names = ['jac', 'lu', 'solve(6)', 'rhs(6)']
    tot = ph[:4].sum()
    out = dict(config=which, args=sys.argv[2:], status=int(r['status'][0]), nsteps=int(r['nsteps'][0]),
               wall_s=wall, us_per_step=1e6 * wall / max(int(r['nsteps'][0]), 1),
               cycles_per_step={n: ph[k] / steps for k, n in enumerate(names)},
               share={n: ph[k] / tot for k, n in enumerate(names)})
    print(json.dumps(out))


if __name__ == '__main__':
    main()
