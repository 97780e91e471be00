"""Diagnostic (GPU): where a step of the one-lane-per-condition integrator
goes, on the bench workload (the 1024 x 1024 COOxVolcano grid in patch order,
cost-ordered dispatch, STEADY_TRANSIENT), from the PCK_PHASE build
(mk_solver.h: PCK_LPH; tools/ab_build.sh phase -DPCK_PHASE=1): shader-clock
cycles per integrator step of the sampled wavefronts, by phase.

    python tools/phase_lane.py --lib pycatkin_amd/_diag/lib_phase.so [OUT.json]

The stamps are scheduling barriers: the build runs slower than the product
(no overlap across phases), so the shares, not the absolute cycles, are the
result.  Cycles are counted while the other waves of the SIMD run too.
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = ['jacobian', 'lu', 'solve(6)', 'rhs(7)', 'stage combinations', 'control/projection']


def main():
    args = sys.argv[1:]
    if '--lib' in args:
        i = args.index('--lib')
        os.environ['PCK_LIB'] = os.path.abspath(args[i + 1])
        del args[i:i + 2]
    screen = 'auto'
    if '--screen' in args:                     # --screen 0: the single pass
        i = args.index('--screen')
        screen = float(args[i + 1]) or None
        del args[i:i + 2]
    import torch
    import pycatkin_amd as P
    from pycatkin_amd import _lib as L
    from pycatkin_amd.functions.volcano import set_volcano_energies, tile_order
    lib = L.load()
    lib.pck_lphase_get.argtypes = [C.c_void_p]
    s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    be = np.linspace(-2.5, 0.5, 1024)
    ECO, EO = np.meshgrid(be, be, indexing='ij')
    order = tile_order((1024, 1024))
    kw = dict(T=np.full(order.size, 600.0), desc={'ECO': ECO.ravel()[order], 'EO': EO.ravel()[order]},
              tof_terms=('CO_ox',), steady=True, activity=True, to_numpy=False, screen=screen)
    s.solve_batch(**kw)                        # warm
    torch.cuda.synchronize()
    L.check(lib.pck_lphase_reset())
    t0 = time.perf_counter()
    r = s.solve_batch(**kw)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ph = np.zeros(8)
    L.check(lib.pck_lphase_get(ph.ctypes.data_as(C.c_void_p)))
    steps, waves = max(ph[6], 1.0), ph[7]
    tot = ph[:6].sum()
    out = dict(workload='volcano 1024x1024 patch order, steady, screen %s' % screen, wall_ms=1e3 * wall, sampled_waves=int(waves),
               steps_per_wave=steps / max(waves, 1.0),
               cycles_per_step={n: ph[k] / steps for k, n in enumerate(NAMES)},
               share={n: ph[k] / tot for k, n in enumerate(NAMES)},
               total_cycles_per_step=tot / steps)
    print(json.dumps(out, indent=1))
    if args:
        json.dump(out, open(args[0], 'w'), indent=1)


if __name__ == '__main__':
    main()
