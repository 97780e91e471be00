"""Diagnostic: can a cheap preview solve order the volcano wavefronts
longest-first?  Solves the bench grid (16 x 4 patch order) as a transient at
the bench tolerances (rtol 1e-8 / atol 1e-10) and at loose ones, and writes
the per-condition step counts to gpurun_out/predictor_probe.npz (the
scheduling model tools/sched_sim.py evaluates orders from them on the CPU)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import time
    import torch
    import pycatkin_amd as P
    from pycatkin_amd.functions.volcano import set_volcano_energies, tile_order
    sim = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    set_volcano_energies(sim)
    G = 1024
    be = np.linspace(-2.5, 0.5, G)
    E1, E2 = np.meshgrid(be, be, indexing='ij')
    perm = tile_order(E1.shape)
    n = E1.size
    kw = dict(T=np.full(n, 600.0), desc={'ECO': E1.ravel()[perm], 'EO': E2.ravel()[perm]}, tof_terms=('CO_ox',),
              steady=False, to_numpy=False)
    out = {}
    for key, rtol, atol in (('r8', 1e-8, 1e-10), ('r6', 1e-6, 1e-8), ('r4', 1e-4, 1e-6), ('r3', 1e-3, 1e-5)):
        sim.solve_batch(rtol=rtol, atol=atol, **kw)
        torch.cuda.synchronize()
        t = time.time()
        r = sim.solve_batch(rtol=rtol, atol=atol, **kw)
        torch.cuda.synchronize()
        out[key] = r['nsteps'].cpu().numpy()
        print(key, 'mean steps %.1f' % out[key].mean(), 'max', out[key].max(), '%.2f ms' % ((time.time() - t) * 1e3),
              flush=True)
        # one lane per 64-condition patch (what a preview launch would solve)
        kw1 = dict(kw, T=np.full(n // 64, 600.0), desc={k: v[::64] for k, v in kw['desc'].items()})
        sim.solve_batch(rtol=rtol, atol=atol, **kw1)
        torch.cuda.synchronize()
        t = time.time()
        r1 = sim.solve_batch(rtol=rtol, atol=atol, **kw1)
        torch.cuda.synchronize()
        out[key + '_lane0'] = r1['nsteps'].cpu().numpy()
        print(key, 'one lane per patch: %.2f ms' % ((time.time() - t) * 1e3), flush=True)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    np.savez(os.path.join(ROOT, 'gpurun_out', 'predictor_probe.npz'), perm=perm, **out)


if __name__ == '__main__':
    main()
