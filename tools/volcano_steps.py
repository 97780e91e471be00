"""Diagnostic (GPU): the integrator step count of every point of the bench's
1024 x 1024 volcano grid under the steady rule (System.solve_batch(steady=True),
as bench.py's volcano workload), saved as a compressed npz with the grid axes,
plus the step-count histogram and the slowest points on stdout.  The slowest
points are the strong-scaling floor (DESIGN.md "Multi-GPU"); feed them to
tools/rodas_mirror.py volcano ECO EO to see where their steps go.

    python tools/volcano_steps.py [OUT.npz] [G]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import pycatkin_amd as P
    from pycatkin_amd.functions.volcano import volcano_activity
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, 'gpurun_out', 'volcano_steps.npz')
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    sim = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    axis = np.linspace(-2.5, 0.5, G)
    _, r = volcano_activity(sim, axis, axis, steady=True)
    ns = np.asarray(r['nsteps']).reshape(G, G)
    st = np.asarray(r['status']).reshape(G, G)
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    np.savez_compressed(out, nsteps=ns.astype(np.int32), status=st.astype(np.int8), eco=axis, eo=axis)
    flat = ns.ravel()
    print('mean %.1f, p50 %d, p99 %d, p99.9 %d, max %d' % (flat.mean(), *np.percentile(flat, [50, 99, 99.9]), flat.max()))
    edges = [0, 100, 200, 300, 400, 500, 600, 800, 1000, 1200, 1500, 2000, 10 ** 9]
    h, _ = np.histogram(flat, edges)
    print('histogram:', dict(zip(['<%d' % e for e in edges[1:]], h.tolist())))
    for k in np.argsort(flat)[::-1][:20]:
        i, j = divmod(int(k), G)
        print('  ECO %.6f EO %.6f (i %d j %d): %d steps, status %d' % (axis[i], axis[j], i, j, flat[k], st.ravel()[k]))


if __name__ == '__main__':
    main()
