"""Per-step latency of the lane-group solver on the synthetic 50 x 150
network: a batch of n conditions with a fixed step budget (every condition
runs the budget out or finishes), wall time / steps.  usage:
python tools/synth_latency.py N MAXSTEPS"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pycatkin_amd.functions.synthetic import synthetic_system
    n, ms = int(sys.argv[1]), int(sys.argv[2])
    sim, _ = synthetic_system()
    D = np.random.default_rng(0).uniform(-0.5, 0.5, (n, 4))
    kw = dict(T=np.full(n, 500.0), desc={'D%d' % k: D[:, k] for k in range(4)}, tof_terms=('R0',), steady=False)
    sim.solve_batch(max_steps=10, **kw)
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = sim.solve_batch(max_steps=ms, **kw)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    ns = np.asarray(r['nsteps'])
    print('n %d max_steps %d: %.3f s, steps max %d mean %.0f -> %.1f us per step of the longest' % (
        n, ms, dt, ns.max(), ns.mean(), 1e6 * dt / ns.max()), flush=True)


if __name__ == '__main__':
    main()
