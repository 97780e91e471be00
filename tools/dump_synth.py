"""Synthetic 50 x 150 network on the GPU (the bench's synthetic workload):
solve time, and status / integrator steps of every condition to
gpurun_out/synth_<n>.npz for straggler analysis.  usage: python tools/dump_synth.py N [max_steps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pycatkin_amd.functions.synthetic import synthetic_system
    n = int(sys.argv[1])
    ms = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
    sim, _ = synthetic_system()
    D = np.random.default_rng(0).uniform(-0.5, 0.5, (n, 4))
    kw = dict(T=np.full(n, 500.0), desc={'D%d' % k: D[:, k] for k in range(4)}, tof_terms=('R0',))
    sim.solve_batch(max_steps=20, **kw)
    torch.cuda.synchronize()
    t = time.time()
    r = sim.solve_batch(steady=True, max_steps=ms, **kw)
    torch.cuda.synchronize()
    dt = time.time() - t
    st, ns = np.asarray(r['status']), np.asarray(r['nsteps'])
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    np.savez(os.path.join(ROOT, 'gpurun_out', 'synth_%d.npz' % n), st=st, ns=ns, D=D, s=dt)
    print('n %d  %.2f s  status %s  steps p50 %d p99 %d max %d' % (
        n, dt, dict(zip(*[a.tolist() for a in np.unique(st, return_counts=True)])), np.median(ns),
        np.percentile(ns, 99), ns.max()), flush=True)


if __name__ == '__main__':
    main()
