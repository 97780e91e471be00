"""GPU diagnostic for the synthetic stress network: timing, status counts,
step-count distribution; dumps a few non-regular conditions for CPU replay."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pycatkin_amd.functions.synthetic import synthetic_system  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
sim, net = synthetic_system()
rng = np.random.default_rng(0)
D = rng.uniform(-0.5, 0.5, (n, 4))
kw = dict(T=np.full(n, 500.0), desc={'D%d' % k: D[:, k] for k in range(4)}, tof_terms=('R0',))
out = {}
for steady in (False, True):
    sim.solve_batch(max_steps=50, **kw)                     # warm-up / plan build
    torch.cuda.synchronize()
    t = time.time()
    r = sim.solve_batch(steady=steady, **kw)
    torch.cuda.synchronize()
    dt = time.time() - t
    st, ns = r['status'], r['nsteps']
    out['steady' if steady else 'transient'] = dict(
        seconds=dt, status=np.unique(st, return_counts=True)[0].tolist(),
        counts=np.unique(st, return_counts=True)[1].tolist(),
        nsteps_pct=np.percentile(ns, [0, 50, 90, 99, 100]).tolist(),
        ymin=float(r['y'].min()))
    if steady:
        bad = np.flatnonzero(st != 0)[:6]
        out['bad'] = dict(idx=bad.tolist(), D=D[bad].tolist(), st=st[bad].tolist(), ns=ns[bad].tolist(),
                          y=r['y'][:, bad].T.tolist())
    print(json.dumps(out['steady' if steady else 'transient']), flush=True)
os.makedirs('gpurun_out', exist_ok=True)
json.dump(out, open('gpurun_out/diag_synth.json', 'w'))
