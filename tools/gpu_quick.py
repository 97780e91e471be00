import sys, time, os
sys.path.insert(0, '/root/repo')
import numpy as np, torch
print('device', torch.cuda.get_device_name(0), flush=True)
import pycatkin_amd as P
from pycatkin_amd.functions.volcano import volcano_activity
from oracle import mk_oracle as O
inp = '/root/repo/tests/golden/inputs/COOxVolcano/input.json'
s = P.read_from_input_file(inp)
be = np.array([-2.5, -1.5, -1.0, -0.5, 0.5])
for steady in (False, True):
    t = time.time()
    act, r = volcano_activity(s, be, be, steady=steady)
    torch.cuda.synchronize()
    print('steady', steady, 'time', time.time() - t, 'status', r['status'].tolist(), 'nsteps', r['nsteps'].tolist(), flush=True)
    print(np.array2string(act, precision=9), flush=True)
spec = O.load_spec(inp)
for eco, eo in [(-1.0, -1.0), (-2.5, -2.5), (0.5, -1.5)]:
    ref = O.volcano_point(spec, eco, eo, steady=True)
    print(eco, eo, 'oracle steady', ref['activity'], flush=True)
for n in (1024, 1024 * 1024):
    eco = np.random.default_rng(0).uniform(-2.5, 0.5, n); eo = np.random.default_rng(1).uniform(-2.5, 0.5, n)
    for rep in range(2):
        torch.cuda.synchronize(); t = time.time()
        r = s.solve_batch(T=np.full(n, 600.0), desc={'ECO': eco, 'EO': eo}, tof_terms=('CO_ox',), steady=True, activity=True, to_numpy=False)
        torch.cuda.synchronize(); dt = time.time() - t
        print('n', n, 'time %.4f s' % dt, 'solves/s %.3e' % (n / dt), 'status!=0', int((r['status'] != 0).sum()), 'mean steps', float(r['nsteps'].double().mean()), 'max', int(r['nsteps'].max()), flush=True)
