"""Cost and accuracy of the degenerate-root retry pass on the bench grid.

Solves the 1024 x 1024 COOxVolcano grid with the bench's settings (Newton
polish after a transient at rtol 1e-8 / atol 1e-10) and each retry tolerance
pair (pck_solve_params.retry_rtol / retry_atol); reports the kernel time, the
step counts and, on the status-4 conditions, |d log10 TOF| against the
tightest retry.  Writes gpurun_out/retry_probe.json and the status map
gpurun_out/volcano_status.npy (int8, [E_CO, E_O]).
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import pycatkin_amd as P
    from pycatkin_amd import _lib as L
    from pycatkin_amd.engine import _ptr
    from pycatkin_amd.functions.volcano import set_volcano_energies, tile_order
    sim = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    set_volcano_energies(sim)
    plan = sim.plan(('CO_ox',))
    net = sim.device(('CO_ox',))
    G = int(os.environ.get('GRID', '1024'))
    be = np.linspace(-2.5, 0.5, G)
    E1, E2 = np.meshgrid(be, be, indexing='ij')
    perm = tile_order(E1.shape)
    n = E1.size
    T, p, d, fx, y0, inflow = sim._inputs(net, plan, n, np.full(n, 600.0), None,
                                          {'ECO': E1.ravel()[perm], 'EO': E2.ravel()[perm]}, None, None, None)
    cond, keep = net.conditions(n, T, p, d, fx, y0, inflow)
    out = dict(y=torch.empty((net.NDYN, n), dtype=torch.float64, device='cuda'),
               tof=torch.empty(n, dtype=torch.float64, device='cuda'),
               status=torch.empty(n, dtype=torch.int32, device='cuda'),
               nsteps=torch.empty(n, dtype=torch.int32, device='cuda'))
    o = L.Outputs()
    o.y, o.ld_y, o.tof, o.status, o.nsteps = _ptr(out['y']), n, _ptr(out['tof']), _ptr(out['status']), _ptr(out['nsteps'])
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    variants = [None, (1e-8, 1e-22), (1e-7, 1e-22), (1e-6, 1e-22), (1e-5, 1e-22), (1e-6, 1e-24), (1e-12, 1e-24)]
    res = {}
    inv = np.empty_like(perm)
    inv[perm] = np.arange(n)
    for v in variants:
        prm = net.params(t0=0.0, t_end=3600.0, rtol=1e-8, atol=1e-10, max_steps=200000, newton=True, retry=v)
        L.check(net.lib.pck_solve(net.h, C.byref(cond), C.byref(prm), C.byref(o), sp))
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            L.check(net.lib.pck_solve(net.h, C.byref(cond), C.byref(prm), C.byref(o), sp))
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        st = out['status'].cpu().numpy()[inv]
        tof = out['tof'].cpu().numpy()[inv]
        ns = out['nsteps'].cpu().numpy()[inv]
        key = 'none' if v is None else '%g/%g' % v
        res[key] = dict(ms=float(np.median(ts)), status=np.bincount(st, minlength=5).tolist(),
                        steps=int(ns.astype(np.int64).sum()), steps_status4=int(ns[st == 4].astype(np.int64).sum()),
                        l10=np.log10(np.where(tof > 0, tof, np.nan)),
                        steps4_pct=[int(x) for x in np.percentile(ns[st == 4], [50, 90, 99, 100])] if (st == 4).any() else [])
        print(key, res[key]['ms'], res[key]['status'], res[key]['steps'], flush=True)
        if v is None:
            os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
            np.save(os.path.join(ROOT, 'gpurun_out', 'volcano_status.npy'), st.reshape(G, G).astype(np.int8))
    ref = res['1e-12/1e-24']['l10']
    summary = {}
    st_map = np.load(os.path.join(ROOT, 'gpurun_out', 'volcano_status.npy')).ravel()
    m4 = st_map == 4
    for key, r in res.items():
        d = np.abs(r['l10'][m4] - ref[m4])
        rel = d / np.maximum(np.abs(ref[m4]), 1e-300)
        summary[key] = dict(ms=r['ms'], status=r['status'], steps=r['steps'], steps_status4=r['steps_status4'],
                            steps_status4_p50_p90_p99_max=r['steps4_pct'],
                            max_abs_dl10_vs_tightest=float(np.nanmax(d)) if d.size else 0.0,
                            max_rel_dl10_vs_tightest=float(np.nanmax(rel)) if d.size else 0.0,
                            p99_abs_dl10=float(np.nanpercentile(d, 99)) if d.size else 0.0,
                            n_status4=int(m4.sum()))
    json.dump(summary, open(os.path.join(ROOT, 'gpurun_out', 'retry_probe.json'), 'w'), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == '__main__':
    main()
