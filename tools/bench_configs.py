"""Throughput of the other BASELINE.json configs (bench.py measures the
headline volcano grid).  One JSON line per config; device time of the solve
launch(es) by HIP events on the launch stream, inputs resident in HBM.

  cstr       COOxReactor (Pd111) CSTR temperature sweep, 1e4 temperatures,
             transient + Newton (configs[1])
  dmtm_drc   DMTM degree of rate control over a T x p grid (2R+1 = 23
             solves per condition, lane groups of 16) (configs[3])
  synthetic  50 species / 150 reactions, random descriptors, transient +
             Newton (configs[4])
  ch4        test/CH4_input.json, patched formulation, transient to 1e4 s over
             a T sweep (configs[0] batched)

    python tools/bench_configs.py [--configs cstr,dmtm_drc,synthetic,ch4] [--n N] [--reps K]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
INPUTS = os.path.join(ROOT, 'tests', 'golden', 'inputs')


def log(msg):
    print('[bench_configs] ' + msg, file=sys.stderr, flush=True)


def timed(torch, fn, reps):
    s = torch.cuda.current_stream()
    fn()                                            # warm-up
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1e-3


PLAN_MODE = 0
MAX_STEPS = 200000          # the library default (classes/system.py: solve_batch)


def run(sim, T, desc, tof_terms, steady, drc, reps, torch, t_end=None, rtol=None, atol=None, p=None,
        max_steps=None, eps=5e-2, dump=None):
    from pycatkin_amd import _lib as L
    from pycatkin_amd.engine import _ptr
    max_steps = MAX_STEPS if max_steps is None else max_steps
    plan = sim.plan(tuple(tof_terms))
    net = sim.device(tuple(tof_terms))
    net.set_plan_mode(PLAN_MODE)
    n = len(T)
    Tt, pp, d, fx, y0, inflow = sim._inputs(net, plan, n, T, p, desc, None, None, None)
    cond, keep = net.conditions(n, Tt, pp, d, fx, y0, inflow)
    times = sim.params['times']
    prm = net.params(t0=times[0], t_end=times[-1] if t_end is None else t_end,
                     rtol=sim.params['rtol'] if rtol is None else rtol, atol=sim.params['atol'] if atol is None else atol,
                     max_steps=max_steps, newton=steady, newton_iters=60, drc_eps=eps)
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    st = torch.zeros(n, dtype=torch.int32, device='cuda')
    if drc:
        xi = torch.zeros((net.NRXN, n), dtype=torch.float64, device='cuda')
        tof0 = torch.empty(n, dtype=torch.float64, device='cuda')

        def fn():
            L.check(net.lib.pck_drc(net.h, C.byref(cond), C.byref(prm), _ptr(xi), n, _ptr(tof0), _ptr(st), C.c_void_p(0), sp))
    else:
        out = dict(y=torch.empty((net.NDYN, n), dtype=torch.float64, device='cuda'),
                   tof=torch.empty(n, dtype=torch.float64, device='cuda'),
                   nsteps=torch.empty(n, dtype=torch.int32, device='cuda'))
        o = L.Outputs()
        o.y, o.ld_y, o.tof, o.status, o.nsteps = _ptr(out['y']), n, _ptr(out['tof']), _ptr(st), _ptr(out['nsteps'])

        def fn():
            L.check(net.lib.pck_solve(net.h, C.byref(cond), C.byref(prm), C.byref(o), sp))
    sec = timed(torch, fn, reps)
    s = st.cpu().numpy()
    res = dict(n=n, seconds_per_launch=sec, solves_per_s=n / sec, ndyn=net.NDYN, nrxn=net.NRXN,
               status={int(k): int(v) for k, v in zip(*np.unique(s, return_counts=True))})
    res['max_steps'] = max_steps
    if not drc:
        ns = out['nsteps'].double()
        res['nsteps_median'] = float(ns.median())
        res['nsteps_max'] = float(ns.max())
    if dump:                                        # failing conditions, for the diagnosis
        bad = np.flatnonzero((s != 0) & (s != 4))
        rec = dict(idx=bad.tolist(), status=s[bad].tolist(), T=np.asarray(T)[bad].tolist())
        if p is not None:
            rec['p'] = np.broadcast_to(np.asarray(p, float), (n,))[bad].tolist()
        if desc:
            rec['desc'] = {k: np.asarray(v)[bad].tolist() for k, v in desc.items()}
        if not drc:
            rec['nsteps'] = out['nsteps'].cpu().numpy()[bad].tolist()
            rec['nsteps_hist'] = np.percentile(out['nsteps'].cpu().numpy(), [50, 90, 99, 99.9, 100]).tolist()
        os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
        json.dump(rec, open(os.path.join(ROOT, 'gpurun_out', 'fail_%s.json' % dump), 'w'))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--configs', default='cstr,dmtm_drc,synthetic,ch4')
    ap.add_argument('--n', type=int, default=0, help='conditions (0: the config default)')
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--plan-mode', type=int, default=0, help='0 auto, 1 runtime plan, 2 lane-group solver')
    ap.add_argument('--max-steps', type=int, default=200000)
    ap.add_argument('--dump', action='store_true', help='write gpurun_out/fail_<config>.json')
    args = ap.parse_args()
    import torch
    import pycatkin_amd as P
    global PLAN_MODE, MAX_STEPS
    PLAN_MODE = args.plan_mode
    MAX_STEPS = args.max_steps
    dump = (lambda c: c) if args.dump else (lambda c: None)
    lines = []
    for cfg in args.configs.split(','):
        t0 = time.time()
        if cfg == 'cstr':
            sim = P.read_from_input_file(os.path.join(INPUTS, 'COOxReactor', 'input_Pd111.json'))
            n = args.n or 10000
            r = run(sim, np.linspace(423.0, 623.0, n), None, ('CO_ox',), True, False, args.reps, torch,
                    dump=dump('cstr'))
            r['workload'] = 'COOxReactor Pd111 CSTR, %d temperatures 423-623 K, t_end 3600 s + Newton' % n
        elif cfg == 'dmtm_drc':
            sim = P.read_from_input_file(os.path.join(INPUTS, 'DMTM', 'input.json'))
            g = int(np.sqrt(args.n)) if args.n else 64
            TT, pp = np.meshgrid(np.linspace(400.0, 800.0, g), np.logspace(4, 6, g), indexing='ij')
            r = run(sim, TT.ravel(), None, ('r5', 'r9'), True, True, args.reps, torch, p=pp.ravel(),
                    rtol=1e-8, atol=1e-12, dump=dump('dmtm_drc'))
            r['workload'] = 'DMTM DRC(r5+r9, eps 5e-2) on a %dx%d (T 400-800 K) x (p 1e4-1e6 Pa) grid, t_end 1e12 s + Newton' % (g, g)
        elif cfg == 'synthetic':
            from pycatkin_amd.functions.synthetic import synthetic_system
            sim, _ = synthetic_system()
            n = args.n or 65536
            rng = np.random.default_rng(0)
            D = rng.uniform(-0.5, 0.5, (n, 4))
            r = run(sim, np.full(n, 500.0), {'D%d' % k: D[:, k] for k in range(4)}, ('R0',), True, False, args.reps,
                    torch, dump=dump('synthetic'))
            r['workload'] = 'synthetic 50 species / 150 reactions, %d random-descriptor conditions, t_end 1e4 s + Newton' % n
        elif cfg == 'ch4':
            sim = P.read_from_input_file(os.path.join(INPUTS, 'CH4', 'input.json'), formulation='patched')
            sim.reactions['C_ads'].dErxn_user = 1.0
            sim.reactions['O_ads'].dErxn_user = 1.0
            sim.states['sC'].Gelec = 1.0
            sim.states['sO'].Gelec = 1.0
            n = args.n or 16384
            r = run(sim, np.linspace(473.0, 573.0, n), None, (), False, False, args.reps, torch, t_end=1e4,
                    rtol=1e-10, atol=1e-12, dump=dump('ch4'))
            r['workload'] = 'CH4_input.json (patched), %d temperatures, transient to 1e4 s (solver.py:374)' % n
        else:
            raise SystemExit('unknown config %s' % cfg)
        r['config'] = cfg
        r['plan_mode'] = args.plan_mode
        r['wall_s'] = time.time() - t0
        log('%s done in %.1f s' % (cfg, r['wall_s']))
        print(json.dumps(r), flush=True)
        lines.append(r)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    name = 'bench_configs.json' if not args.plan_mode else 'bench_configs_pm%d.json' % args.plan_mode
    with open(os.path.join(ROOT, 'gpurun_out', name), 'w') as fh:
        json.dump(lines, fh, indent=1)


if __name__ == '__main__':
    main()
