"""Benchmark: steady-state MK solves/sec on the COOx volcano descriptor grid.

One step = one batched solve of this rank's 1024 x 1024 (E_CO x E_O) shard of
the COOxVolcano grid (BASELINE.json configs[2]; examples/COOxVolcano): kernel
(1) rate constants from the descriptor energies, kernel (3) Rodas4 transient
to t_end = 3600 s + Newton steady-state polish, kernel (4) activity.  Inputs
are resident in HBM before the timed region.  With N ranks the E_CO axis is
N x 1024 points (weak scaling, no data-path collective); the activity map is
gathered with one all_gather after the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_VECTOR_PEAK_TFLOPS = 78.6   # MI355X datasheet FP64 vector peak (the guides list no FP64 figure)


def flops_per_step(plan):
    """Algorithmic fp64 FLOPs of one Rodas4 step of kernel (3) for this plan
    (mk_kernels.hip: integrate): 6 rhs, 1 Jacobian, 1 LU, 6 triangular solves
    and the stage / error-norm vector arithmetic."""
    NS = len(plan.dyn)
    S = plan.extra['S']
    ip = plan.ip
    from pycatkin_amd import _lib as L
    R = int(ip[L.I_NRXN])
    ef = ip[ip[L.I_OFF_EXPF]: ip[L.I_OFF_EXPF] + R * NS].reshape(R, NS)
    er = ip[ip[L.I_OFF_EXPR]: ip[L.I_OFF_EXPR] + R * NS].reshape(R, NS)
    nnzS = int(np.count_nonzero(S))
    mults = int(np.sum(np.maximum(ef - 1, 0) + (ef > 0)) + np.sum(np.maximum(er - 1, 0) + (er > 0)))
    rhs = NS + mults + R + 2 * nnzS + 4 * NS                 # conc, products, net, S.net, reactor rows
    jac = 0
    for j in range(R):
        for e in (ef[j], er[j]):
            nz = np.nonzero(e)[0]
            jac += len(nz) * (3 + len(nz))                     # k*e*cf*c^(e-1)*prod(others)
    jac += 2 * nnzS * NS + NS * NS + NS                        # S * dnet, row scaling, flow diagonal
    lu = (2 * NS ** 3) // 3 + NS * NS
    solve = 2 * NS * NS
    vec = NS * (2 + 3 + 4 + 5 + 6 + 7 + 6 + 8)                 # stage combinations, W diagonal, error norm
    return 6 * rhs + jac + lu + 6 * solve + vec + NS * NS


def cpu_baseline(n_points=160, workers=16, seed=0, budget_s=25.0):
    """Oracle (numpy/scipy BDF + Newton, the reference algorithm restated) on
    a bounded random sample of the same grid, in a process pool; stops after
    `budget_s` seconds and reports completed points / elapsed."""
    import multiprocessing as mp
    rng = np.random.default_rng(seed)
    pts = [tuple(p) for p in rng.uniform(-2.5, 0.5, (n_points, 2))]
    ctx = mp.get_context('spawn')
    pool = ctx.Pool(workers)
    try:
        pool.map(_cpu_warm, range(workers))            # imports outside the timed sample
        t = time.time()
        done = 0
        for _ in pool.imap_unordered(_cpu_point, pts):
            done += 1
            if time.time() - t > budget_s:
                break
        dt = time.time() - t
    finally:
        pool.terminate()
    return done / dt, dt, done


def _cpu_warm(_):
    from oracle import mk_oracle  # noqa: F401
    return 0


def _cpu_point(p):
    from oracle import mk_oracle as O
    spec = O.load_spec(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    return O.volcano_point(spec, p[0], p[1], steady=True, rtol=1e-8, atol=1e-10)['activity']


def log(msg):
    print('[bench] ' + msg, file=sys.stderr, flush=True)


def profiled_traffic(kernel_name, grid):
    """HBM bytes per launch of `kernel_name` from the committed rocprofv3 PMC
    summary named in profiles/CURRENT (else the last of profiles/r*/*/summary.json;
    written by tools/pmc_summary.py from a tools/profile.sh run of this bench at
    the same grid), or (None, None)."""
    import glob
    key = kernel_name.replace('PlanCT<', 'PlanCT<pck::nets::')
    found = None
    files = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*', '*', 'summary.json')))
    cur = os.path.join(ROOT, 'profiles', 'CURRENT')      # the profile of the current kernel, searched last (wins)
    if os.path.isfile(cur):
        files.append(os.path.join(ROOT, open(cur).read().strip(), 'summary.json'))
    for f in files:
        try:
            s = json.load(open(f))
        except (OSError, ValueError):
            continue
        for k, v in s.items():
            short = k.replace('pck::', '').replace(' ', '')
            if short == key.replace('pck::', '').replace(' ', '') and 'traffic_bytes' in v \
                    and v.get('grid', grid) == grid:
                found = (v['traffic_bytes'], os.path.relpath(f, ROOT))
    return found or (None, None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--grid', type=int, default=1024)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-points', type=int, default=160)
    ap.add_argument('--no-newton', action='store_true', help='A/B diagnostic: transient only (not the bench workload)')
    ap.add_argument('--shard', choices=('cyclic', 'contiguous'), default='cyclic',
                    help='E_CO rows of the (N*G) x G weak-scaling grid per rank: every N-th row (default) or a band')
    ap.add_argument('--emulate', default=None, metavar='R/N',
                    help='single-GPU A/B: solve the shard rank R of N would own, without a process group')
    ap.add_argument('--tile', default='16x4', help='patch shape (rows x cols) of --order tile')
    ap.add_argument('--order', choices=('tile', 'row', 'oracle-steps'), default='tile',
                    help="condition order in HBM: 'tile' = one grid patch per wave (default), 'row' = row-major")
    ap.add_argument('--runtime-plan', action='store_true',
                    help='A/B: force the runtime-plan solver instead of the compiled-in network')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    import pycatkin_amd as P
    from pycatkin_amd import _lib as L
    from pycatkin_amd.engine import _ptr
    from pycatkin_amd.functions.volcano import set_volcano_energies, tile_order
    from pycatkin_amd.parallel import assemble_weak_grid, weak_grid_rows

    sim = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    set_volcano_energies(sim)
    plan = sim.plan(('CO_ox',))
    net = sim.device(('CO_ox',))
    net.set_plan_mode(args.runtime_plan)
    kernel_name = 'k_solve<PlanRT<4>>' if (args.runtime_plan or not net.compiled_plan) else 'k_solve<PlanCT<Volcano>>'
    G = args.grid
    eo = np.linspace(-2.5, 0.5, G)
    shard_rank, shard_world = (rank, world) if not args.emulate else map(int, args.emulate.split('/'))
    cyclic = args.shard == 'cyclic'
    eco_loc = weak_grid_rows(G, shard_rank, shard_world, cyclic=cyclic)   # rank's rows of the (world*G) x G grid
    E1, E2 = np.meshgrid(eco_loc, eo, indexing='ij')
    n = E1.size
    perm = None
    if args.order == 'tile':                        # one wave = one 16x4 patch of the grid (E_CO x E_O)
        perm = tile_order(E1.shape, tuple(int(x) for x in args.tile.split('x')))
        E1, E2 = E1.ravel()[perm], E2.ravel()[perm]
    T = float(sim.params['temperature'])
    Tt, p, d, fx, y0, inflow = sim._inputs(net, plan, n, np.full(n, T), None,
                                           {'ECO': E1.ravel(), 'EO': E2.ravel()}, None, None, None)
    cond, keep = net.conditions(n, Tt, p, d, fx, y0, inflow)       # device-resident inputs
    times = sim.params['times']
    prm = net.params(t0=times[0], t_end=times[-1], rtol=sim.params['rtol'], atol=sim.params['atol'],
                     max_steps=200000, newton=not args.no_newton, newton_iters=30, activity=True)
    out = dict(y=torch.empty((net.NDYN, n), dtype=torch.float64, device='cuda'),
               tof=torch.empty(n, dtype=torch.float64, device='cuda'),
               status=torch.empty(n, dtype=torch.int32, device='cuda'),
               nsteps=torch.empty(n, dtype=torch.int32, device='cuda'))
    o = L.Outputs()
    o.y, o.ld_y, o.tof, o.status, o.nsteps = _ptr(out['y']), n, _ptr(out['tof']), _ptr(out['status']), _ptr(out['nsteps'])
    kf = torch.empty((net.NRXN, n), dtype=torch.float64, device='cuda')
    kr = torch.empty_like(kf)
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream)

    def step():
        L.check(net.lib.pck_solve(net.h, C.byref(cond), C.byref(prm), C.byref(o), sp))

    def rate_constants_only():
        L.check(net.lib.pck_rate_constants(net.h, C.byref(cond), _ptr(kf), _ptr(kr), n, sp))

    if args.order == 'oracle-steps':
        # DIAGNOSTIC ONLY (never the bench line's order): sort the conditions by
        # the step counts of a first solve, heaviest first -- the ceiling of
        # any a-priori condition ordering
        step()
        torch.cuda.synchronize()
        srt = torch.argsort(out['nsteps'].long() * 4 - out['status'].long(), descending=True).cpu().numpy()
        E1, E2 = E1.ravel()[srt], E2.ravel()[srt]
        Tt, p, d, fx, y0, inflow = sim._inputs(net, plan, n, np.full(n, T), None,
                                               {'ECO': E1.ravel(), 'EO': E2.ravel()}, None, None, None)
        cond, keep = net.conditions(n, Tt, p, d, fx, y0, inflow)
    log('rank %d: %d conditions, warmup %d' % (rank, n, args.warmup))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    log('rank %d: timing %d steps' % (rank, args.steps))
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    solve_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    # kernel (1) alone, same stream, to split pck_solve's two launches
    e1 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a, b in e1:
        a.record(stream)
        rate_constants_only()
        b.record(stream)
    torch.cuda.synchronize()
    k1_ms = float(np.mean([a.elapsed_time(b) for a, b in e1]))
    k3_ms = max(solve_ms - k1_ms, 1e-9)

    st = out['status']
    n_ok = int((st == 0).sum())
    n_degen = int((st == 4).sum())
    n_fail = n - n_ok - n_degen
    steps_total = float(out['nsteps'].double().sum())
    ns = out['nsteps'].double()
    pad = (-n) % 64
    wave_max = torch.nn.functional.pad(ns, (0, pad)).reshape(-1, 64).max(dim=1).values
    lane_eff = float(ns.mean() / wave_max.mean())     # useful lane-steps / issued wave-steps
    fl = flops_per_step(plan) * steps_total
    achieved = fl / (k3_ms * 1e-3) / 1e12
    # algorithmic HBM bytes of one k_solve launch: kf, kr in; y, activity, status, steps out
    algo_bytes = n * (16 * net.NRXN + 8 * net.NDYN + 8 + 4 + 4)
    traffic, traffic_src = profiled_traffic(kernel_name, G)

    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device='cuda')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt)
        # final gather of the activity map (RCCL over xGMI), outside the timed region
        gathered = [torch.empty_like(out['tof']) for _ in range(world)]
        dist.all_gather(gathered, out['tof'])
        act_map = assemble_weak_grid(gathered, G, G, perm, cyclic)      # (world*G) x G activity map
        assert act_map.shape == (world * G, G)
        cnt = torch.tensor([n_fail], dtype=torch.int64, device='cuda')
        dist.all_reduce(cnt)
        n_fail = int(cnt)
    per_step = elapsed / args.steps
    value = n * world / per_step

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            workers = min(16, os.cpu_count() or 1)
            log('cpu baseline: %d points, %d workers' % (args.cpu_points, workers))
            v, dt, done = cpu_baseline(args.cpu_points, workers)
            cpu = dict(value=v, unit='solves/s', cores=workers, kind='port',
                       sample='%d random (E_CO, E_O) points of the same grid solved in %.1f s: oracle scipy BDF '
                              '(rtol 1e-8, atol 1e-10) to t_end = 3600 s + Newton polish, %d worker processes'
                              % (done, dt, workers))
        line = {
            'metric': 'steady-state MK solves/sec (whole node) on COOx volcano grid at 1/2/4/8 GPUs',
            'value': value, 'unit': 'solves/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': per_step * 1e3, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'f64', 'data': 'synthetic descriptor grid (E_CO, E_O in [-2.5, 0.5] eV) on the reference '
                                    'COOxVolcano network',
            'config': {'workload': 'COOxVolcano %dx%d (E_CO x E_O) grid per GPU, T=600 K, t_end=3600 s, '
                                   'rtol 1e-8 / atol 1e-10, Newton steady-state polish, activity' % (G, G),
                       'grid_per_gpu': [G, G], 'global_grid': [G * world, G], 'parallelism': 'dp%d' % world,
                       'shard': args.shard + ('' if not args.emulate else ' (emulated rank %s)' % args.emulate),
                       'order': args.order if args.order == 'row' else 'tile %s' % args.tile},
            'roofline': {'bound': 'valu_fp64', 'achieved': achieved, 'peak': FP64_VECTOR_PEAK_TFLOPS,
                         'unit': 'TFLOP/s', 'frac': achieved / FP64_VECTOR_PEAK_TFLOPS, 'traffic': traffic,
                         'traffic_unit': 'bytes per launch (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE)',
                         'traffic_source': traffic_src, 'algorithmic_bytes': algo_bytes,
                         'kernel': kernel_name, 'kernel_ms': k3_ms, 'rate_constants_ms': k1_ms,
                         'flops_per_launch': fl, 'flops_per_step': flops_per_step(plan),
                         'integrator_steps': steps_total, 'lane_efficiency': lane_eff},
            'cpu_baseline': cpu,
            'status': {'regular_root': n_ok * (world if dist else 1), 'degenerate_root_transient_kept':
                       n_degen, 'failed': n_fail},
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
