"""Benchmark: steady-state MK solves/sec on the COOx volcano descriptor grid
(BASELINE.json configs[2]) and, with --config, the other BASELINE configs.

One step = one batched solve of this rank's share of the workload: kernel (1)
rate constants from the descriptor energies, kernel (3) RODAS4P transient to
t_end + Newton steady-state polish, kernel (4) TOF / activity.  Inputs are
resident in HBM before the timed region.

Multi-GPU (one process per GPU).  `--gpus N` without a torch.distributed
environment spawns N rank processes (RANK / LOCAL_RANK / WORLD_SIZE set per
child) before anything touches the GPU; under `torch.distributed.run` the
ranks come from the environment.  The conditions are independent, so ranks
share nothing in the timed region; one RCCL all_gather of the results follows
it.

  --scaling strong (default)  BASELINE configs[2]: the fixed 1024 x 1024 grid
                              sharded over the N ranks, rank r solving E_CO
                              rows r, r+N, ... (cyclic rows: every rank samples
                              the whole volcano).  At N = 8 each GPU holds
                              2 048 wavefronts for 3 072 wave slots and runs at
                              the latency of its slowest wavefronts (DESIGN.md
                              "Multi-GPU"; tools/emulate_scaling.py)
  --scaling weak              every rank solves its own 1024 x 1024 share of an
                              (N*1024) x 1024 grid (the same cyclic rows):
                              the per-GPU work stays BASELINE's grid at every N

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling strong|weak]
                    [--config volcano|cstr|dmtm_drc|ch4|synthetic]
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
INPUTS = os.path.join(ROOT, 'tests', 'golden', 'inputs')

FP64_VECTOR_PEAK_TFLOPS = 78.6   # MI355X datasheet FP64 vector peak (the guides list no FP64 figure)
METRIC = 'steady-state MK solves/sec (whole node) on COOx volcano grid at 1/2/4/8 GPUs'


# ----------------------------------------------------------------------------
# algorithmic FLOPs of one RODAS4P step (structural nonzeros only)
# ----------------------------------------------------------------------------
def flops_per_step(plan):
    """fp64 FLOPs of one accepted RODAS4P step of kernel (3) on this plan,
    counting only structurally non-zero work (mk_solver.h: integrate / rhs /
    jac, mk_group.h for the lane-group path): 6 rate evaluations (5 stages +
    F0 at the accepted state), 1 Jacobian, 1 dense LU, 6 triangular solves,
    the stage combinations, the error norm and the site-balance projection.
    Integer/selects/compares, reciprocal refinements, the Newton polish,
    kernel (1) and the TOF are not counted: a lower bound."""
    from pycatkin_amd import _lib as L
    ip = plan.ip
    NS = len(plan.dyn)
    R = int(ip[L.I_NRXN])
    ef = ip[ip[L.I_OFF_EXPF]: ip[L.I_OFF_EXPF] + R * NS].reshape(R, NS).astype(int)
    er = ip[ip[L.I_OFF_EXPR]: ip[L.I_OFF_EXPR] + R * NS].reshape(R, NS).astype(int)
    S = plan.extra['S']
    dyn = plan.dp[ip[L.I_HDR + L.D_DYN]: ip[L.I_HDR + L.D_DYN] + 4 * NS].reshape(NS, 4)
    cf, rs0, rsT, fl = dyn[:, 0], dyn[:, 1], dyn[:, 2], dyn[:, 3]
    Cm = plan.conservation
    conc = int(np.sum(cf != 1.0))
    # rates: k * prod c^e per side, net, S accumulation
    rhs = conc + int(ef.sum() + er.sum()) + R + 2 * int(np.count_nonzero(S))
    rowsc = int(np.sum((rs0 != 1.0) | (rsT != 0.0))) + 2 * int(np.sum(rsT != 0.0))
    rhs += rowsc + 3 * int(np.sum(fl != 0.0))
    # Jacobian: per reaction side, per participant q: k e cf_q c_q^(e-1) prod_{i!=q} c_i^e_i
    jac = conc
    Jnz = np.zeros((NS, NS), bool)
    for j in range(R):
        parts = set()
        for e in (ef[j], er[j]):
            nz = np.nonzero(e)[0]
            tot = int(e.sum())
            for q in nz:
                parts.add(q)
                jac += int(e[q] != 1) + int(cf[q] != 1.0) + max(int(e[q]) - 1, 0) + (tot - int(e[q]))
        both = np.nonzero((ef[j] > 0) & (er[j] > 0))[0]
        jac += len(both)
        rows = np.nonzero(S[:, j])[0]
        jac += 2 * len(rows) * len(parts)
        for i in rows:
            for q in parts:
                Jnz[i, q] = True
    nnzJ = int(Jnz.sum())
    jac += nnzJ * int(np.any((rs0 != 1.0) | (rsT != 0.0))) + int(np.sum(fl != 0.0))
    w = NS + 2                                                   # W diagonal, 1/h, 1/(h g)
    lu = sum(1 + (NS - 1 - k) * (1 + 2 * (NS - 1 - k)) for k in range(NS))
    solve = 2 * NS * (NS - 1) + NS
    stages = NS * (sum(2 * (i - 1) for i in range(2, 6)) + 1 + 1  # u_2..u_5, u_6 = u_5 + k5, y_new
                   + sum(2 * (i - 1) + 1 for i in range(2, 7)))  # stage right-hand sides 2..6
    err = 6 * NS + 1
    proj = sum(2 * int(np.count_nonzero(Cm[l])) + 1 + int(np.count_nonzero(Cm[l])) for l in range(Cm.shape[0]))
    return int(6 * rhs + jac + w + lu + 6 * solve + stages + err + proj + 1)


# ----------------------------------------------------------------------------
# CPU baseline: the oracle (reference algorithm restated) on a bounded sample
# ----------------------------------------------------------------------------
def cpu_baseline(config, n_points=160, workers=16, seed=0, budget_s=25.0):
    """Oracle (numpy/scipy, the reference algorithm restated) on a bounded
    random sample of the same workload, in a process pool; stops after
    `budget_s` seconds and reports completed units / elapsed."""
    import multiprocessing as mp
    rng = np.random.default_rng(seed)
    pts = [(config, tuple(p)) for p in rng.uniform(0.0, 1.0, (n_points, 4))]
    ctx = mp.get_context('spawn')
    # one core per worker: the spawned interpreters inherit single-threaded BLAS
    keep = {k: os.environ.get(k) for k in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS')}
    os.environ.update({k: '1' for k in keep})
    try:
        pool = ctx.Pool(workers)
    finally:
        for k, v in keep.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        pool.map(_cpu_warm, range(workers))            # imports outside the timed sample
        t = time.time()
        done = 0
        it = pool.imap_unordered(_cpu_point, pts)
        # the sample ends at budget_s whether or not results keep arriving: a
        # worker can sit minutes on one stiff point (lsoda crawling through the
        # O-poisoned corner), and with every worker on one the loop would wait
        while True:
            left = budget_s - (time.time() - t)
            if left <= 0:
                break
            try:
                it.next(timeout=left)
            except StopIteration:
                break
            except mp.TimeoutError:
                break
            done += 1
        dt = time.time() - t
    finally:
        pool.terminate()
    return done / dt, dt, done


def host_cores():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU
    quota (cpu.max) when one is set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return n


# A one-GPU box is given 16 of the host's CPUs (the pool's rule for one GPU:
# nproc / os.cpu_count() report the whole machine there); the CPU baseline runs
# one worker per CPU of that share.
BOX_CPU_SHARE = 16


# which reference path the CPU baseline's oracle call restates, per config
CPU_PATH = dict(
    volcano='System.solve_odes with ode_solver "ode" (lsoda, the input\'s rtol 1e-8 / atol 1e-10) then the Newton '
            'polish of find_steady (old_system.py:315-468), i.e. activity(ss_solve=True) after a transient; this '
            'port runs at 0.785x the reference\'s own activity() per core (7.22 vs 9.20 solves/s, '
            'profiles/r3/cpu_reference_vs_port.json), so the reference itself would do ~1.27x this value',
    cstr='System.solve_odes (lsoda) + find_steady on the Pd111 CSTR (presets.run_temperatures, '
         'steady_state_solve=True)',
    dmtm_drc='System.degree_of_rate_control (2R+1 transients, old_system.py:490-515)',
    ch4='SteadyStateSolver.solve_ode (scipy BDF to 1e4 s, solver.py:374-418)',
    synthetic='System.solve_odes (scipy BDF) + find_steady on the synthetic network')


def _cpu_warm(_):
    from oracle import mk_oracle  # noqa: F401
    return 0


def _cpu_point(arg):
    """One unit of each config's workload on the oracle; u = 4 uniforms in [0, 1)."""
    config, u = arg
    from oracle import mk_oracle as O
    if config == 'volcano':
        spec = O.load_spec(os.path.join(INPUTS, 'COOxVolcano', 'input.json'))
        # the reference's volcano path: lsoda (input ode_solver 'ode') at the input tolerances, then the root
        return O.volcano_point(spec, -2.5 + 3.0 * u[0], -2.5 + 3.0 * u[1], steady=True, rtol=1e-8, atol=1e-10,
                               method='LSODA')['activity']
    if config == 'cstr':
        spec = O.load_spec(os.path.join(INPUTS, 'COOxReactor', 'input_Pd111.json'))
        m = O.ClassicModel(spec, T=423.0 + 200.0 * u[0])
        y, _ = m.solve_odes(method='LSODA')
        return m.find_steady(y)[0]
    if config == 'dmtm_drc':
        spec = O.load_spec(os.path.join(INPUTS, 'DMTM', 'input.json'))
        m = O.ClassicModel(spec, T=400.0 + 400.0 * u[0], p=10.0 ** (4.0 + 2.0 * u[1]))
        return m.drc(['r5', 'r9'], eps=5.0e-2, steady=False)['r9']
    if config == 'ch4':
        spec = O.ch4_setup(O.load_spec(os.path.join(INPUTS, 'CH4', 'input.json')), 1.0, 1.0)
        m = O.PatchedModel(spec, T=473.0 + 100.0 * u[0])
        y, _ = m.solve_ode(tmax=1e4, rtol=1e-10, atol=1e-12, method='BDF')
        return y[0]
    if config == 'synthetic':
        sys.path.insert(0, os.path.join(ROOT, 'tests'))
        from _synth import spec_of
        from pycatkin_amd.functions.synthetic import synthetic_network
        m = O.ClassicModel(spec_of(synthetic_network(), np.asarray(u) - 0.5), T=500.0)
        y, _ = m.solve_odes(rtol=1e-8, atol=1e-10)
        return m.find_steady(y)[0]
    raise KeyError(config)


def log(msg):
    print('[bench] ' + msg, file=sys.stderr, flush=True)


def profiled_counters(kernel_name, tag):
    """Per-launch PMC figures of `kernel_name` from the committed rocprofv3
    summary named in profiles/CURRENT (written by tools/pmc_summary.py from a
    tools/profile.sh run of this bench, same workload `tag`): (summary entry,
    path) or ({}, None)."""
    cur = os.path.join(ROOT, 'profiles', 'CURRENT')
    if not os.path.isfile(cur):
        return {}, None
    f = os.path.join(ROOT, open(cur).read().strip(), 'summary.json')
    try:
        s = json.load(open(f))
    except (OSError, ValueError):
        return {}, None
    def norm(name):      # 'pck::k_solve<pck::PlanCT<pck::nets::Volcano>, false>' -> 'k_solve<PlanCT<Volcano>>'
        return name.replace('pck::', '').replace('nets::', '').replace(' ', '').replace(',false', '')
    want = norm(kernel_name)
    for k, v in s.items():
        short = norm(k)
        if short == want and 'traffic_bytes' in v and v.get('tag', tag) == tag:
            return v, os.path.relpath(f, ROOT)
    return {}, None


# ----------------------------------------------------------------------------
# rank launcher (--gpus N outside torch.distributed.run)
# ----------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """Start n fresh rank processes of this script (nothing here has touched
    the GPU) and return the worst exit code; a failing rank ends the others."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0:
                rc = rc or (c if c > 0 else 128 - c)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


# ----------------------------------------------------------------------------
# workloads
# ----------------------------------------------------------------------------
class Workload:
    """One config's per-rank share: device inputs, a step() that launches the
    solve, and the result tensors of the last step."""
    kernel_name = ''
    units = 'solves'
    tag = ''

    def solved_units(self):
        return self.n_local


def _outputs(torch, net, n, L, _ptr):
    out = dict(y=torch.empty((net.NDYN, max(n, 1)), dtype=torch.float64, device='cuda'),
               tof=torch.empty(max(n, 1), dtype=torch.float64, device='cuda'),
               status=torch.empty(max(n, 1), dtype=torch.int32, device='cuda'),
               nsteps=torch.empty(max(n, 1), dtype=torch.int32, device='cuda'))
    o = L.Outputs()
    o.y, o.ld_y, o.tof, o.status, o.nsteps = _ptr(out['y']), max(n, 1), _ptr(out['tof']), _ptr(out['status']), \
        _ptr(out['nsteps'])
    return out, o


def _solve_workload(wl, sim, net, plan, n, T, p, desc, tof_terms, steady, activity, t_end=None, rtol=None,
                    atol=None, args=None):
    import torch
    from pycatkin_amd.classes.system import (ROOT_DIST, SCREEN_MARGIN, SCREEN_MAX_LANE_SPECIES, SCREEN_RTOL,
                                             STEADY_TRANSIENT)
    from pycatkin_amd import _lib as L
    from pycatkin_amd.engine import _ptr
    Tt, pp, d, fx, y0, inflow = sim._inputs(net, plan, n, T, p, desc, None, None, None)
    wl.cond, wl.keep = net.conditions(n, Tt, pp, d, fx, y0, inflow)
    times = sim.params['times']
    # steady-state solves: System.solve_batch(steady=True)'s rule -- the
    # transient at STEADY_TRANSIENT, the Newton root where the transient has
    # reached it to ROOT_DIST, else the transient end (DESIGN.md "Steady state")
    if steady:
        rtol = STEADY_TRANSIENT[0] if rtol is None else rtol
        atol = STEADY_TRANSIENT[1] if atol is None else atol
    wl.prm = net.params(t0=times[0], t_end=times[-1] if t_end is None else t_end,
                        rtol=args.rtol or (sim.params['rtol'] if rtol is None else rtol),
                        atol=args.atol or (sim.params['atol'] if atol is None else atol), max_steps=args.max_steps,
                        newton=steady and not args.no_newton, newton_iters=60, activity=activity,
                        retry=tuple(args.retry) if args.retry else None,
                        root_dist=(ROOT_DIST if args.root_dist is None else args.root_dist) if steady else 0.0)
    # the screening pass of System.solve_batch(steady=True, screen='auto'):
    # SCREEN_RTOL on networks of at most SCREEN_MAX_LANE_SPECIES dynamic
    # species, off beyond (--screen X forces it, --screen 0 turns it off)
    scr = ((SCREEN_RTOL if net.NDYN <= SCREEN_MAX_LANE_SPECIES else 0.0)
           if getattr(args, 'screen', None) is None else args.screen)
    if steady and wl.prm.newton and wl.prm.root_dist > 0.0 and not args.retry and scr > 0.0:
        wl.prm.screen_rtol = float(scr)
        wl.prm.screen_margin = SCREEN_MARGIN if getattr(args, 'screen_margin', None) is None else args.screen_margin
    wl.tolerances = (wl.prm.rtol, wl.prm.atol)
    wl.prm.wave_order = {'auto': 0, 'on': 1, 'off': -1}[getattr(args, 'wave_order', 'auto')]
    # solver launches per step: the first pass, the degenerate-root retry and,
    # on the lane solver with cost-ordered dispatch, its preview
    ordered = net.NDYN <= 8 and (wl.prm.wave_order == 1 or (wl.prm.wave_order == 0 and n >= 131072))
    # (the screening pass runs inside the first pass's launch)
    wl.solver_launches = 1 + int(bool(wl.prm.newton and wl.prm.retry_rtol > 0.0)) + int(ordered)
    wl.out, wl.o = _outputs(torch, net, n, L, _ptr)
    wl.kf = torch.empty((max(net.NRXN, 1), max(n, 1)), dtype=torch.float64, device='cuda')
    wl.kr = torch.empty_like(wl.kf)
    wl.net, wl.plan, wl.n_local = net, plan, n

    def step(sp):
        L.check(net.lib.pck_solve(net.h, C.byref(wl.cond), C.byref(wl.prm), C.byref(wl.o), sp))

    def rate_constants(sp):
        L.check(net.lib.pck_rate_constants(net.h, C.byref(wl.cond), _ptr(wl.kf), _ptr(wl.kr), max(n, 1), sp))
    wl.step, wl.rate_constants = step, rate_constants
    wl.status = lambda: wl.out['status'][:n]
    wl.nsteps = lambda: wl.out['nsteps'][:n]
    wl.result = lambda: wl.out['tof'][:n]
    # algorithmic HBM bytes of one solve launch: kf, kr in; y, tof, status, steps out
    wl.algo_bytes = n * (16 * net.NRXN + 8 * net.NDYN + 8 + 4 + 4)
    return wl


def volcano_workload(args, rank, world):
    import pycatkin_amd as P
    from pycatkin_amd.functions.volcano import set_volcano_energies, tile_order
    from pycatkin_amd.parallel import weak_grid_rows
    wl = Workload()
    sim = P.read_from_input_file(os.path.join(INPUTS, 'COOxVolcano', 'input.json'))
    set_volcano_energies(sim)
    plan = sim.plan(('CO_ox',))
    net = sim.device(('CO_ox',))
    net.set_plan_mode(2 if args.group else 1 if args.runtime_plan else 0)
    wl.kernel_name = ('k_solve_grp<4, 16>' if args.group else 'k_solve<PlanRT<4>>'
                      if (args.runtime_plan or not net.compiled_plan) else 'k_solve<PlanCT<Volcano>>')
    G = args.grid
    if args.scaling == 'strong':
        if G % world:
            raise SystemExit('--scaling strong needs the grid rows (%d) divisible by the ranks (%d)' % (G, world))
        rows = G // world
        wl.global_grid = (G, G)
    else:
        rows = G
        wl.global_grid = (G * world, G)
    wl.rows = rows
    eo = np.linspace(-2.5, 0.5, G)
    eco_loc = weak_grid_rows(rows, rank, world)          # cyclic rows of the global E_CO axis
    E1, E2 = np.meshgrid(eco_loc, eo, indexing='ij')
    n = E1.size
    wl.perm = tile_order(E1.shape, tuple(int(x) for x in args.tile.split('x'))) if args.order == 'tile' else None
    if wl.perm is not None:                              # one wave = one 16x4 patch of the grid (E_CO x E_O)
        E1, E2 = E1.ravel()[wl.perm], E2.ravel()[wl.perm]
    T = float(sim.params['temperature'])
    _solve_workload(wl, sim, net, plan, n, np.full(n, T), None, {'ECO': E1.ravel(), 'EO': E2.ravel()},
                    ('CO_ox',), True, True, args=args)
    # the profile tag names the per-GPU workload: a weak-scaling rank's share is
    # the same 1024 x 1024 solve at every N, so N > 1 lines carry its counters
    wl.tag = 'volcano %dx%d %s rtol %g atol %g' % (rows, G, args.order, wl.prm.rtol, wl.prm.atol) + \
        (' screen %g' % wl.prm.screen_rtol if wl.prm.screen_rtol > 0.0 else '')
    wl.config = {'workload': 'COOxVolcano %dx%d (E_CO x E_O) grid, %s over %d GPU(s): %d E_CO rows x %d E_O per rank, '
                             'T=600 K, transient to t_end=3600 s at rtol %g / atol %g, Newton steady-state polish, '
                             'the root where the transient has reached it to %g (else the transient end), activity%s'
                             % (wl.global_grid[0], wl.global_grid[1], 'sharded' if args.scaling == 'strong'
                                else 'one grid share per GPU', world, rows, G, wl.prm.rtol, wl.prm.atol,
                                wl.prm.root_dist,
                                '; screening pass at rtol %g accepting roots within %g of its transient end, the '
                                'rest solved again at rtol %g' % (wl.prm.screen_rtol,
                                                                  wl.prm.screen_margin * wl.prm.root_dist,
                                                                  wl.prm.rtol)
                                if wl.prm.screen_rtol > 0.0 else ''),
                 'global_grid': list(wl.global_grid), 'grid_per_gpu': [rows, G],
                 'parallelism': 'dp%d' % world, 'shard': 'cyclic E_CO rows',
                 'order': 'row' if wl.perm is None else 'tile %s' % args.tile}
    wl.data = 'synthetic descriptor grid (E_CO, E_O in [-2.5, 0.5] eV) on the reference COOxVolcano network'
    return wl


def _shard(x, rank, world):
    return np.asarray(x)[rank::world]


def cstr_workload(args, rank, world):
    import pycatkin_amd as P
    wl = Workload()
    sim = P.read_from_input_file(os.path.join(INPUTS, 'COOxReactor', 'input_Pd111.json'))
    plan = sim.plan(('CO_ox',))
    net = sim.device(('CO_ox',))
    if args.group:
        net.set_plan_mode(2)
    n_tot = args.n or 10000
    T = _shard(np.linspace(423.0, 623.0, n_tot if args.scaling == 'strong' else n_tot * world), rank, world)
    _solve_workload(wl, sim, net, plan, T.size, T, None, None, ('CO_ox',), True, False, args=args)
    wl.kernel_name = ('k_solve_grp<6, 16>' if args.group else
                      'k_solve<PlanCT<CstrPd111>>' if net.compiled_plan else 'k_solve<PlanRT<6>>')
    wl.tag = 'cstr %d' % n_tot
    wl.config = {'workload': 'COOxReactor Pd111 CSTR temperature sweep: %d temperatures 423-623 K, t_end 3600 s '
                             '(input rtol 1e-8 / atol 1e-10) + Newton steady state' % n_tot,
                 'parallelism': 'dp%d' % world}
    wl.data = 'reference examples/COOxReactor Pd111 input (OUTCAR / log.vib thermochemistry), temperature grid'
    return wl


def ch4_workload(args, rank, world):
    import pycatkin_amd as P
    wl = Workload()
    sim = P.read_from_input_file(os.path.join(INPUTS, 'CH4', 'input.json'), formulation='patched')
    for r, s in (('C_ads', 'sC'), ('O_ads', 'sO')):
        sim.reactions[r].dErxn_user = 1.0
        sim.states[s].Gelec = 1.0
    plan = sim.plan()
    net = sim.device()
    n_tot = args.n or 16384
    T = _shard(np.linspace(473.0, 573.0, n_tot if args.scaling == 'strong' else n_tot * world), rank, world)
    _solve_workload(wl, sim, net, plan, T.size, T, None, None, (), False, False, t_end=1e4, rtol=1e-10, atol=1e-12,
                    args=args)
    wl.kernel_name = 'k_solve_grp<16, 16>'
    wl.tag = 'ch4 %d' % n_tot
    wl.config = {'workload': 'test/CH4_input.json (patched System, 16 surface species / 58 reactions, descriptors '
                             'E_C = E_O = 1 eV), SteadyStateSolver.solve_ode to 1e4 s (rtol 1e-10 / atol 1e-12) '
                             'at %d temperatures 473-573 K' % n_tot,
                 'parallelism': 'dp%d' % world}
    wl.data = 'reference test/CH4_input.json, temperature grid'
    return wl


SYNTHETIC_TOL = (1.0e-7, 1.0e-22)


def synthetic_workload(args, rank, world):
    from pycatkin_amd.functions.synthetic import synthetic_system
    wl = Workload()
    sim, _ = synthetic_system()
    plan = sim.plan(('R0',))
    net = sim.device(('R0',))
    n_tot = args.n or 65536
    rng = np.random.default_rng(0)
    D = _shard(rng.uniform(-0.5, 0.5, (n_tot if args.scaling == 'strong' else n_tot * world, 4)), rank, world)
    n = D.shape[0]
    # the steady rule's transient at rtol 1e-7: at the default 1e-6 two of the
    # 324 fixture rows miss the 1e-6 bound against the oracle's rtol 1e-11
    # transient (profiles/r4/synthetic_tol_probe.jsonl)
    _solve_workload(wl, sim, net, plan, n, np.full(n, 500.0), None, {'D%d' % k: D[:, k] for k in range(4)},
                    ('R0',), True, False, rtol=SYNTHETIC_TOL[0], atol=SYNTHETIC_TOL[1], args=args)
    wl.kernel_name = 'k_solve_grp<50, 64>'
    wl.tag = 'synthetic %d' % n_tot
    wl.config = {'workload': 'synthetic 50 species / 150 reactions, %d random-descriptor conditions, T=500 K, '
                             'transient to t_end 1e4 s at rtol %g / atol %g + Newton, steady rule (root where '
                             'reached, else the transient end)' % ((n_tot,) + SYNTHETIC_TOL),
                 'parallelism': 'dp%d' % world}
    wl.data = 'synthetic network (functions/synthetic.py), uniform random descriptors in [-0.5, 0.5] eV'
    return wl


def dmtm_drc_workload(args, rank, world):
    import torch
    import pycatkin_amd as P
    from pycatkin_amd import _lib as L
    from pycatkin_amd.engine import _ptr
    wl = Workload()
    sim = P.read_from_input_file(os.path.join(INPUTS, 'DMTM', 'input.json'))
    plan = sim.plan(('r5', 'r9'))
    net = sim.device(('r5', 'r9'))
    g = int(round(np.sqrt(args.n))) if args.n else 64
    TT, pp = np.meshgrid(np.linspace(400.0, 800.0, g), np.logspace(4.0, 6.0, g), indexing='ij')
    T, p = _shard(TT.ravel(), rank, world), _shard(pp.ravel(), rank, world)
    n = T.size
    Tt, p2, d, fx, y0, inflow = sim._inputs(net, plan, n, T, p, None, None, None, None)
    wl.cond, wl.keep = net.conditions(n, Tt, p2, d, fx, y0, inflow)
    times = sim.params['times']
    wl.prm = net.params(t0=times[0], t_end=times[-1], rtol=sim.params['rtol'], atol=sim.params['atol'],
                        max_steps=args.max_steps, newton=False, drc_eps=5.0e-2)
    xi = torch.zeros((net.NRXN, max(n, 1)), dtype=torch.float64, device='cuda')
    tof0 = torch.empty(max(n, 1), dtype=torch.float64, device='cuda')
    st = torch.zeros(max(n, 1), dtype=torch.int32, device='cuda')
    ns = torch.zeros(max(n, 1), dtype=torch.int32, device='cuda')

    def step(sp):
        L.check(net.lib.pck_drc(net.h, C.byref(wl.cond), C.byref(wl.prm), _ptr(xi), max(n, 1), _ptr(tof0), _ptr(st),
                                _ptr(ns), sp))
    wl.step, wl.rate_constants = step, None
    wl.status, wl.nsteps, wl.result = (lambda: st[:n]), (lambda: ns[:n]), (lambda: tof0[:n])
    wl.net, wl.plan, wl.n_local = net, plan, n
    wl.algo_bytes = n * (8 * net.NRXN + 8 + 4 + 4)
    wl.kernel_name = 'k_solve_grp<16, 16>'
    wl.units = 'DRC conditions'
    wl.tag = 'dmtm_drc %dx%d' % (g, g)
    wl.config = {'workload': 'DMTM degree of rate control (TOF = r5 + r9, eps 5e-2, 2R+1 = 23 transient solves to '
                             't = 1e12 s per condition at the input tolerances rtol 1e-6 / atol 1e-8, as '
                             'run_temperatures(tof_terms=...) calls it) on a %dx%d grid of T 400-800 K x p 1e4-1e6 Pa'
                             % (g, g), 'parallelism': 'dp%d' % world}
    wl.data = 'reference examples/DMTM input, (T, p) grid'
    return wl


CONFIGS = dict(volcano=volcano_workload, cstr=cstr_workload, ch4=ch4_workload, synthetic=synthetic_workload,
               dmtm_drc=dmtm_drc_workload)


# ----------------------------------------------------------------------------
# CPU stand-in (tests only): the launcher / sharding / gather / reductions on
# gloo without a GPU or the HIP library
# ----------------------------------------------------------------------------
def cpu_standin_workload(args, rank, world):
    import torch
    from pycatkin_amd.parallel import weak_grid_rows
    wl = Workload()
    G = args.grid
    rows = G // world if args.scaling == 'strong' else G
    wl.global_grid = (G, G) if args.scaling == 'strong' else (G * world, G)
    wl.rows = rows
    eco = weak_grid_rows(rows, rank, world)
    E1, E2 = np.meshgrid(eco, np.linspace(-2.5, 0.5, G), indexing='ij')
    wl.perm = None
    val = torch.from_numpy(E1.ravel() * 10.0 + E2.ravel())
    st = torch.from_numpy(((np.arange(E1.size) + rank) % 7 == 0).astype(np.int32) * 4)   # a few 'degenerate'
    wl.n_local = E1.size
    wl.step = lambda sp: None
    wl.rate_constants = None
    wl.status, wl.nsteps, wl.result = (lambda: st), (lambda: torch.ones(E1.size, dtype=torch.int32)), (lambda: val)
    wl.config = {'workload': 'CPU stand-in of the volcano grid layout', 'global_grid': list(wl.global_grid),
                 'grid_per_gpu': [rows, G], 'parallelism': 'dp%d' % world}
    wl.data = 'stand-in'
    return wl


def build_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    # defaults: volcano 20 timed after 10 untimed steps (the clock ramps over
    # the first few: profiles/r4/volcano trace, the solve launch 6.97 -> 5.68 ms
    # over 8 steps; 10 untimed steps cost ~60 ms); the other configs 5 after 2
    ap.add_argument('--steps', type=int, default=None)
    ap.add_argument('--warmup', type=int, default=None)
    ap.add_argument('--config', choices=sorted(CONFIGS), default='volcano')
    ap.add_argument('--scaling', choices=('strong', 'weak'), default='strong')
    ap.add_argument('--grid', type=int, default=1024)
    ap.add_argument('--n', type=int, default=0, help='conditions of the non-volcano configs (0: config default)')
    ap.add_argument('--max-steps', type=int, default=200000, help='integrator step budget per condition (library default)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-points', type=int, default=4000,
                    help='CPU baseline sample (stopped after 25 s of wall time)')
    ap.add_argument('--no-newton', action='store_true', help='A/B diagnostic: transient only (not the bench workload)')
    ap.add_argument('--rtol', type=float, default=0.0, help='A/B: first-pass rtol (0: the input\'s)')
    ap.add_argument('--atol', type=float, default=0.0, help='A/B: first-pass atol (0: the input\'s)')
    ap.add_argument('--retry', type=float, nargs=2, default=None, metavar=('RTOL', 'ATOL'),
                    help='A/B: integrate the status-4 conditions again at these tolerances (default: no retry)')
    ap.add_argument('--screen-margin', type=float, default=None,
                    help='screening acceptance as a fraction of the root distance (default SCREEN_MARGIN; A/B)')
    ap.add_argument('--screen', type=float, default=None,
                    help='screening-pass rtol of steady solves (default SCREEN_RTOL; 0: off)')
    ap.add_argument('--root-dist', type=float, default=None,
                    help='A/B: pck_solve_params.root_dist of steady solves (default ROOT_DIST)')
    ap.add_argument('--emulate', default=None, metavar='R/N',
                    help='single-GPU A/B: solve the shard rank R of N would own, without a process group')
    ap.add_argument('--wave-order', choices=('auto', 'on', 'off'), default='auto',
                    help='cost-ordered wavefront dispatch of the lane solver (pck_solve_params.wave_order)')
    ap.add_argument('--tile', default='16x4', help='patch shape (rows x cols) of --order tile')
    ap.add_argument('--order', choices=('tile', 'row'), default='tile',
                    help="condition order in HBM: 'tile' = one grid patch per wave (default), 'row' = row-major")
    ap.add_argument('--runtime-plan', action='store_true',
                    help='A/B: force the runtime-plan solver instead of the compiled-in network')
    ap.add_argument('--group', action='store_true',
                    help='A/B (cstr, volcano): one 16-lane group per condition (the lane-group solver) instead of one lane')
    ap.add_argument('--device', choices=('gpu', 'cpu-standin'), default='gpu', help=argparse.SUPPRESS)
    return ap


def _heartbeat(period=45.0):
    """A line on stderr every `period` s from a daemon thread: one solver
    launch of a large config (synthetic 1e6) runs for minutes without output,
    and a GPU-box harness takes a silent process for a hung one."""
    import threading

    def beat():
        t0 = time.time()
        while True:
            time.sleep(period)
            log('alive, %.0f s' % (time.time() - t0))
    threading.Thread(target=beat, daemon=True).start()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = build_parser().parse_args(argv)
    if args.steps is None:
        args.steps = 20 if args.config == 'volcano' else 5
    if args.warmup is None:
        args.warmup = 10 if args.config == 'volcano' else 2
    _heartbeat()

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        if args.emulate:
            raise SystemExit('--emulate is a single-process diagnostic; do not combine it with --gpus N')
        sys.exit(launch_ranks(args.gpus, argv))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1 and args.emulate:
        raise SystemExit('--emulate runs without a process group (WORLD_SIZE must be 1)')
    if world > 1 and args.gpus != world:
        log('rank %d: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE' % (rank, args.gpus, world))
    cpu = args.device == 'cpu-standin'
    import torch
    dist = None
    if cpu:
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group('gloo')
    else:
        torch.cuda.set_device(local)
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    shard_rank, shard_world = (rank, world) if not args.emulate else map(int, args.emulate.split('/'))
    wl = (cpu_standin_workload if cpu else CONFIGS[args.config])(args, shard_rank, shard_world)
    sp = C.c_void_p(0 if cpu else torch.cuda.current_stream().cuda_stream)
    stream = None if cpu else torch.cuda.current_stream()
    sync = (lambda: None) if cpu else torch.cuda.synchronize
    n = wl.n_local

    log('rank %d/%d: %s, %d local units, warmup %d' % (rank, world, args.config, n, args.warmup))
    for _ in range(args.warmup):
        wl.step(sp)
    sync()
    if dist:
        dist.barrier()
    sync()
    ev = [] if cpu else [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                         for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        if ev:
            ev[k][0].record(stream)
        wl.step(sp)
        if ev:
            ev[k][1].record(stream)
    sync()
    if dist:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    solve_ms = float(np.mean([a.elapsed_time(b) for a, b in ev])) if ev else 0.0
    k1_ms = 0.0
    if wl.rate_constants is not None and ev:
        # kernel (1) alone, same stream, to split pck_solve's two launches
        e1 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in e1:
            a.record(stream)
            wl.rate_constants(sp)
            b.record(stream)
        sync()
        k1_ms = float(np.mean([a.elapsed_time(b) for a, b in e1]))
    k3_ms = max(solve_ms - k1_ms, 1e-9)

    dev = 'cpu' if cpu else 'cuda'
    st = wl.status()
    counts = torch.tensor([int((st == 0).sum()), int((st == 4).sum()), int(((st != 0) & (st != 4) & (st != 5)).sum()),
                           n, int((st == 1).sum()), int((st == 2).sum()), int((st == 3).sum()), int((st == 5).sum())],
                          dtype=torch.int64, device=dev)
    ns = wl.nsteps().double()
    steps_local = float(ns.sum())
    pad = (-n) % 64
    wave_max = torch.nn.functional.pad(ns, (0, pad)).reshape(-1, 64).max(dim=1).values if n else ns
    lane_eff = float(ns.mean() / wave_max.mean()) if n else 1.0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt)
        dist.all_reduce(counts)
        # final gather of the results (RCCL over xGMI), outside the timed region
        res = wl.result().contiguous()
        gathered = [torch.empty_like(res) for _ in range(world)]
        dist.all_gather(gathered, res)
        if hasattr(wl, 'global_grid'):
            from pycatkin_amd.parallel import assemble_weak_grid
            act_map = assemble_weak_grid(gathered, wl.rows, args.grid, wl.perm, True)
            assert tuple(act_map.shape) == tuple(wl.global_grid), (act_map.shape, wl.global_grid)
            if cpu and rank == 0:
                E1, E2 = np.meshgrid(np.linspace(-2.5, 0.5, wl.global_grid[0]), np.linspace(-2.5, 0.5, args.grid),
                                     indexing='ij')
                assert np.allclose(act_map.numpy(), E1 * 10.0 + E2), 'gathered grid out of order'
    n_ok, n_degen, n_fail, n_total, n_maxsteps, n_stepfail, n_nonfinite, n_loose = (int(x) for x in counts.tolist())
    per_step = elapsed / args.steps
    value = n_total / per_step

    if rank == 0:
        roof, cpu_line = None, None
        if not cpu:
            fps = flops_per_step(wl.plan)
            fl_struct = fps * steps_local
            # a group network of at most 16 species ran on the quad kernel
            # unless it was kept on the 16-lane one (pck_network_group_lanes)
            if wl.kernel_name == 'k_solve_grp<16, 16>' and wl.net.group_lanes() == 4:
                wl.kernel_name = 'k_solve_q4<Jit>'
            pmc, traffic_src = profiled_counters(wl.kernel_name, wl.tag)
            # launches of the solver kernel per step (first pass, retry over the
            # compacted list, cost-order preview): the profile's per-launch
            # averages times this are per-step totals
            nl = getattr(wl, 'solver_launches', 1)
            traffic = pmc['traffic_bytes'] * nl if 'traffic_bytes' in pmc else None
            # the smaller of the structural count and the fp64 instruction
            # counters of the committed profile of this same workload (which
            # count exec-masked lanes too, so they are an upper bound themselves)
            fl_pmc = pmc['f64_flops_counted'] * nl if 'f64_flops_counted' in pmc else None
            fl = min(fl_struct, fl_pmc) if fl_pmc else fl_struct
            achieved = fl / (k3_ms * 1e-3) / 1e12
            roof = {'bound': 'mfma' if False else 'valu_fp64', 'achieved': achieved, 'peak': FP64_VECTOR_PEAK_TFLOPS,
                    'unit': 'TFLOP/s', 'frac': achieved / FP64_VECTOR_PEAK_TFLOPS, 'traffic': traffic,
                    'traffic_unit': 'bytes per step over the solver launches (rocprofv3 PMC FETCH_SIZE x2 + '
                                    'WRITE_SIZE, per-launch average x solver launches per step)',
                    'traffic_source': traffic_src, 'algorithmic_bytes': wl.algo_bytes,
                    'kernel': wl.kernel_name, 'kernel_ms': k3_ms, 'rate_constants_ms': k1_ms,
                    'flops_per_bench_step': fl, 'flops_structural': fl_struct, 'flops_pmc_f64': fl_pmc,
                    'flops_per_integrator_step': fps, 'flop_count': 'min(structural nonzeros of one accepted RODAS4P step x '
                    'integrator steps of rank 0 (every solver pass: screening + full, or first pass + retry; the preview, Newton polish, kernel 1 and TOF not counted), '
                    '64 x (ADD+MUL+TRANS) + 128 x FMA fp64 wave instructions of the committed PMC profile of this '
                    'workload, per launch x solver launches per step)',
                    'integrator_steps': steps_local, 'lane_efficiency': lane_eff, 'solver_launches_per_step': nl}
            if not args.no_cpu_baseline:
                # N > 1: stated once for the node, on rank 0 after the timed
                # region (the other ranks wait in the closing barrier); the
                # node's CPU share is BOX_CPU_SHARE per GPU
                avail = host_cores()
                workers = min(BOX_CPU_SHARE * world, avail)
                log('cpu baseline: %d points, %d workers' % (args.cpu_points, workers))
                v, dt, done = cpu_baseline(args.config, args.cpu_points, workers)
                cpu_line = dict(value=v, unit='%s/s' % wl.units, cores=workers, kind='port',
                                sample='%d random units of the same %s workload solved in %.1f s by the oracle '
                                       '(numpy/scipy restatement of the reference path: %s), %d single-threaded '
                                       'worker processes = %d GPU(s) x the %d-CPU share per GPU (affinity/cgroup '
                                       'show %d, os.cpu_count() %d for the whole host)'
                                       % (done, args.config, dt, CPU_PATH.get(args.config, ''), workers, world,
                                          BOX_CPU_SHARE, avail, os.cpu_count() or 0))
        line = {
            'metric': METRIC if args.config == 'volcano' else
            '%s/sec (whole node), BASELINE config %s' % (wl.units, args.config),
            'value': value, 'unit': '%s/s' % wl.units, 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': per_step * 1e3, 'higher_is_better': True, 'scaling': args.scaling, 'vs_baseline': None,
            'dtype': 'f64', 'data': wl.data, 'config': wl.config, 'roofline': roof, 'cpu_baseline': cpu_line,
            'status': {'regular_root': n_ok, 'degenerate_root_tight_transient': n_degen,
                       'degenerate_root_input_tolerance_transient': n_loose, 'failed': n_fail,
                       'units': n_total, 'failed_by_code': {'max_steps': n_maxsteps, 'step_failure': n_stepfail,
                                                            'non_finite': n_nonfinite}},
        }
        if args.emulate:
            line['config']['emulated_shard'] = args.emulate
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
