"""Diagnostic (GPU): the lane-vs-group status split of
tests/test_gpu_group.py::test_group_solver_matches_lane_solver_on_volcano.

The same 1024 volcano points (seed 11) through every solver path, each run
twice, before and after unrelated GPU work, so that a path whose answer
depends on process state shows up as a difference between its own repeats:

  lane_rt   runtime-plan lane solver   (set_plan_mode(1), k_solve<PlanRT<4>>)
  lane_ct   compiled-in lane solver    (set_plan_mode(0), k_solve<PlanCT<Volcano>>)
  grp_ct    lane-group solver, network compiled in (set_plan_mode(2), hipRTC)
  grp_tab   lane-group solver, record tables (PCK_GRP_CT=0)
  grp_builtin  lane-group solver, compiled-in padded kernel (PCK_JIT=0)

for the steady rule and for the transient alone (STEADY_TRANSIENT).

    python tools/diag_split.py [OUTDIR]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, 'gpurun_out', 'diag_split')
    os.makedirs(out_dir, exist_ok=True)
    import pycatkin_amd as P
    from pycatkin_amd.classes.system import STEADY_TRANSIENT
    from pycatkin_amd.functions.volcano import set_volcano_energies
    s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    rng = np.random.default_rng(11)
    n = 1024
    kw = dict(T=np.full(n, 600.0), desc={'ECO': rng.uniform(-2.5, 0.5, n), 'EO': rng.uniform(-2.5, 0.5, n)},
              tof_terms=('CO_ox',), activity=True)
    modes = {'lane_rt': (1, {}), 'lane_ct': (0, {}), 'grp_ct': (2, {}), 'grp_tab': (2, {'PCK_GRP_CT': '0'}),
             'grp_builtin': (2, {'PCK_JIT': '0'})}
    res = {}

    def run(tag, mode, env, steady):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        set_volcano_energies(s)
        net = s.device(('CO_ox',))
        net.set_plan_mode(mode)
        try:
            if steady:
                r = s.solve_batch(steady=True, **kw)
            else:
                r = s.solve_batch(rtol=STEADY_TRANSIENT[0], atol=STEADY_TRANSIENT[1], **kw)
        finally:
            net.set_plan_mode(0)
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        res[tag] = r
        st = r['status']
        print('%-22s plan %3d grp %d  statuses %s  steps %d' % (
            tag, net.plan_id(), net.group_kernel(), dict(zip(*[a.tolist() for a in np.unique(st, return_counts=True)])),
            int(r['nsteps'].sum())), flush=True)

    def sweep(rep):
        for name, (mode, env) in modes.items():
            run('%s/steady/%d' % (name, rep), mode, env, True)
            run('%s/transient/%d' % (name, rep), mode, env, False)

    sweep(0)
    sweep(1)
    # unrelated GPU work in between: a 256 x 256 volcano grid on the product
    # path and a DMTM lane-group solve
    from pycatkin_amd.functions.volcano import volcano_activity
    be = np.linspace(-2.5, 0.5, 256)
    volcano_activity(s, be, be, steady=True)
    d = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'DMTM', 'input.json'))
    d.solve_batch(T=np.linspace(400, 800, 512), steady=True)
    sweep(2)

    summary = {}
    for kind in ('steady', 'transient'):
        for name in modes:
            a = res['%s/%s/0' % (name, kind)]
            for rep in (1, 2):
                b = res['%s/%s/%d' % (name, kind, rep)]
                key = '%s/%s rep0 vs rep%d' % (name, kind, rep)
                summary[key] = dict(status_diff=int((a['status'] != b['status']).sum()),
                                    y_bitwise_diff=int((a['y'] != b['y']).any(axis=0).sum()),
                                    steps_diff=int((a['nsteps'] != b['nsteps']).sum()))
        for rep in (0, 1, 2):
            ref = res['lane_ct/%s/%d' % (kind, rep)]
            for name in modes:
                if name == 'lane_ct':
                    continue
                b = res['%s/%s/%d' % (name, kind, rep)]
                pairs = {}
                for x, y in zip(ref['status'].tolist(), b['status'].tolist()):
                    pairs['%d,%d' % (x, y)] = pairs.get('%d,%d' % (x, y), 0) + 1
                ok = (ref['status'] == 0) & (b['status'] == 0)
                rel = np.abs(b['tof'] - ref['tof']) / np.maximum(np.abs(ref['tof']), 1e-300)
                summary['lane_ct vs %s/%s/%d' % (name, kind, rep)] = dict(
                    pairs=pairs, max_rel_act_both0=float(rel[ok].max()) if ok.any() else None,
                    max_rel_act_all=float(np.nanmax(rel)))
    # every steady run against the oracle's rule and roots
    # (tests/golden/split_fixture.npz, make_split_fixture.py)
    fx = np.load(os.path.join(ROOT, 'tests', 'golden', 'split_fixture.npz'))
    reg, yr = fx['regular'], fx['y_root'].T
    for tag, r in res.items():
        if '/steady/' not in tag:
            continue
        ok = (r['status'] == 0) & reg
        dev = np.abs(r['y'][:, ok] - yr[:, ok]) / np.abs(yr[:, ok])
        summary['%s vs oracle' % tag] = dict(status_off=int(((r['status'] == 0) != reg).sum()),
                                             max_root_dev=float(dev.max()) if ok.any() else None,
                                             n_dev_1e10=int((dev.max(0) > 1e-10).sum()) if ok.any() else 0)
    for k, v in summary.items():
        print(k, json.dumps(v), flush=True)
    json.dump(summary, open(os.path.join(out_dir, 'summary.json'), 'w'), indent=1)
    np.savez_compressed(os.path.join(out_dir, 'runs.npz'), ECO=kw['desc']['ECO'], EO=kw['desc']['EO'],
                        **{k.replace('/', '__') + '__' + f: v[f] for k, v in res.items()
                           for f in ('status', 'tof', 'y', 'nsteps')})


if __name__ == '__main__':
    main()
