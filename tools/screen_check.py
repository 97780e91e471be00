"""Diagnostic (GPU): the screening pass (pck_solve_params.screen_rtol) against
the single pass on the bench workload -- the 1024 x 1024 COOxVolcano grid
(patch order, cost-ordered dispatch, steady rule) -- node by node.

    python tools/screen_check.py [OUT.json] [--screen RTOL] [--margin M] [--config volcano|cstr]

Reports the status pairs (single, screened), the largest relative activity
difference on nodes with equal status (roots: the same root to rounding;
transient ends: the same solve, bitwise), and the nodes whose status differs
with their single-pass root distance (where the rule sits near its bound).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    args = sys.argv[1:]
    opt = {}
    config = 'volcano'
    if '--config' in args:
        i = args.index('--config')
        config = args[i + 1]
        del args[i:i + 2]
    for k in ('--screen', '--margin', '--grid'):
        if k in args:
            i = args.index(k)
            opt[k] = float(args[i + 1])
            del args[i:i + 2]
    import torch
    import pycatkin_amd as P
    from pycatkin_amd.classes import system as S
    from pycatkin_amd.functions.volcano import set_volcano_energies, tile_order
    if '--margin' in opt:
        S.SCREEN_MARGIN = opt['--margin']
    G = int(opt.get('--grid', 1024))
    if config == 'cstr':
        # the bench's CSTR sweep (COOxReactor Pd111, 1e4 temperatures, steady rule)
        s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxReactor', 'input_Pd111.json'))
        T = np.linspace(423.0, 623.0, 10000)
        order = np.arange(T.size)
        ECO = EO = np.full(T.size, np.nan)
        kw = dict(T=T, tof_terms=('CO_ox',), steady=True, activity=False)
    else:
        s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
        set_volcano_energies(s)
        be = np.linspace(-2.5, 0.5, G)
        ECO, EO = np.meshgrid(be, be, indexing='ij')
        order = tile_order((G, G))
        kw = dict(T=np.full(order.size, 600.0), desc={'ECO': ECO.ravel()[order], 'EO': EO.ravel()[order]},
                  tof_terms=('CO_ox',), steady=True, activity=True)
    res = {}
    for name, scr in (('single', None), ('screened', opt.get('--screen', S.SCREEN_RTOL))):
        s.solve_batch(screen=scr, **kw)                       # warm (hipRTC, allocator)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = s.solve_batch(screen=scr, **kw)
        torch.cuda.synchronize()
        r['wall_ms'] = 1e3 * (time.perf_counter() - t0)
        res[name] = r
    a, b = res['single'], res['screened']
    pairs = {}
    for x, y in zip(a['status'].tolist(), b['status'].tolist()):
        pairs['%d->%d' % (x, y)] = pairs.get('%d->%d' % (x, y), 0) + 1
    same = a['status'] == b['status']
    rel = np.abs(b['tof'] - a['tof']) / np.maximum(np.abs(a['tof']), 1e-300)
    diff = np.nonzero(~same)[0]
    out = dict(config=config, grid=G, screen_rtol=opt.get('--screen', S.SCREEN_RTOL), margin=S.SCREEN_MARGIN,
               wall_ms={k: v['wall_ms'] for k, v in res.items()},
               steps={k: int(v['nsteps'].astype(np.int64).sum()) for k, v in res.items()},
               status_pairs=pairs, n_status_differs=int(diff.size),
               max_rel_activity_same_status_0=float(rel[same & (a['status'] == 0)].max(initial=0.0)),
               max_rel_activity_same_status_4=float(rel[same & (a['status'] == 4)].max(initial=0.0)),
               bitwise_equal_status_4=int(np.sum((b['tof'] == a['tof']) & same & (a['status'] == 4))),
               n_status_4=int(np.sum(same & (a['status'] == 4))),
               differing=[dict(node=int(order[i]), eco=float(ECO.ravel()[order[i]]), eo=float(EO.ravel()[order[i]]),
                               single=int(a['status'][i]), screened=int(b['status'][i]),
                               act_single=float(a['tof'][i]), act_screened=float(b['tof'][i]))
                          for i in diff[:50]])
    print(json.dumps(out, indent=1))
    if args:
        json.dump(out, open(args[0], 'w'), indent=1)


if __name__ == '__main__':
    main()
