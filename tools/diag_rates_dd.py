"""Diagnostic (GPU): the Newton refinement's double-double residual
(mk_solver.h: rhs_dd, through pck_species_rates with PCK_RATES_DD=1) and the
plain one (rhs) at the oracle's roots of the 1024 split-fixture volcano points,
against the exact rational residual of the oracle (ClassicModel.rhs_exact),
each relative to the species' gross flux.

    python tools/diag_rates_dd.py [OUT.json]
"""
import copy
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import pycatkin_amd as P
    from oracle import mk_oracle as O
    from pycatkin_amd.functions.volcano import set_volcano_energies
    fx = np.load(os.path.join(ROOT, 'tests', 'golden', 'split_fixture.npz'))
    s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    plan = s.plan(('CO_ox',))
    net = s.device(('CO_ox',))
    n = fx['ECO'].size
    desc = {'ECO': fx['ECO'], 'EO': fx['EO']}
    T = np.full(n, 600.0)
    Tt, p, d, fix, _, inflow = s._inputs(net, plan, n, T, None, desc, None, None, None)
    kf, kr = net.rate_constants(n, Tt, p, d)
    y = np.ascontiguousarray(fx['y_root'].T)
    plain = net.species_rates(n, Tt, p, y, kf, kr, d, fix, inflow).cpu().numpy()
    os.environ['PCK_RATES_DD'] = '1'
    ddr = net.species_rates(n, Tt, p, y, kf, kr, d, fix, inflow).cpu().numpy()
    os.environ.pop('PCK_RATES_DD')
    spec = O.load_spec(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    ks = list(range(0, n, 8))
    err_dd, err_pl = [], []
    for k in ks:
        sp = copy.deepcopy(spec)
        O.set_volcano_point(sp, fx['ECO'][k], fx['EO'][k])
        m = O.ClassicModel(sp)
        full = m.y0.copy()
        full[[m.idx[q] for q in plan.dyn]] = y[:, k]
        ex = m.rhs_exact(full)[[m.idx[q] for q in plan.dyn]]
        g = m.gross_flux(full)[[m.idx[q] for q in plan.dyn]]
        err_dd.append(np.abs(ddr[:, k] - ex) / g)
        err_pl.append(np.abs(plain[:, k] - ex) / g)
    err_dd, err_pl = np.array(err_dd), np.array(err_pl)
    out = dict(points=len(ks), dd_max_per_species=err_dd.max(0).tolist(), plain_max_per_species=err_pl.max(0).tolist(),
               dd_worst=[int(ks[i]) for i in np.argsort(-err_dd.max(1))[:5]])
    print(json.dumps(out))
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], 'w'), indent=1)


if __name__ == '__main__':
    main()
