"""Time the REFERENCE PyCatKin volcano path next to the oracle port that
bench.py's cpu_baseline runs (the reference cannot travel to the GPU box, so
the bench times the port; this states how the two compare).  Runs in the
build container only, single-threaded, on the same random grid points:

  reference  old_system.System.activity(tof_terms=['CO_ox']) -- the volcano
             driver's call (cooxvolcano.py:47: lsoda transient to 3600 s at
             the input's tolerances), and with ss_solve=True (+ find_steady's
             least_squares polish), with the duck-typed states of
             make_golden.py
  port       oracle.mk_oracle.volcano_point(steady=True, method='LSODA'),
             bench.py: _cpu_point('volcano')

    OMP_NUM_THREADS=1 python tests/golden/time_reference.py [N]
writes profiles/r3/cpu_reference_vs_port.json
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)

from make_golden import O, REF, build_reference_system  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    rng = np.random.default_rng(0)
    pts = -2.5 + 3.0 * rng.uniform(0.0, 1.0, (n, 2))
    spec = O.load_spec(os.path.join(REF, 'examples/COOxVolcano/input.json'))
    SCOg, SO2g = 2.0487e-3, 2.1261e-3
    T = spec['system']['T']
    s = build_reference_system(spec, 'classic')
    s.params['ode_solver'] = 'ode'
    s.params['nsteps'] = int(1e4)

    def set_point(ECO, EO):
        s.reactions['CO_ads'].dErxn_user = ECO
        s.reactions['CO_ads'].dGrxn_user = ECO + SCOg * T
        s.reactions['2O_ads'].dErxn_user = 2.0 * EO
        s.reactions['2O_ads'].dGrxn_user = 2.0 * EO + SO2g * T
        spec['reactions']['CO_ads']['user'].update(dErxn_user=ECO, dGrxn_user=ECO + SCOg * T)
        spec['reactions']['2O_ads']['user'].update(dErxn_user=2.0 * EO, dGrxn_user=2.0 * EO + SO2g * T)
        th = O.Thermo(spec, T, spec['system']['p'])
        EO2 = th.elec('sO2')
        s.reactions['O2_ads'].dErxn_user = EO2
        s.reactions['O2_ads'].dGrxn_user = EO2 + SO2g * T
        s.reactions['CO_ox'].dEa_fwd_user = np.max((th.elec('SRTS_ox') - (ECO + EO), 0.0))
        s.reactions['O2_2O'].dEa_fwd_user = np.max((th.elec('SRTS_O2') - EO2, 0.0))

    out = {'points': n, 'threads': 1}
    for key, ss in (('reference_activity_transient', False), ('reference_activity_ss_solve', True)):
        t = time.time()
        for ECO, EO in pts:
            set_point(ECO, EO)
            s.activity(tof_terms=['CO_ox'], ss_solve=ss)
        out[key] = n / (time.time() - t)
    spec0 = O.load_spec(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    t = time.time()
    for ECO, EO in pts:
        O.volcano_point(spec0, ECO, EO, steady=True, rtol=1e-8, atol=1e-10, method='LSODA')
    out['port_cpu_baseline'] = n / (time.time() - t)
    out['unit'] = 'solves/s on one core'
    # the volcano driver's call is the transient one; ss_solve=True calls only
    # find_steady, whose guess is the PREVIOUS point's stored solution
    # (old_system.py:392-397), so it skips the transient and is not the workload
    out['port_over_reference_driver'] = out['port_cpu_baseline'] / out['reference_activity_transient']
    os.makedirs(os.path.join(ROOT, 'profiles', 'r3'), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, 'profiles', 'r3', 'cpu_reference_vs_port.json'), 'w'), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
