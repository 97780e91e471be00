"""Oracle fixture of BASELINE configs[3]: the DMTM degree of rate control over
temperatures AND pressures, as run_parameters(sim, [1e4, 1e5, 1e6],
'pressure', tof_terms=['r5', 'r9']) computes it at each temperature
(pycatkin/functions/presets.py:170-201 -> old_system.py:490-515).

For every (T, p) the oracle (oracle/mk_oracle.py, the reference algorithm
restated) stores, with eps = 5e-2 and TOF = r5 + r9:

  drc_steady     degree_of_rate_control(ss_solve=True): each of the 2R+1
                 perturbed systems integrated then polished to its root
  drc_input      degree_of_rate_control(ss_solve=False) at the input's
                 tolerances (rtol 1e-6 / atol 1e-8, t_end 1e12 s): the
                 reference's run_parameters path
  drc_tight      the same transient DRC at rtol 1e-10 / atol 1e-16
  tof0_*         the unperturbed TOF of each

    OMP_NUM_THREADS=1 python tests/golden/make_dmtm_drc_fixture.py

writes tests/golden/dmtm_drc_fixture.json.
"""
import json
import multiprocessing as mp
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
INPUT = os.path.join(HERE, 'inputs', 'DMTM', 'input.json')
OUT = os.path.join(HERE, 'dmtm_drc_fixture.json')
TEMPERATURES = (450.0, 600.0, 750.0)
PRESSURES = (1.0e4, 1.0e5, 1.0e6)
EPS = 5.0e-2
TOF_TERMS = ['r5', 'r9']


def _cond(tp):
    sys.path.insert(0, ROOT)
    from oracle import mk_oracle as O
    T, p = tp
    spec = O.load_spec(INPUT)
    out = dict(T=T, p=p)
    m = O.ClassicModel(spec, T=T, p=p)
    out['drc_steady'] = m.drc(TOF_TERMS, eps=EPS, steady=True)
    m = O.ClassicModel(spec, T=T, p=p)
    out['drc_input'] = m.drc(TOF_TERMS, eps=EPS, steady=False)

    class Tight(O.ClassicModel):
        def solve_odes(self, t_end=None, rtol=None, atol=None, y0=None, method='BDF'):
            return super().solve_odes(t_end=t_end, rtol=1e-10, atol=1e-16, y0=y0, method=method)
    m = Tight(spec, T=T, p=p)
    out['drc_tight'] = m.drc(TOF_TERMS, eps=EPS, steady=False)
    for key, steady, cls in (('tof0_steady', True, O.ClassicModel), ('tof0_input', False, O.ClassicModel),
                             ('tof0_tight', False, Tight)):
        mm = cls(spec, T=T, p=p)
        if steady:
            y, _ = mm.solve_odes(rtol=1e-6, atol=1e-12)
            y = mm.find_steady(y)
        else:
            y, _ = mm.solve_odes()
        out[key] = mm.tof(y, TOF_TERMS)
    return out


def main():
    conds = [(T, p) for T in TEMPERATURES for p in PRESSURES]
    with mp.get_context('fork').Pool(min(8, len(conds))) as pool:
        res = pool.map(_cond, conds)
    json.dump(dict(eps=EPS, tof_terms=TOF_TERMS, temperatures=list(TEMPERATURES), pressures=list(PRESSURES),
                   conditions=res), open(OUT, 'w'), indent=1)
    print('wrote', OUT)


if __name__ == '__main__':
    main()
