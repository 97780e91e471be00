"""Evaluate preview-solve predictors of the volcano wavefront cost
(tools/predictor_probe.py output) with the wave-scheduling model of
tools/sched_sim.py: the makespan of the launch when the wavefronts are
dispatched in descending predicted cost, against the as-launched order and
the oracle longest-first order.

    python tools/predictor_eval.py gpurun_out/predictor_probe.npz [CAP]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sched_sim import makespan  # noqa: E402


def main():
    d = dict(np.load(sys.argv[1]))
    cap = float(sys.argv[2]) if len(sys.argv) > 2 else 1.6
    cost = d['r8'].astype(np.float64).reshape(-1, 64).max(axis=1)     # the bench pass
    base = makespan(cost, cap)
    best = makespan(np.sort(cost)[::-1], cap)
    print('as launched %.0f   oracle longest-first %.0f (speedup %.3f)' % (base, best, base / best))
    for key in sorted(k for k in d if k.startswith('r') and k != 'r8'):
        pred = d[key].astype(np.float64)
        if pred.size == cost.size * 64:
            pred = pred.reshape(-1, 64).max(axis=1)
        order = np.argsort(-pred, kind='stable')
        m = makespan(cost[order], cap)
        rho = np.corrcoef(np.argsort(np.argsort(pred)), np.argsort(np.argsort(cost)))[0, 1]
        print('%-10s rank corr %.3f  makespan %.0f  speedup %.3f' % (key, rho, m, base / m))


if __name__ == '__main__':
    main()


def subsets(path, cap=1.6):
    """Predictors from a subset of each patch's lanes of the loose full-grid
    preview: what a preview launch over those lanes only would see."""
    d = dict(np.load(path))
    cost = d['r8'].astype(np.float64).reshape(-1, 64).max(axis=1)
    base = makespan(cost, cap)
    for key in ('r3', 'r4', 'r6'):
        w = d[key].astype(np.float64).reshape(-1, 64)
        for name, lanes in (('4 corners', [0, 3, 60, 63]), ('every 16th', list(range(0, 64, 16))),
                            ('every 8th', list(range(0, 64, 8))), ('every 4th', list(range(0, 64, 4))),
                            ('every 2nd', list(range(0, 64, 2)))):
            pred = w[:, lanes].max(axis=1)
            m = makespan(cost[np.argsort(-pred, kind='stable')], cap)
            print('%s %-11s (%2d lanes) speedup %.3f' % (key, name, len(lanes), base / m))
