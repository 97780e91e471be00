"""Wave-scheduling model of the volcano launch (tools/dump_steps.py output):
waves of 64 consecutive conditions cost max(steps) of their lanes; waves are
dispatched in launch order to the first free slot (SIMDS x WAVES slots); a
SIMD with k resident waves advances each at speed min(1, CAP / k) (CAP =
waves' worth of issue the SIMD sustains).  Prints the makespan of several
orders relative to the as-launched order.

usage: python tools/sched_sim.py gpurun_out/steps_tile.npy [CAP]"""
import heapq
import sys

import numpy as np

SIMDS, WAVES = 1024, 3


def makespan(cost, cap):
    """processor-sharing event simulation per SIMD; dispatch in order to the
    SIMD with the fewest resident waves (ties: lowest index)."""
    n = len(cost)
    nxt = 0
    # per SIMD: list of remaining work of resident waves
    res = [[] for _ in range(SIMDS)]
    t = 0.0
    # fill
    for w in range(WAVES):
        for s in range(SIMDS):
            if nxt < n:
                res[s].append(float(cost[nxt]))
                nxt += 1
    # event loop: advance to the next completion anywhere
    while True:
        best = None
        for s in range(SIMDS):
            k = len(res[s])
            if k:
                sp = min(1.0, cap / k)
                dt = min(res[s]) / sp
                if best is None or dt < best[0]:
                    best = (dt, s)
        if best is None:
            return t
        dt = best[0]
        t += dt
        for s in range(SIMDS):
            k = len(res[s])
            if k:
                sp = min(1.0, cap / k)
                r = [x - dt * sp for x in res[s]]
                res[s] = [x for x in r if x > 1e-9]
                while len(res[s]) < WAVES and nxt < n and len(res[s]) < k:
                    res[s].append(float(cost[nxt]))
                    nxt += 1
        # refill every SIMD that has room
        for s in range(SIMDS):
            while len(res[s]) < WAVES and nxt < n:
                res[s].append(float(cost[nxt]))
                nxt += 1


def main():
    steps = np.load(sys.argv[1]).astype(np.float64)
    cap = float(sys.argv[2]) if len(sys.argv) > 2 else 1.6
    pad = (-len(steps)) % 64
    w = np.pad(steps, (0, pad)).reshape(-1, 64)
    cost = w.max(axis=1)
    lane_eff = steps.sum() / (cost.sum() * 64)
    ideal = cost.sum() / (SIMDS * cap)
    print('waves %d  mean wave cost %.1f  max %.0f  lane_eff %.4f' % (len(cost), cost.mean(), cost.max(), lane_eff))
    base = makespan(cost, cap)
    print('as launched   %.0f  (ideal %.0f, ratio %.3f)' % (base, ideal, base / ideal))
    srt = np.sort(cost)[::-1]
    m = makespan(srt, cap)
    print('LPT (desc)    %.0f  speedup %.3f' % (m, base / m))
    srt_steps = np.sort(steps)[::-1]
    c2 = np.pad(srt_steps, (0, pad)).reshape(-1, 64).max(axis=1)
    m2 = makespan(c2, cap)
    print('lane-sorted   %.0f  speedup %.3f  (lane_eff %.4f)' % (m2, base / m2, steps.sum() / (c2.sum() * 64)))



def two_phase(steps, cap, s1, sort2=False):
    """phase 1: every lane runs at most s1 steps; phase 2: the unfinished
    lanes, compacted (launch order, or sorted by remaining steps), run the
    rest.  Returns (makespan1, makespan2, unfinished lanes)."""
    pad = (-len(steps)) % 64
    c1 = np.minimum(np.pad(steps, (0, pad)).reshape(-1, 64).max(axis=1), s1)
    rem = steps[steps > s1] - s1
    if sort2:
        rem = np.sort(rem)[::-1]
    pad2 = (-len(rem)) % 64
    c2 = np.pad(rem, (0, pad2)).reshape(-1, 64).max(axis=1) if len(rem) else np.zeros(0)
    return makespan(c1, cap), (makespan(c2, cap) if len(c2) else 0.0), len(rem)


if __name__ == '__main__' and len(sys.argv) > 3:
    steps = np.load(sys.argv[1]).astype(np.float64)
    cap = float(sys.argv[2])
    base = makespan(np.pad(steps, (0, (-len(steps)) % 64)).reshape(-1, 64).max(axis=1), cap)
    for s1 in [int(x) for x in sys.argv[3].split(',')]:
        for srt in (False, True):
            a, b, k = two_phase(steps, cap, s1, srt)
            print('s1 %4d sort2 %d: phase1 %.0f phase2 %.0f (%d lanes) total %.0f speedup %.3f'
                  % (s1, srt, a, b, k, a + b, base / (a + b)))


if __name__ == '__main__' and len(sys.argv) <= 3:
    main()
