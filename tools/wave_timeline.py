"""Diagnostic (GPU): the wave timeline of the headline bench's main lane-solver
launch, from the PCK_WAVE_TIMES build (mk_solver.h; built by hand:
hipcc ... -DPCK_WAVE_TIMES=1 -o pycatkin_amd/_diag/lib_wt.so csrc/mk_kernels.hip).

    python tools/wave_timeline.py --lib pycatkin_amd/_diag/lib_wt.so [OUT.json] [bench args ...]

Every block (one wavefront) of the launch records its start / end on the
real-time clock (100 MHz) and its hardware slot.  Reported: the launch span,
the active-wave count over time (in 20 bins), when the last 1 / 5 / 10 % of
the waves end, the per-wave durations against the wave's largest step count
(the cost the dispatch order predicts), and where the costliest waves sat in
the dispatch order.
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
RT_HZ = 100e6          # s_memrealtime: the constant 100 MHz clock


def main():
    args = sys.argv[1:]
    if '--lib' in args:
        i = args.index('--lib')
        os.environ['PCK_LIB'] = os.path.abspath(args[i + 1])
        del args[i:i + 2]
    out_path = args.pop(0) if args and args[0].endswith('.json') else None
    import torch
    import bench
    from pycatkin_amd import _lib as L
    lib = L.load()
    lib.pck_wtimes_get.argtypes = [C.c_void_p, C.c_int]
    a = bench.build_parser().parse_args(args)
    wl = bench.volcano_workload(a, 0, 1)
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(4):
        wl.step(sp)
    torch.cuda.synchronize()
    wl.step(sp)
    torch.cuda.synchronize()
    n = wl.n_local
    W = (n + 63) // 64
    wt = np.zeros(3 * W, dtype=np.int64)
    L.check(lib.pck_wtimes_get(wt.ctypes.data_as(C.c_void_p), W))
    wt = wt.reshape(W, 3)
    t0 = wt[:, 0].min()
    start = (wt[:, 0] - t0) / RT_HZ * 1e3        # ms
    end = (wt[:, 1] - t0) / RT_HZ * 1e3
    dur = end - start
    wsteps = wt[:, 2] & 0xffffffff                # the block's largest step count
    hw = (wt[:, 2] >> 32) & 0xffffffff
    span = end.max()
    bins = np.linspace(0.0, span, 21)
    active = [int(np.sum((start < b1) & (end > b0))) for b0, b1 in zip(bins[:-1], bins[1:])]
    q = np.sort(end)
    res = dict(bench_args=args, waves=int(W), span_ms=float(span), first_end_ms=float(q[0]),
               end_p50_ms=float(np.percentile(end, 50)), end_p90_ms=float(np.percentile(end, 90)),
               end_p95_ms=float(np.percentile(end, 95)), end_p99_ms=float(np.percentile(end, 99)),
               last_start_ms=float(start.max()), dur_max_ms=float(dur.max()), dur_mean_ms=float(dur.mean()),
               dur_p99_ms=float(np.percentile(dur, 99)),
               active_waves_per_bin=active, bin_ms=float(bins[1] - bins[0]),
               slowest_blocks=[dict(block=int(b), start_ms=float(start[b]), end_ms=float(end[b]),
                                    hw_id=hex(int(hw[b])), steps=int(wsteps[b])) for b in np.argsort(-end)[:10]],
               wave_steps_max=int(wsteps.max()), wave_steps_mean=float(wsteps.mean()),
               wave_steps_p99=float(np.percentile(wsteps, 99)))
    # how long does a wave of s steps take, by the time it started
    order = np.argsort(start)
    thirds = np.array_split(order, 3)
    res['dur_mean_by_start_third_ms'] = [float(dur[t].mean()) for t in thirds]
    res['steps_mean_by_start_third'] = [float(wsteps[t].mean()) for t in thirds]
    # time per step of a wave against when it ran
    per = dur / np.maximum(wsteps, 1)
    res['us_per_step_by_start_third'] = [float(1e3 * np.median(per[t])) for t in thirds]
    heavy = np.argsort(-wsteps)[:max(1, W // 100)]
    res['heaviest_1pct'] = dict(steps_min=int(wsteps[heavy].min()), start_ms_max=float(start[heavy].max()),
                                end_ms_max=float(end[heavy].max()), us_per_step_median=float(1e3 * np.median(per[heavy])))
    print(json.dumps(res, indent=1))
    if out_path:
        json.dump(res, open(out_path, 'w'), indent=1)


if __name__ == '__main__':
    main()
