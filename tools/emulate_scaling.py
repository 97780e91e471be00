"""Predicted multi-GPU curve of the headline bench from one GPU.

The ranks of `bench.py --gpus N` share nothing in the timed region (cyclic
E_CO rows of the grid, no collective until after timing), so rank r's step
time on an 8-GPU node is the time of its shard alone on one GPU: this runs
every shard r of N = 1, 2, 4, 8 in one process (the bench's own workload
builder, HIP-event timing on the solve stream) and reports, per N, the
per-rank times, the max over ranks (the bench's step time) and the whole-node
value = units / max.  Strong scaling (default, BASELINE configs[2]: the fixed
1024 x 1024 grid) and, for N = 8, the weak layout (1024 x 1024 per rank).

    python tools/emulate_scaling.py [--steps 3] > gpurun_out/emulate_scaling.json
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def shard_ms(bench, torch, scaling, rank, world, steps, extra=()):
    args = bench.build_parser().parse_args(['--scaling', scaling] + list(extra))
    wl = bench.volcano_workload(args, rank, world)
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(3):                 # warm-up: clocks and the pool allocator settle
        wl.step(sp)
    torch.cuda.synchronize()
    ts = []
    for _ in range(steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        wl.step(sp)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    st = wl.status().cpu().numpy()
    ns = wl.nsteps().cpu().numpy().astype(np.int64)
    pad = (-ns.size) % 64
    waves = np.concatenate([ns, np.zeros(pad, ns.dtype)]).reshape(-1, 64).max(axis=1)
    return dict(rank=rank, ms=float(np.median(ts)), units=int(wl.n_local), steps_max=int(ns.max()),
                steps_mean=float(ns.mean()), lane_eff=float(ns.mean() / waves.mean()),
                wave_steps_p99=float(np.percentile(waves, 99)), degenerate=int((st == 4).sum()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--worlds', default='1,2,4,8', help="strong-scaling world sizes (',' or '+' separated)")
    ap.add_argument('--no-weak', action='store_true')
    ap.add_argument('--bench-args', default='', help="extra bench.py arguments, '+'-separated (A/B)")
    a = ap.parse_args()
    extra = [x for x in a.bench_args.split('+') if x]
    import torch
    import bench
    out = []
    plan = [('strong', tuple(int(w) for w in a.worlds.replace('+', ',').split(',')))] + ([] if a.no_weak else [('weak', (8,))])
    for scaling, worlds in plan:
        for N in worlds:
            ranks = [shard_ms(bench, torch, scaling, r, N, a.steps, extra) for r in range(N)]
            t = max(x['ms'] for x in ranks)
            units = sum(x['units'] for x in ranks)
            line = dict(scaling=scaling, n_gpus=N, bench_args=extra, rank_ms=[x['ms'] for x in ranks], max_rank_ms=t,
                        predicted_value=units / (t * 1e-3), units=units, ranks=ranks)
            print(json.dumps(line), flush=True)
            out.append(line)
    base = [x for x in out if x['scaling'] == 'strong'][0]['predicted_value']
    for x in out:
        x['predicted_speedup_vs_1'] = x['predicted_value'] / base
    print(json.dumps(dict(summary=[{k: x[k] for k in ('scaling', 'n_gpus', 'max_rank_ms', 'predicted_value',
                                                     'predicted_speedup_vs_1')} for x in out])))


if __name__ == '__main__':
    main()
