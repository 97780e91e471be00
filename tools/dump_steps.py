"""Dump the integrator step count of every condition of the bench's volcano
grid, in the order the conditions sit in HBM (the 16x4 patch order by
default), to gpurun_out/<out>.npy -- input of tools/sched_sim.py (wave
scheduling / tail analysis).  usage: python tools/dump_steps.py OUT [bench args]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse
    import ctypes as C
    import torch
    import bench
    out = sys.argv[1]
    ap = argparse.ArgumentParser()

    ap.add_argument('--grid', type=int, default=1024)
    ap.add_argument('--tile', default='16x4')
    ap.add_argument('--order', default='tile')
    ap.add_argument('--scaling', default='strong')
    ap.add_argument('--max-steps', type=int, default=200000)
    ap.add_argument('--no-newton', action='store_true')
    ap.add_argument('--runtime-plan', action='store_true')
    ap.add_argument('--no-retry', action='store_true')
    a = ap.parse_args(sys.argv[2:])
    torch.cuda.set_device(0)
    wl = bench.volcano_workload(a, 0, 1)
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    wl.step(sp)
    torch.cuda.synchronize()
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    np.save(os.path.join(ROOT, 'gpurun_out', out + '.npy'), wl.nsteps().cpu().numpy())
    np.save(os.path.join(ROOT, 'gpurun_out', out + '_status.npy'), wl.status().cpu().numpy())
    np.save(os.path.join(ROOT, 'gpurun_out', out + '_perm.npy'), wl.perm if wl.perm is not None else np.arange(wl.n_local))
    print('saved', out, int(wl.nsteps().sum()))


if __name__ == '__main__':
    main()
