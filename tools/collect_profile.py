"""Copy a tools/profile.sh run (gpurun_out/<run>) into profiles/<dest> under
the names tools/pmc_summary.py reads (kernel_stats.csv, pmc_<pass>_counters.csv,
the trace's kernel_trace.csv) and write its summary.json.

    python tools/collect_profile.py gpurun_out/r3k/volcano profiles/r3/volcano \
        --tag 'k_solve<pck::PlanCT<pck::nets::Volcano>' 'volcano 1024x1024 tile'
"""
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    for f in ('run_kernel_stats.csv', 'run_kernel_trace.csv'):
        p = os.path.join(src, 'trace', f)
        if os.path.isfile(p):
            shutil.copy(p, os.path.join(dst, f.replace('run_', '')))
    for d in sorted(glob.glob(os.path.join(src, 'pmc_*'))):
        if not os.path.isdir(d):
            continue
        p = os.path.join(d, 'run_counter_collection.csv')
        if os.path.isfile(p):
            shutil.copy(p, os.path.join(dst, os.path.basename(d) + '_counters.csv'))
    if os.path.isfile(os.path.join(src, 'summary.txt')):
        shutil.copy(os.path.join(src, 'summary.txt'), os.path.join(dst, 'passes.txt'))
    subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'pmc_summary.py'), dst] + sys.argv[3:], check=True)


if __name__ == '__main__':
    main()
