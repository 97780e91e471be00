"""Summarise a rocprofv3 profile directory (kernel_stats.csv + pmc_*_counters.csv
as copied into profiles/) into summary.json: per kernel, the average duration and
the per-launch counter averages.  HBM traffic follows MI355X_MICROARCH.md's
rocprofv3 section: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of coalesced reads, so it is doubled.

usage: python tools/pmc_summary.py profiles/r1/compiled_plan
"""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    return name.split('(')[0].replace('void ', '').strip()


def summarise(d):
    out = collections.defaultdict(dict)
    stats = os.path.join(d, 'kernel_stats.csv')
    if os.path.isfile(stats):
        for r in csv.DictReader(open(stats)):
            out[short(r['Name'])].update(calls=int(r['Calls']), avg_ns=float(r['AverageNs']))
    for f in sorted(glob.glob(os.path.join(d, 'pmc_*_counters.csv'))):
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            acc[short(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
        for k, cs in acc.items():
            for c, v in cs.items():
                out[k][c] = sum(v) / len(v)
    for k, v in out.items():
        if 'FETCH_SIZE' in v or 'WRITE_SIZE' in v:
            v['fetch_bytes'] = 2.0 * 1024.0 * v.get('FETCH_SIZE', 0.0)
            v['write_bytes'] = 1024.0 * v.get('WRITE_SIZE', 0.0)
            v['traffic_bytes'] = v['fetch_bytes'] + v['write_bytes']
        if 'SQ_INSTS_VALU_FMA_F64' in v:
            # fp64 FLOPs from the instruction counters (per wave instruction: 64
            # lanes, FMA = 2): an upper bound, exec-masked lanes count as active
            f64 = v.get('SQ_INSTS_VALU_ADD_F64', 0.0) + v.get('SQ_INSTS_VALU_MUL_F64', 0.0) + \
                v['SQ_INSTS_VALU_FMA_F64'] + v.get('SQ_INSTS_VALU_TRANS_F64', 0.0)
            v['f64_wave_insts'] = f64
            v['f64_flops_counted'] = 64.0 * (v.get('SQ_INSTS_VALU_ADD_F64', 0.0) + v.get('SQ_INSTS_VALU_MUL_F64', 0.0) +
                                             v.get('SQ_INSTS_VALU_TRANS_F64', 0.0) + 2.0 * v['SQ_INSTS_VALU_FMA_F64'])
            if v.get('SQ_INSTS_VALU'):
                v['f64_share_of_valu'] = f64 / v['SQ_INSTS_VALU']
    return dict(out)


if __name__ == '__main__':
    # python tools/pmc_summary.py DIR [--tag KERNEL_SUBSTRING TAG]: the tag names
    # the bench workload the profile is of (bench.py: profiled_counters)
    d = sys.argv[1]
    s = summarise(d)
    if '--tag' in sys.argv:
        i = sys.argv.index('--tag')
        sub, tag = sys.argv[i + 1], sys.argv[i + 2]
        for k, v in s.items():
            if sub in k:
                v['tag'] = tag
    with open(os.path.join(d, 'summary.json'), 'w') as fh:
        json.dump(s, fh, indent=1, sort_keys=True)
    for k, v in s.items():
        print(k, {a: b for a, b in v.items() if a in ('avg_ns', 'traffic_bytes', 'SQ_INSTS_VALU')})
