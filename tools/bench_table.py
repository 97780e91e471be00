"""Summarise bench JSON lines (one per file) as a table: ms/step, value,
integrator steps, lane efficiency, statuses.  python tools/bench_table.py FILES"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        print('%-40s (no line)' % f)
        continue
    r = d.get('roofline') or {}
    s = d.get('status', {})
    print('%-40s %9.3f ms  %8.2f M/s  steps %.4g  eff %.3f  frac %.3f  reg %d deg %d loose %d fail %d %s' % (
        f, d['ms_per_step'], d['value'] / 1e6, r.get('integrator_steps', 0), r.get('lane_efficiency', 0),
        r.get('frac', 0), s.get('regular_root', 0), s.get('degenerate_root_tight_transient', 0),
        s.get('degenerate_root_input_tolerance_transient', 0), s.get('failed', 0),
        s.get('failed_by_code', '')))
