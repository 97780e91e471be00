"""bench.py's multi-GPU plumbing on CPU (no GPU, no HIP library): `--gpus N`
spawns N rank processes before anything touches a device, the ranks shard the
volcano grid (strong: the fixed G x G grid; weak: an (N*G) x G grid), the
status counts are all-reduced, the result map is gathered and reassembled,
and rank 0 prints exactly one JSON line with n_gpus = N (gloo backend)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_PORT')}
    env['OMP_NUM_THREADS'] = '1'
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--device', 'cpu-standin'] + args,
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize('scaling, grid', [('strong', [32, 32]), ('weak', [64, 32])])
def test_launcher_world2(scaling, grid):
    line = _run(['--gpus', '2', '--steps', '2', '--warmup', '1', '--grid', '32', '--scaling', scaling])
    assert line['n_gpus'] == 2
    assert line['scaling'] == scaling
    assert line['config']['global_grid'] == grid
    assert line['config']['grid_per_gpu'] == [grid[0] // 2, 32]
    # every rank's statuses are counted once (the stand-in marks every 7th local unit 'degenerate')
    st = line['status']
    assert st['units'] == grid[0] * grid[1]
    local = grid[0] * 32 // 2
    exp_degen = sum(sum(1 for i in range(local) if (i + r) % 7 == 0) for r in range(2))
    assert st['degenerate_root_tight_transient'] == exp_degen
    assert st['regular_root'] + st['degenerate_root_tight_transient'] + st['failed'] == st['units']
    assert line['value'] > 0


def test_default_multi_gpu_layout_is_strong():
    """Without --scaling, the N ranks shard one fixed G x G grid: BASELINE
    configs[2]'s 1024 x 1024 grid sharded over the GPUs of the node."""
    line = _run(['--gpus', '2', '--steps', '1', '--warmup', '0', '--grid', '16'])
    assert line['scaling'] == 'strong'
    assert line['config']['global_grid'] == [16, 16] and line['config']['grid_per_gpu'] == [8, 16]


def test_launcher_single_rank():
    line = _run(['--steps', '1', '--warmup', '0', '--grid', '16'])
    assert line['n_gpus'] == 1 and line['config']['global_grid'] == [16, 16]


def test_strong_needs_divisible_rows():
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK')}
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--device', 'cpu-standin', '--gpus', '3',
                        '--steps', '1', '--warmup', '0', '--grid', '16', '--scaling', 'strong'], capture_output=True, text=True,
                       timeout=240, env=env, cwd=ROOT)
    assert p.returncode != 0


def test_emulate_rejected_with_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK')}
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--device', 'cpu-standin', '--gpus', '2',
                        '--emulate', '0/8'], capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0


def test_flop_count_is_structural():
    """bench.flops_per_step counts structural non-zeros: the volcano plan's
    count is below the dense count of the same step."""
    sys.path.insert(0, ROOT)
    import bench
    import pycatkin_amd as P
    from pycatkin_amd.functions.volcano import set_volcano_energies
    s = P.read_from_input_file(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    set_volcano_energies(s)
    plan = s.plan(('CO_ox',))
    f = bench.flops_per_step(plan)
    NS = len(plan.dyn)
    dense_lu = (2 * NS ** 3) // 3
    assert 400 < f < 1000, f
    assert f > dense_lu + 6 * 2 * NS * NS - 6 * NS   # at least the LU and the solves
