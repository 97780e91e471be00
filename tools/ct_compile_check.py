"""Offline build of the lane-group solver with a compile-time network
(mk_group.h: ct_rhs / ct_jac; the hipRTC kernel csrc/mk_jit.h:
jit_group_ct_kernel compiles at the first solve) for the shipped group
networks: hipcc --offload-arch=gfx950 on this container, reporting each
kernel's VGPRs, spills, occupancy and code size from the compiler's
resource-usage remarks.  No GPU needed.

    python tools/ct_compile_check.py [ch4|dmtm|synthetic ...] [--tables] [-DNAME=VALUE ...] [--llvm=OPT ...]

--tables builds the record-table kernel of the same exact size instead,
--quad the quad-group kernel (mk_quad.h);
-D options go to hipcc (e.g. -DPCK_GRP_WAVES16=3, -DPCK_CT_CHUNK=2);
--asm=PATH also writes the assembly (%s in PATH = the network's name).
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
INPUTS = os.path.join(ROOT, 'tests', 'golden', 'inputs')
TABLES = False
ASM = None


def plan_of(name):
    import pycatkin_amd as P
    if name == 'ch4':
        s = P.read_from_input_file(os.path.join(INPUTS, 'CH4', 'input.json'), formulation='patched')
        for r, st in (('C_ads', 'sC'), ('O_ads', 'sO')):
            s.reactions[r].dErxn_user = 1.0
            s.states[st].Gelec = 1.0
        return s.plan()
    if name == 'dmtm':
        return P.read_from_input_file(os.path.join(INPUTS, 'DMTM', 'input.json')).plan(('r5', 'r9'))
    if name == 'synthetic':
        from pycatkin_amd.functions.synthetic import synthetic_system
        return synthetic_system()[0].plan(('R0',))
    raise KeyError(name)


def main():
    from gen_networks import emit
    global TABLES
    TABLES = '--tables' in sys.argv
    quad = '--quad' in sys.argv            # the quad-group kernel (mk_quad.h)
    global ASM
    ASM = next((a[len('--asm='):] for a in sys.argv[1:] if a.startswith('--asm=')), None)
    defs = [a for a in sys.argv[1:] if a.startswith('-D')]
    for a in sys.argv[1:]:                  # --llvm=OPT -> -mllvm OPT
        if a.startswith('--llvm='):
            defs += ['-mllvm', a[len('--llvm='):]]
    names = [a for a in sys.argv[1:] if not a.startswith('-')] or ['dmtm', 'ch4', 'synthetic']
    for name in names:
        plan = plan_of(name)
        NS = len(plan.dyn)
        G = 16 if NS <= 16 else 32 if NS <= 32 else 64
        src = ('#define PCK_GRP_EXACT 1\n#ifndef PCK_CHK_P\n#define PCK_CHK_P 1\n#endif\n#define PCK_GRP_BAL 0\n#include "mk_solver.h"\nnamespace pck {\nnamespace nets {\n'
               + emit('Jit', plan) + '\n}\n}\n#include "mk_group.h"\n'
               'template __global__ void pck::k_solve_grp<%d, %d, PCK_CHK_P, false, false, %s>('
               'pck::NetView, pck::GrpView, pck::CondView, const double*, const double*, int64_t, pck::SolveArgs, '
               'pck::GrpArgs);\n' % (NS, G, 'pck::NoNet' if TABLES else 'pck::nets::Jit'))
        if quad:
            src = ('#define PCK_GRP_EXACT 1\n#define PCK_GRP_BAL 0\n#include "mk_solver.h"\nnamespace pck {\nnamespace nets {\n'
                   + emit('Jit', plan) + '\n}\n}\n#include "mk_quad.h"\n'
                   'template __global__ void pck::k_solve_q4<pck::nets::Jit, %s, %s>(pck::NetView, pck::CondView, '
                   'const double*, const double*, int64_t, pck::SolveArgs, pck::GrpArgs);\n'
                   % ('true' if '--newton' in sys.argv else 'false', 'true' if '--traj' in sys.argv else 'false'))
        kname = 'k_solve_q4' if quad else 'k_solve_grp'
        with tempfile.TemporaryDirectory() as d:
            f = os.path.join(d, 'ct_%s.hip' % name)
            open(f, 'w').write(src)
            cmd = ['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fno-signed-zeros',
                   '--cuda-device-only', '-c', '-I' + os.path.join(ROOT, 'include'),
                   '-I' + os.path.join(ROOT, 'pycatkin_amd', 'csrc'), '-Rpass-analysis=kernel-resource-usage',
                   *defs, '-o', os.path.join(d, 'k.o'), f]
            p = subprocess.run(cmd, capture_output=True, text=True)
            if ASM:                          # --asm=PATH: the kernel's assembly too
                subprocess.run([c for c in cmd if c not in ('-c', '-Rpass-analysis=kernel-resource-usage')][:-3]
                               + ['-S', '-o', ASM.replace('%s', name), f], capture_output=True, text=True)
            if p.returncode:
                print(name, 'FAILED'); print(p.stderr[-4000:]); continue
            lines = p.stderr.splitlines()
            # the remarks of the solver kernel (the header's k_drc_combine comes first)
            start = max(i for i, l in enumerate(lines) if 'Function Name' in l and kname in l)
            keep = [l.split('remark: ')[-1].split(' [-R')[0].strip() for l in lines[start:]
                    if re.search(r'(VGPRs:|AGPRs:|Spill|Occupancy|ScratchSize)', l)]
            sym = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-readelf', '-s', '-W', os.path.join(d, 'k.o')],
                                 capture_output=True, text=True).stdout
            size = [int(l.split()[2]) for l in sym.splitlines() if kname in l and 'FUNC' in l]
            print('%s%s (NS=%d, R=%d, G=%d): %s; code %s bytes' % (name, ' [tables]' if TABLES else '', NS,
                                                                  len(plan.reactions), G, '; '.join(keep), size))


if __name__ == '__main__':
    main()
