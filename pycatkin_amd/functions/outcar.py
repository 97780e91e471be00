"""Minimal VASP OUTCAR / ASE log.vib readers (state.py:266-400 read these
through `ase`, which this image does not ship)."""
from __future__ import annotations

import os


def read_frequencies(base):
    """state.py:318-371: frequencies (Hz) from <base>/log.vib or <base>/OUTCAR."""
    from ..constants.physical_constants import JtoeV, h
    logvib = os.path.join(base, 'log.vib')
    if os.path.isfile(logvib):
        with open(logvib) as fh:
            lines = fh.readlines()
        initat = endat = 0
        for lind, line in enumerate(lines):
            if '#' in line:
                initat, endat = lind + 2, 0
            if lind > initat and not endat and '---' in line:
                endat = lind - 1
        rows = lines[initat:endat + 1]
        freq = [float(l.strip().split()[1]) * 1e-3 / (h * JtoeV) for l in rows if 'i' not in l]
        ifreq = [float(l.strip().split()[1].split('i')[0]) * 1e-3 / (h * JtoeV) for l in rows if 'i' in l]
        return freq, ifreq
    path = os.path.join(base, 'OUTCAR') if os.path.isdir(base) else base
    freq, ifreq, first = [], [], 0
    with open(path) as fh:
        for line in fh:
            data = line.split()
            if 'THz' in data:
                if first + 1 == int(data[0]):
                    fHz = float(data[-8]) * 1.0e12
                    (ifreq if ('f/i=' in data or 'f/i' in data) else freq).append(fHz)
                    first = int(data[0])
                else:
                    break
    return freq, ifreq


def read_outcar(path):
    raise NotImplementedError('OUTCAR geometry/energy reading (ase.io.read vasp-out) is not implemented yet; '
                              'give mass / inertia / Gelec in the input file')
