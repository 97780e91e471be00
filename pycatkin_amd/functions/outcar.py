"""Minimal VASP OUTCAR / ASE log.vib readers (state.py:77-211 read these
through `ase`, which this image does not ship)."""
from __future__ import annotations

import os

import numpy as np


def read_frequencies(base):
    """state.py:126-182: frequencies (Hz) from <base>/log.vib or <base>/OUTCAR."""
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


# Standard atomic weights (IUPAC 2016, the table ase.data.atomic_masses holds)
# for the elements that occur in heterogeneous-catalysis inputs.
ATOMIC_MASS = {
    'H': 1.008, 'He': 4.002602, 'Li': 6.94, 'Be': 9.0121831, 'B': 10.81, 'C': 12.011, 'N': 14.007,
    'O': 15.999, 'F': 18.998403163, 'Ne': 20.1797, 'Na': 22.98976928, 'Mg': 24.305, 'Al': 26.9815385,
    'Si': 28.085, 'P': 30.973761998, 'S': 32.06, 'Cl': 35.45, 'Ar': 39.948, 'K': 39.0983, 'Ca': 40.078,
    'Sc': 44.955908, 'Ti': 47.867, 'V': 50.9415, 'Cr': 51.9961, 'Mn': 54.938044, 'Fe': 55.845,
    'Co': 58.933194, 'Ni': 58.6934, 'Cu': 63.546, 'Zn': 65.38, 'Ga': 69.723, 'Ge': 72.63, 'As': 74.921595,
    'Se': 78.971, 'Br': 79.904, 'Kr': 83.798, 'Rb': 85.4678, 'Sr': 87.62, 'Y': 88.90584, 'Zr': 91.224,
    'Nb': 92.90637, 'Mo': 95.95, 'Tc': 97.90721, 'Ru': 101.07, 'Rh': 102.9055, 'Pd': 106.42,
    'Ag': 107.8682, 'Cd': 112.414, 'In': 114.818, 'Sn': 118.71, 'Sb': 121.76, 'Te': 127.6,
    'I': 126.90447, 'Xe': 131.293, 'Cs': 132.90545196, 'Ba': 137.327, 'La': 138.90547, 'Ce': 140.116,
    'Hf': 178.49, 'Ta': 180.94788, 'W': 183.84, 'Re': 186.207, 'Os': 190.23, 'Ir': 192.217,
    'Pt': 195.084, 'Au': 196.966569, 'Hg': 200.592, 'Tl': 204.38, 'Pb': 207.2, 'Bi': 208.9804,
}


class OutcarAtoms:
    """The final ionic step of a VASP OUTCAR: element symbols, Cartesian
    positions (Angstrom) and the force-consistent energy (free energy TOTEN,
    eV) -- what state.py:92-95 and :264 take from `ase.io.read(..., 'vasp-out')`."""

    def __init__(self, symbols, positions, energy):
        self.symbols = list(symbols)
        self.positions = np.asarray(positions, dtype=float).reshape(-1, 3)
        self.energy = energy

    def get_masses(self):
        return np.array([ATOMIC_MASS[s] for s in self.symbols])

    def total_mass(self):
        return float(np.sum(self.get_masses()))

    def moments_of_inertia(self):
        """Principal moments (amu Angstrom^2, ascending) about the centre of
        mass: eigenvalues of sum_i m_i (|r_i|^2 1 - r_i r_i^T)."""
        m = self.get_masses()
        r = self.positions - (m[:, None] * self.positions).sum(0) / m.sum()
        I = np.eye(3) * float(np.sum(m * np.sum(r * r, axis=1))) - np.einsum('i,ij,ik->jk', m, r, r)
        return np.linalg.eigvalsh(I)


def _element(token):
    return token.split('_')[0].split('.')[0]


def read_outcar(path):
    """Parse <path>/OUTCAR (or the file `path`): species from the VRHFIN
    lines (one per POTCAR, in POTCAR order) times 'ions per type', positions
    from the last 'POSITION ... TOTAL-FORCE' block, energy from the last
    'free  energy   TOTEN' line."""
    f = os.path.join(path, 'OUTCAR') if os.path.isdir(path) else path
    if not os.path.isfile(f):
        raise FileNotFoundError(f)
    types, counts, positions, energy = [], None, None, None
    with open(f) as fh:
        lines = fh.readlines()
    i = 0
    while i < len(lines):
        line = lines[i]
        if 'VRHFIN' in line:
            types.append(_element(line.split('=')[1].split(':')[0].strip()))
        elif 'ions per type' in line:
            counts = [int(x) for x in line.split('=')[1].split()]
        elif 'POSITION' in line and 'TOTAL-FORCE' in line:
            block = []
            j = i + 2
            while j < len(lines) and not lines[j].strip().startswith('---'):
                block.append([float(x) for x in lines[j].split()[:3]])
                j += 1
            positions = block
            i = j
        elif 'free  energy   TOTEN' in line:
            energy = float(line.split('=')[1].split()[0])
        i += 1
    if counts is None or positions is None or len(types) < len(counts):
        raise ValueError('%s: no species / ionic positions found' % f)
    symbols = [s for s, c in zip(types, counts) for _ in range(c)]
    if len(symbols) != len(positions):
        raise ValueError('%s: %d ions per type but %d positions' % (f, len(symbols), len(positions)))
    return OutcarAtoms(symbols, positions, energy)
