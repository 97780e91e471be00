"""Physical constants -- the set pycatkin/constants/physical_constants.py:10-27
uses (the "Butadiene paper" values), so every result is computed with the
reference's numbers."""
NA = 6.02214076e23
bartoPa = 1.0e5
atmtoPa = 1.01325e5
kB = 1.380662e-23       # J/K
h = 6.626176e-34        # J s
JtoeV = 6.242e18
eVtokJ = 96.485
eVtokcal = 23.06
kcaltoJ = 4184
amutokg = 1.66053886e-27
amuA2tokgm2 = 1.66053907e-47
R = 8.31446262          # J/(K mol)
