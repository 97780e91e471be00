"""Symbolic energies: the host half of kernel (1).

The reference evaluates free energies and reaction energies one condition at a
time in Python floats (pycatkin/classes/state.py:247-386,
pycatkin/classes/reaction.py:43-69/222-274).  Here the same formulas are run
ONCE per network with `LinearForm`s instead of floats.  Every energy in the
reference is affine in a small feature vector

    phi(c) = [1, T, descriptors..., vib_s(T), tran_s(T, p), rot_s(T) per state,
              clamp registers...]

so the result is a tiny straight-line "energy program" that the device
evaluates per condition (pycatkin_amd/csrc/mk_device.h: thermo_features).
"""
from __future__ import annotations

import itertools
import numbers

__all__ = ['LinearForm', 'Descriptor', 'TSYM', 'PSYM', 'clamp0', 'as_form', 'tkeyed', 'TKEYED']

_clamp_ids = itertools.count()


class LinearForm:
    """sum_k coef_k * feature_k with features keyed by tuples:
    ('1',) ('T',) ('desc', name) ('vib'|'tran'|'rot', state_name) ('clamp', id)."""

    __slots__ = ('terms', 'clamps', 'refs')

    def __init__(self, terms=None, clamps=None, refs=None):
        self.terms = dict(terms or {})
        self.clamps = dict(clamps or {})     # id -> LinearForm (inner of max(inner, 0))
        self.refs = dict(refs or {})         # state name -> State object of a thermal feature

    # -- algebra -------------------------------------------------------------
    def _merge(self, other, sign):
        other = as_form(other)
        t = dict(self.terms)
        for k, v in other.terms.items():
            t[k] = t.get(k, 0.0) + sign * v
        c = dict(self.clamps)
        c.update(other.clamps)
        r = dict(self.refs)
        for name, st in other.refs.items():
            if r.setdefault(name, st) is not st:
                raise ValueError('energy terms of two different states named %r meet in one expression; '
                                 'state names must be unique within a network' % name)
        return LinearForm(t, c, r)

    def __add__(self, o):
        return self._merge(o, 1.0)

    __radd__ = __add__

    def __sub__(self, o):
        return self._merge(o, -1.0)

    def __rsub__(self, o):
        return as_form(o)._merge(self, -1.0)

    def __neg__(self):
        return LinearForm({k: -v for k, v in self.terms.items()}, self.clamps, self.refs)

    def __mul__(self, s):
        if isinstance(s, LinearForm):
            if s.is_constant():
                s = s.constant()
            elif self.is_constant():
                return s * self.constant()
            else:
                raise TypeError('energies are affine in the features; cannot multiply two non-constant forms')
        if not isinstance(s, numbers.Real):
            raise TypeError('LinearForm * %r' % type(s))
        return LinearForm({k: v * float(s) for k, v in self.terms.items()}, self.clamps, self.refs)

    __rmul__ = __mul__

    def __truediv__(self, s):
        if isinstance(s, LinearForm):
            if not s.is_constant():
                raise TypeError('cannot divide by a non-constant form')
            s = s.constant()
        return self * (1.0 / float(s))

    # -- queries -------------------------------------------------------------
    def is_constant(self):
        return all(k == ('1',) or v == 0.0 for k, v in self.terms.items())

    def constant(self):
        return self.terms.get(('1',), 0.0)

    def __float__(self):
        if not self.is_constant():
            raise TypeError('form depends on %s; evaluate it on the device' %
                            sorted(k for k, v in self.terms.items() if k != ('1',) and v != 0.0))
        return float(self.constant())

    def __repr__(self):
        return 'LinearForm(%s)' % ' + '.join('%g*%s' % (v, ':'.join(map(str, k))) for k, v in self.terms.items())

    # Python's max((x, 0.0)) in a driver works on constants; use clamp0 otherwise
    def __gt__(self, o):
        return float(self) > float(as_form(o))

    def __lt__(self, o):
        return float(self) < float(as_form(o))

    def __ge__(self, o):
        return float(self) >= float(as_form(o))

    def __le__(self, o):
        return float(self) <= float(as_form(o))


def as_form(x):
    if isinstance(x, LinearForm):
        return x
    if x is None:
        return None
    return LinearForm({('1',): float(x)})


def Descriptor(name):
    """A per-condition input (eV), e.g. the CO / O binding energies of a volcano."""
    return LinearForm({('desc', str(name)): 1.0})


TKEYED = {}
"""Temperature-keyed user energies (reaction.py:228-262: ``dErxn_user[T]``):
descriptor name -> {T: value in eV}.  System._inputs fills such a descriptor's
column from each condition's temperature."""


def tkeyed(values):
    """A user energy given as a dict keyed by temperature, as a per-condition
    descriptor named after its content (the same dict is the same descriptor,
    so a network's structural digest does not depend on object identity)."""
    table = {float(k): float(v) for k, v in values.items()}
    import hashlib
    name = '@T:' + hashlib.sha1(repr(sorted(table.items())).encode()).hexdigest()[:16]
    TKEYED[name] = table
    return Descriptor(name)


TSYM = LinearForm({('T',): 1.0})
"""The per-condition temperature as a form (dGrxn_user = E + S*TSYM)."""

PSYM = object()
"""Marker for the per-condition pressure (only enters through tran features)."""


def clamp0(x):
    """max(x, 0) -- the np.max((E_TS - E_IS, 0.0)) of the volcano driver
    (examples/COOxVolcano/cooxvolcano.py:41,45)."""
    f = as_form(x)
    if f.is_constant():
        return as_form(max(f.constant(), 0.0))
    cid = next(_clamp_ids)
    clamps = dict(f.clamps)
    clamps[cid] = f
    return LinearForm({('clamp', cid): 1.0}, clamps, f.refs)


def feature_form(kind, state):
    """vib / tran / rot feature of a State (evaluated per condition on the device)."""
    return LinearForm({(kind, state.name): 1.0}, refs={state.name: state})
