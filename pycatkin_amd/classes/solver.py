"""SteadyStateSolver: pycatkin/classes/solver.py on the device.

The reference wraps scipy (solve_ivp / root / minimize) around the patched
System's _fun_ss / _jac_ss (solver.py:17-418).  Here every rate, Jacobian
and integration is a launch of the HIP library through the C-ABI:

  solve_ode       transient of the surface species from the normalised
                  initial state to tmax (device RODAS4P, the reference's
                  solve_ivp with rtol 1e-10 / atol 1e-12 -- the tolerances
                  solver.py:406-407 hard-codes whatever its arguments say),
                  then test_convergence; solve_ode_batch does it for a batch
                  of temperatures in one launch;
  solve_root /    the reference restarts scipy root / minimize from a
  solve_minimize  renormalised guess until test_convergence passes; here the
                  guess is polished by the device Newton (conservation rows
                  for the site balances, solver.py's `_norm` applied to the
                  guess first) and scored the same way.

test_convergence / _score / compare_scores keep the reference's checks: rate
residual (device _fun_ss), non-negative coverages, site sums, and the
eigenvalues of the device _jac_ss (numpy on the host: a check on an
NS x NS matrix, not a solve).
"""
from __future__ import annotations

from typing import NamedTuple

import numpy as np

from .system import SteadyStateResults, System


class SolScore(NamedTuple):
    """solver.py:8-15"""
    y_surf: np.ndarray
    max_rate: float
    max_jac: float
    surf_sum: list


class SteadyStateSolver:
    """solver.py:17-65"""

    def __init__(self, system, ss_guess=None, verbose=False):
        if not isinstance(system, System):
            raise ValueError('system must be Pycatkin System')
        if system.formulation != 'patched':
            raise ValueError('SteadyStateSolver works on the patched System (System(formulation="patched"))')
        self.sys = system
        self.verbose = verbose
        if getattr(system, 'initial_system', None) is None:
            system.build()
        self.ygas = self.sys.initial_system[:len(self.sys.gas_indices)]
        self.surf_map = {sid: {i - len(self.ygas) for i in idx} for sid, idx in self.sys.coverage_map.items()}
        n_surf = sum(len(v) for v in self.surf_map.values())
        if ss_guess is None:
            self.ss_guess = self._norm(np.random.uniform(size=n_surf))
        elif len(ss_guess) != n_surf:
            raise ValueError('Initial guess must have same length as number of surface sites = %d' % n_surf)
        else:
            self.ss_guess = np.asarray(ss_guess, float)

    # -- checks (solver.py:69-219) ------------------------------------------------
    def test_convergence(self, y_surf, rate_tol=1e-4, coverage_tol=5e-2, pos_jac_tol=1e-2, log=False, **kwargs):
        """solver.py:69-120: True when every check passes."""
        y_surf = np.asarray(y_surf, float)
        rate_residual = float(np.max(np.abs(self.sys._fun_ss(y_surf))))
        rate_fail = rate_residual > rate_tol
        spos_fail = bool(np.any(np.round(y_surf, 2) < 0))
        y_all = np.concatenate((self.ygas, y_surf))
        surf_sum = [float(np.sum(y_all[sorted(idx)])) for idx in self.sys.coverage_map.values()]
        ssum_fail = bool(np.any(np.abs(np.array(surf_sum) - 1) > coverage_tol))
        eig = np.linalg.eigvals(self.sys._jac_ss(y_surf))
        cplx = bool(np.iscomplex(eig).any())
        negjac_fail = bool(np.any(eig.real > pos_jac_tol)) if cplx else bool(np.any(eig.real > pos_jac_tol))
        if log:
            print('    - CHECKS: rate %s | surf_sum %s | jac_eigV %s\n        - surf_sum = %s\n'
                  '        - rate_residual = %s\n        - jacobian_eigV_max = %s'
                  % (not rate_fail, not ssum_fail, not negjac_fail, surf_sum, rate_residual, float(np.max(eig.real))))
        return not any([rate_fail, spos_fail, ssum_fail, negjac_fail])

    def test_convergence_batch(self, Y, desc=None, T=None, rate_tol=1e-4, coverage_tol=5e-2, pos_jac_tol=1e-2,
                               log=False, **kwargs):
        """test_convergence for surface states Y [n_surface, n] (index_map
        order) in two launches (rates, Jacobians), each column at its own
        temperature / descriptor energies; the eigenvalues of the n Jacobians
        in one batched LAPACK call."""
        Y = np.asarray(Y, float)
        n = Y.shape[1]
        if n == 0:
            return np.zeros(0, bool)
        f = self.sys._fun_ss_batch(Y, desc=desc, T=T)
        J = self.sys._jac_ss_batch(Y, desc=desc, T=T)
        rate_fail = np.max(np.abs(f), axis=0) > rate_tol
        spos_fail = np.any(np.round(Y, 2) < 0, axis=0)
        y_all = np.concatenate((np.repeat(self.ygas[:, None], n, axis=1), Y))
        surf_sum = np.array([y_all[sorted(idx)].sum(axis=0) for idx in self.sys.coverage_map.values()])
        ssum_fail = np.any(np.abs(surf_sum - 1) > coverage_tol, axis=0)
        eig = np.linalg.eigvals(np.moveaxis(J, 2, 0))
        negjac_fail = np.any(eig.real > pos_jac_tol, axis=1)
        if log:
            for c in range(n):
                print('    - CHECKS: rate %s | surf_sum %s | jac_eigV %s\n        - surf_sum = %s\n'
                      '        - rate_residual = %s\n        - jacobian_eigV_max = %s'
                      % (not rate_fail[c], not ssum_fail[c], not negjac_fail[c], [float(v) for v in surf_sum[:, c]],
                         float(np.max(np.abs(f[:, c]))), float(np.max(eig[c].real))))
        return ~(rate_fail | spos_fail | ssum_fail | negjac_fail)

    def _norm(self, y_surf):
        """solver.py:122-141"""
        y_surf = np.where(np.asarray(y_surf, float) < self.sys.min_tol, self.sys.min_tol, y_surf).astype(float)
        for idx in self.surf_map.values():
            ii = sorted(idx)
            y_surf[ii] /= np.sum(y_surf[ii])
        return y_surf

    def _score(self, y_surf):
        """solver.py:143-160"""
        y_surf = np.asarray(y_surf, float)
        max_rate = float(np.max(np.abs(self.sys._fun_ss(y_surf))))
        surf_sum = [float(np.sum(y_surf[sorted(idx)])) for idx in self.surf_map.values()]
        eig = np.linalg.eigvals(self.sys._jac_ss(y_surf))
        return SolScore(y_surf=y_surf, max_rate=max_rate, max_jac=float(np.max(eig.real)), surf_sum=surf_sum)

    @staticmethod
    def compare_scores(s1, s2, rate_tol=1e-4, coverage_tol=5e-2, pos_jac_tol=1e-2, **kwargs):
        """solver.py:162-219: the better of two scores."""
        r1 = [s1.max_rate < rate_tol, np.all(np.abs(np.array(s1.surf_sum) - 1) < coverage_tol), s1.max_jac < pos_jac_tol]
        r2 = [s2.max_rate < rate_tol, np.all(np.abs(np.array(s2.surf_sum) - 1) < coverage_tol), s2.max_jac < pos_jac_tol]
        d1 = np.abs(np.linalg.norm(s1.surf_sum) - 1)
        d2 = np.abs(np.linalg.norm(s2.surf_sum) - 1)
        if r1[0] and r2[0]:
            if r1[1] and r2[1]:
                return s1 if s1.max_jac < s2.max_jac else s2
            if r1[1] ^ r2[1]:
                return s1 if r1[1] else s2
            if r1[2] and r2[2]:
                return s1 if d1 < d2 else s2
            if r1[2] ^ r2[2]:
                return s1 if r1[2] else s2
            return s1 if d1 < d2 else s2
        if r1[0] ^ r2[0]:
            return s1 if r1[0] else s2
        return s1 if s1.max_rate < s2.max_rate else s2

    # -- solvers ----------------------------------------------------------------------
    def _surface_y0(self):
        return self.sys.initial_system[len(self.sys.gas_indices):]

    def solve_ode(self, method='RK45', use_jac=True, rtol=1e-10, atol=1e-12, tmax=1e4, test_convergence_kwargs=None):
        """solver.py:374-418 (device RODAS4P at rtol 1e-10 / atol 1e-12)."""
        Y, ok = self.solve_ode_batch(T=[self.sys.T], tmax=tmax, test_convergence_kwargs=test_convergence_kwargs)
        return SteadyStateResults(Y[:, 0], bool(ok[0]))

    def solve_ode_batch(self, T=None, tmax=1e4, test_convergence_kwargs=None, max_steps=200000):
        """solve_ode for a batch of temperatures in one launch: (Y [n_surface, n]
        in index_map order, success [n]).  The convergence checks run at each
        condition's own temperature."""
        kw = dict(test_convergence_kwargs or {})
        kw['log'] = bool(self.verbose)
        s = self.sys
        T = np.atleast_1d(np.asarray(s.T if T is None else T, float))
        plan = s.plan()
        y0 = s._to_plan(plan, self._surface_y0()[:, None])[:, 0]
        r = s.solve_batch(T=T, y0=np.repeat(y0[:, None], T.size, axis=1), t0=0.0, t_end=tmax, rtol=1e-10,
                          atol=1e-12, steady=False, max_steps=max_steps)
        Y = r['y'][s._from_plan(plan)]
        ok = (r['status'] == 0) & self.test_convergence_batch(Y, T=T, **kw)
        return Y, ok

    def _newton(self, x0, max_iters):
        s = self.sys
        plan = s.plan()
        y0 = s._to_plan(plan, np.asarray(x0, float)[:, None])
        r = s.solve_batch(T=[s.T], y0=y0, t0=0.0, t_end=0.0, steady=True, newton_iters=max(int(max_iters), 60))
        return r['y'][s._from_plan(plan)][:, 0], int(r['status'][0])

    def solve_root(self, max_iters=30, method='hybr', use_jac=True, tol=1e-8, test_convergence_kwargs=None,
                   log_every=5):
        """solver.py:223-291 on the device Newton (see the module docstring)."""
        kw = dict(test_convergence_kwargs or {})
        kw['log'] = bool(self.verbose)
        x0 = self._norm(self.ss_guess)
        s_keep = self._score(x0)
        x, st = self._newton(x0, max_iters)
        success = st == 0 and self.test_convergence(x, **kw)
        if success:
            return SteadyStateResults(x, True)
        s_keep = self.compare_scores(s_keep, self._score(x), **kw)
        return SteadyStateResults(s_keep.y_surf, False)

    def solve_minimize(self, max_iters=30, method=None, use_jac=True, tol=1e-8, test_convergence_kwargs=None,
                       log_every=5, use_bounds=True):
        """solver.py:293-372 on the device Newton (see the module docstring)."""
        return self.solve_root(max_iters=max_iters, tol=tol, test_convergence_kwargs=test_convergence_kwargs,
                               log_every=log_every)
