"""Diagnostic (test infrastructure, never the product): a numpy restatement of
the device Rosenbrock integrator (RODAS4P; METHOD=rodas4 for RODAS4) of csrc/mk_solver.h / mk_group.h (same stages,
initial step, error norm, step controller and site-balance projection) that
records the step history of one condition of the oracle's models.

    python tools/rodas_mirror.py synthetic IDX     (a condition of the synthetic bench config)
    python tools/rodas_mirror.py volcano ECO EO    (a volcano grid point, steady-rule tolerances)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

g = 0.25
A = [[], [1.544], [0.9466785280815826, 0.2557011698983284],
     [3.314825187068521, 2.896124015972201, 0.9986419139977817],
     [1.221224509226641, 6.019134481288629, 12.53708332932087, -0.6878860361058950]]
Cc = [[], [-5.6688], [-2.430093356833875, -0.2063599157091915],
      [-0.1073529058151375, -9.594562251023355, -20.47028614809616],
      [7.496443313967647, -10.24680431464352, -33.99990352819905, 11.70890893206160],
      [8.083246795921522, -7.981132988064893, -31.52159432874371, 16.31930543123136, -6.058818238834054]]

DD2 = [10.12623508344586, -7.487995877610167, -34.80091861555747, -7.992771707568823, 1.025137723295662]
DD3 = [-0.6762803392801253, 6.087714651680015, 16.43084320892478, 24.76722511418386, -6.594389125716872]

# the device default (csrc/mk_solver.h PCK_RODAS4P=1): Steinebach's RODAS4P
# and its stiff-limit dense output; METHOD=rodas4 keeps the Hairer-Wanner set
# above (the device's PCK_RODAS4P=0)
if os.environ.get('METHOD', 'rodas4p') == 'rodas4p':
    A = [[], [3.0], [1.831036793486759, 0.4955183967433795],
         [2.304376582692669, -0.05249275245743001, -1.176798761832782],
         [-7.170454962423024, -4.741636671481785, -16.31002631330971, -1.062004044111401]]
    Cc = [[], [-12.0], [-8.791795173947035, -2.207865586973518],
          [10.81793056857153, 6.780270611428266, 19.53485944642410],
          [34.19095006749676, 15.49671153725963, 54.74760875964130, 14.16005392148534],
          [34.62605830930532, 15.30084976114473, 56.99955578662667, 18.40807009793095, -5.714285714285717]]
    DD2 = [26.549127843114945, 10.967258456569217, 35.997973167097996, 8.496032352891316, -40.0 / 7.0]
    DD3 = [0.0, 0.0, 0.0, 0.0, 32.0 / 7.0]

PIVLOG = []
COMP = []       # COMP=1: (t, y, per-species squared scaled error) of every step


def gpu_lu_solve(W, rhs_list):
    """LU with the lane-group kernel's pivot rule (mk_group.h grp_lu): the
    pivot of column k is the free row with the largest float32 |a| (low 6
    mantissa bits replaced by the lane id, ties -> highest lane)."""
    A = W.copy()
    n = A.shape[0]
    free = np.ones(n, bool)
    order = []
    for k in range(n):
        mag = np.abs(A[:, k]).astype(np.float32).view(np.uint32) & ~np.uint32(63)
        key = np.where(free, (mag | np.arange(n, dtype=np.uint32)).astype(np.int64), -1)
        p = int(np.argmax(key))
        piv = A[p, k]
        PIVLOG.append(abs(piv))
        if not (piv != 0.0 and np.isfinite(piv)):
            raise np.linalg.LinAlgError('zero pivot col %d' % k)
        free[p] = False
        order.append(p)
        for r in np.nonzero(free)[0]:
            l = A[r, k] / piv
            A[r, k] = l
            A[r, k + 1:] -= l * A[p, k + 1:]
    P = np.array(order)
    L = np.eye(n)
    U = np.zeros((n, n))
    for i, p in enumerate(P):
        U[i, i:] = A[p, i:]
        L[i, :i] = A[p, :i]
    out = []
    for b in rhs_list:
        z = np.linalg.solve(L, b[P])
        out.append(np.linalg.solve(U, z))
    return out


def rodas4(f, J, y, t0, t_end, rtol, atol, cons=None, max_steps=200000, cons_rows=None, trace=None, gpu_lu=False,
           t_out=None, samples=None, ctrl='std'):
    """Returns (y, status, nsteps).  cons: conservation matrix (rows >= 0 get
    the multiplicative projection).  cons_rows: optional (C, piv) -- replace the
    pivot rows of W by the conservation rows (the index-reduced stage system).
    ctrl: 'std' (the device's controller) or 'pred' (Gustafsson's predictive
    controller, Hairer & Wanner's RODAS: A/B only)."""
    NS = y.size
    F0 = f(y)
    span = t_end - t0
    sc = atol + rtol * np.abs(y)
    d0 = np.sqrt(np.mean((y / sc) ** 2))
    d1 = np.sqrt(np.mean((F0 / sc) ** 2))
    h0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
    h0 = min(h0, span)
    F1 = f(y + h0 * F0)
    d2 = np.sqrt(np.mean(((F1 - F0) / sc) ** 2)) / h0
    h1 = max(1e-6, h0 * 1e-3) if (d1 <= 1e-15 and d2 <= 1e-15) else (0.01 / max(d1, d2)) ** 0.2
    h = min(100 * h0, h1, span)
    c0 = cons @ y if cons is not None else None
    t = t0
    n = 0
    ko = 0
    hacc, erracc, rejected = None, None, False
    if t_out is not None:
        while ko < len(t_out) and t_out[ko] <= t0:
            samples.append(y.copy())
            ko += 1
    while t < t_end:
        if n >= max_steps:
            return y, 1, n
        n += 1
        last = False
        if t + h >= t_end:
            h = t_end - t
            last = True
        ih = 1.0 / h
        W = np.eye(NS) * ih / g - J(y)
        if cons_rows is not None:
            Cr, piv = cons_rows
            for l, p in enumerate(piv):
                W[p] = Cr[l] * np.abs(W[p]).max()
        ks = []
        u = y.copy()
        fu = F0
        ok = True
        for i in range(6):
            if i == 0:
                rhs = F0.copy()
            else:
                rhs = fu + ih * sum(Cc[i][j] * ks[j] for j in range(i))
            if cons_rows is not None:
                for p in cons_rows[1]:
                    rhs[p] = 0.0
            try:
                k = gpu_lu_solve(W, [rhs])[0] if gpu_lu else np.linalg.solve(W, rhs)
            except np.linalg.LinAlgError:
                ok = False
                break
            if os.environ.get('KPROJ') and cons is not None:
                # KPROJ=1: the conserved totals' drift removed along y (the
                # multiplicative projection's direction); KPROJ=orth:
                # orthogonally (spreads rounding onto tiny species: A/B only)
                if os.environ['KPROJ'] == 'orth':
                    for crow in np.linalg.qr(np.asarray(cons, float).T)[0].T:
                        k = k - (crow @ k) * crow
                else:
                    for crow in np.asarray(cons, float):
                        if np.all(crow >= 0.0) and crow @ y > 0.0:
                            # along the law's own species only: a species outside
                            # it (a CSTR gas, another site type) keeps its stage
                            k = k - np.where(crow != 0.0, y, 0.0) * ((crow @ k) / (crow @ y))
            ks.append(k)
            if i < 4:
                u = y + sum(A[i + 1][j] * ks[j] for j in range(i + 1))
                fu = f(u)
            elif i == 4:
                u = u + k
                fu = f(u)
        if not ok:
            h *= 0.25
            continue
        unew = u + ks[5]
        fin = np.all(np.isfinite(unew))
        scl = atol + rtol * np.maximum(np.abs(y), np.abs(unew))
        q = np.mean((ks[5] / scl) ** 2) if fin else np.inf
        if os.environ.get('COMP'):
            COMP.append((t, y.copy(), (ks[5] / scl) ** 2))
        fac = 0.9 * q ** -0.125 if q > 0 else np.inf
        neg = (unew < -atol) & (os.environ.get('NOPOS') is None)
        pf = float(np.min((y[neg] + atol) / (y[neg] - unew[neg]))) if np.any(neg) else 1.0
        acc = q <= 1.0 and pf >= 1.0
        if q <= 1.0 and pf < 1.0:
            if trace is not None:
                trace.append((t, h, q, False))
            h *= max(0.1, 0.9 * pf)
            continue
        if trace is not None:
            trace.append((t, h, q, acc))
            if os.environ.get('ERRDUMP') and t > float(os.environ['ERRDUMP']) and len(trace) % 50 == 0:
                e = ks[5] / scl
                j = int(np.argmax(np.abs(e)))
                print('t %.3e h %.3e q %.3e worst comp %d y %.3e unew %.3e e %.3e |e| sorted %s' % (
                    t, h, q, j, y[j], unew[j], e[j], np.array2string(np.sort(np.abs(e))[::-1][:4], precision=2)))
        if acc:
            t_old, y_old = t, y
            t = t_end if last else t + h
            cm = os.environ.get('CLIPMODE', 'noclip' if os.environ.get('NOCLIP') else 'clip')
            y = np.maximum(unew, 0.0) if cm == 'clip' else unew
            if cons is not None:
                for l in range(cons.shape[0]):
                    if np.all(cons[l] >= 0):
                        sm = cons[l] @ y
                        if sm > 0:
                            y = np.where(cons[l] != 0, y * c0[l] / sm, y)
            if t_out is not None:        # Rodas4 dense output (mk_solver.h rodas4_dense)
                d2 = sum(c * k for c, k in zip(DD2, ks[:5]))
                d3 = sum(c * k for c, k in zip(DD3, ks[:5]))
                while ko < len(t_out) and t_out[ko] <= t:
                    s = min((t_out[ko] - t_old) / h, 1.0)
                    s1 = 1.0 - s
                    samples.append(y_old * s1 + s * (y + s1 * (d2 + s * d3)))
                    ko += 1
            F0 = f(y)
            if cm == 'hybrid':                 # clip only components that are negative and still falling
                neg = (y < 0.0) & (F0 < 0.0)
                if np.any(neg):
                    y = np.where(neg, 0.0, y)
                    F0 = f(y)
            m = min(float(os.environ.get('FACMAX', 10.0)), max(0.2, fac))
            if ctrl == 'pred':
                err = max(np.sqrt(q), 1e-300)
                if hacc is not None:
                    mg = 0.9 * (h / hacc) * (erracc / err ** 2) ** 0.25
                    m = min(m, min(6.0, max(0.2, mg)))
                hacc, erracc = h, max(1e-2, err)
                if rejected:
                    m = min(m, 1.0)
                rejected = False
            h *= m
        else:
            rejected = True
            h *= max(0.2, fac) if fin else 0.25
        if not (h > 2.220446049250313e-15 * max(abs(t), 1e-300)) and t < t_end:
            return y, 2, n
    return y, 0, n


def synthetic_model(idx, n_total=65536):
    from _synth import spec_of
    from oracle import mk_oracle as O
    from pycatkin_amd.functions.synthetic import synthetic_network
    rng = np.random.default_rng(0)
    D = rng.uniform(-0.5, 0.5, (n_total, 4))[idx]
    m = O.ClassicModel(spec_of(synthetic_network(), D), T=500.0)
    return m, D


def dmtm_model(T):
    from oracle import mk_oracle as O
    spec = O.load_spec(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'DMTM', 'input.json'))
    return O.ClassicModel(spec, T=T, p=float(os.environ.get('P', spec['system']['p']))), [T]


def volcano_model(eco, eo):
    import copy
    from oracle import mk_oracle as O
    spec = O.load_spec(os.path.join(ROOT, 'tests', 'golden', 'inputs', 'COOxVolcano', 'input.json'))
    spec = copy.deepcopy(spec)
    O.set_volcano_point(spec, eco, eo, None)
    return O.ClassicModel(spec, T=None), [eco, eo]


def main():
    which = sys.argv[1]
    if which == 'volcano':
        m, D = volcano_model(float(sys.argv[2]), float(sys.argv[3]))
        D = np.array(D)
        idx = 0
        sys.argv = sys.argv[:2] + sys.argv[4:]
        # pycatkin_amd/classes/system.py STEADY_TRANSIENT, the input's t_end
        t_end, rtol, atol = 3600.0, float(os.environ.get('RTOL', 1e-6)), float(os.environ.get('ATOL', 1e-22))
    elif which == 'dmtm':
        m, D = dmtm_model(float(sys.argv[2]))
        D = np.array(D)
        idx = 0
        t_end, rtol, atol = 1e12, float(os.environ.get('RTOL', 1e-10)), float(os.environ.get('ATOL', 1e-14))
    else:
        idx = int(sys.argv[2])
        m, D = synthetic_model(idx)
        t_end, rtol, atol = 1e4, 1e-8, 1e-10
    dyn = m.dyn
    full = m.y0.copy()

    clamp = os.environ.get('CLAMP') is not None      # rates / Jacobian at max(y, 0)

    def f(y):
        full[dyn] = np.maximum(y, 0.0) if clamp else y
        return m.rhs(full)[dyn]

    def J(y):
        full[dyn] = np.maximum(y, 0.0) if clamp else y
        return m.jac(full)[np.ix_(dyn, dyn)]
    y0 = m.y0[dyn].copy()
    C = m.conservation()
    from oracle.mk_oracle import _rref
    Cr, piv = _rref(C)
    mode = sys.argv[3] if len(sys.argv) > 3 else 'plain'
    tr = []
    y, st, n = rodas4(f, J, y0, 0.0, t_end, rtol, atol, cons=Cr, max_steps=int(os.environ.get('MAXSTEPS', 20000)),
                      cons_rows=(Cr, piv) if mode == 'rows' else None, trace=tr, gpu_lu='gpulu' in sys.argv)
    if PIVLOG:
        pl = np.array(PIVLOG)
        print('pivot |min| %.3e, fraction < 1e-30: %.4f' % (pl.min(), np.mean(pl < 1e-30)))
    tr = np.array(tr)
    print(json.dumps(dict(idx=idx, D=D.tolist(), status=st, nsteps=n, mode=mode)))
    if len(tr):
        acc = tr[:, 3] > 0
        print('accepted %d rejected %d; last t %.3e h %.3e' % (acc.sum(), (~acc).sum(), tr[-1, 0], tr[-1, 1]))
        k = len(tr)
        for row in tr[max(0, k - 12):]:
            print('  t %.6e h %.3e q %.3e %s' % (row[0], row[1], row[2], 'acc' if row[3] else 'rej'))
        # where did time go: steps per decade of t
        ts = tr[:, 0]
        dec = np.floor(np.log10(np.maximum(ts, 1e-20)))
        u, c = np.unique(dec, return_counts=True)
        print('steps per decade of t:', dict(zip(u.astype(int).tolist(), c.tolist())))


if __name__ == '__main__':
    main()
