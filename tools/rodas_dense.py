"""Derivation and check of the integrator's coefficient sets (csrc/mk_solver.h
namespaces rodas4 / rodas4_dense; test infrastructure, no GPU).

  1. Order of the step on a nonstiff problem (4 for both sets) and on the
     Prothero-Robinson problem y' = lam (y - sin t) + cos t (RODAS4 drops to
     order ~1 there, RODAS4P keeps ~3).
  2. The RODAS4P dense output: the transformed tableau is mapped to the
     standard form (alpha = A Gamma, Gamma = (diag(1/g) - C)^-1, weights
     m Gamma), the continuous weights b(s) = s m + s(1-s)(D2 + s D3) are made
     to satisfy the four order-3 conditions as polynomials in s, and the free
     parameter of each of D2, D3 is fixed by d2 = d3 = 0 in the stiff limit
     (h lam -> -inf on y' = lam y).  The solution is D3 = (32/7) e5,
     D25 = -40/7 and D21..D24 below; the same conditions hold for RODAS4's
     Hairer-Wanner set (checked).
  3. Interior accuracy of both dense outputs.

    python tools/rodas_dense.py
"""
import numpy as np

g = 0.25
RODAS4 = dict(
    A=[[], [1.544], [0.9466785280815826, 0.2557011698983284],
       [3.314825187068521, 2.896124015972201, 0.9986419139977817],
       [1.221224509226641, 6.019134481288629, 12.53708332932087, -0.6878860361058950]],
    C=[[], [-5.6688], [-2.430093356833875, -0.2063599157091915],
       [-0.1073529058151375, -9.594562251023355, -20.47028614809616],
       [7.496443313967647, -10.24680431464352, -33.99990352819905, 11.70890893206160],
       [8.083246795921522, -7.981132988064893, -31.52159432874371, 16.31930543123136, -6.058818238834054]],
    D2=[10.12623508344586, -7.487995877610167, -34.80091861555747, -7.992771707568823, 1.025137723295662],
    D3=[-0.6762803392801253, 6.087714651680015, 16.43084320892478, 24.76722511418386, -6.594389125716872])
RODAS4P = dict(
    A=[[], [3.0], [1.831036793486759, 0.4955183967433795],
       [2.304376582692669, -0.05249275245743001, -1.176798761832782],
       [-7.170454962423024, -4.741636671481785, -16.31002631330971, -1.062004044111401]],
    C=[[], [-12.0], [-8.791795173947035, -2.207865586973518],
       [10.81793056857153, 6.780270611428266, 19.53485944642410],
       [34.19095006749676, 15.49671153725963, 54.74760875964130, 14.16005392148534],
       [34.62605830930532, 15.30084976114473, 56.99955578662667, 18.40807009793095, -5.714285714285717]],
    D2=[26.549127843114945, 10.967258456569217, 35.997973167097996, 8.496032352891316, -40.0 / 7.0],
    D3=[0.0, 0.0, 0.0, 0.0, 32.0 / 7.0])


def step(M, f, J, y, h, dense=()):
    """One step; returns y1 and the dense-output samples at s in `dense`."""
    A, C = M['A'], M['C']
    W = np.eye(y.size) / (h * g) - J(y)
    ks, u, fu = [], y.copy(), f(y)
    for i in range(6):
        rhs = fu + (1 / h) * sum(C[i][j] * ks[j] for j in range(i)) if i else fu.copy()
        ks.append(np.linalg.solve(W, rhs))
        if i < 4:
            u = y + sum(A[i + 1][j] * ks[j] for j in range(i + 1))
            fu = f(u)
        elif i == 4:
            u = u + ks[4]
            fu = f(u)
    y1 = u + ks[5]
    d2 = sum(M['D2'][j] * ks[j] for j in range(5))
    d3 = sum(M['D3'][j] * ks[j] for j in range(5))
    return y1, [(1 - s) * y + s * (y1 + (1 - s) * (d2 + s * d3)) for s in dense]


def standard_form(M):
    A = np.zeros((6, 6))
    C = np.zeros((6, 6))
    for i in range(1, 5):
        A[i, :i] = M['A'][i]
    A[5, :5] = A[4, :5]
    A[5, 4] = 1.0
    for i in range(1, 6):
        C[i, :i] = M['C'][i]
    Gam = np.linalg.inv(np.diag(np.full(6, 1 / g)) - C)
    m = A[5].copy()
    m[5] = 1.0
    return A @ Gam, Gam, m


def dense_conditions(M):
    """Rows w_k and right-hand sides so that the order-3 conditions of the
    continuous weights read D2 . w_k = r2_k and D3 . w_k = r3_k."""
    alpha, Gam, m = standard_form(M)
    beta = alpha + Gam - np.diag(np.diag(Gam))
    a, bp = alpha.sum(1), beta.sum(1)
    vs = [np.ones(6), bp, a * a, beta @ bp]
    # the conditions' right-hand sides as [s, s^2, s^3] coefficients
    polys = [(1, 0, 0), (-g, 0.5, 0), (0, 0, 1 / 3), (g * g, -g, 1 / 6)]
    W, r2, r3 = [], [], []
    for v, (c1, c2, c3) in zip(vs, polys):
        x = m @ Gam @ v
        W.append((Gam @ v)[:5])
        r2.append(c1 - x)
        r3.append(-c3)
    return np.array(W), np.array(r2), np.array(r3)


def stiff_limit_stages(M):
    """k_i / y0 as h lam -> -inf on y' = lam y: k_i = -u_i."""
    A, ks, u = M['A'], [], 1.0
    for i in range(6):
        ks.append(-u)
        if i < 4:
            u = 1.0 + sum(A[i + 1][j] * ks[j] for j in range(i + 1))
        elif i == 4:
            u = u + ks[4]
    return np.array(ks)


def main():
    np.set_printoptions(precision=3)

    def f1(y):
        return np.array([y[1], -np.sin(y[0]) + 0.1 * y[1] ** 2])

    def J1(y):
        return np.array([[0, 1.0], [-np.cos(y[0]), 0.2 * y[1]]])

    def run(M, f, J, y, T, N):
        for _ in range(N):
            y, _ = step(M, f, J, y, T / N)
        return y
    ref = run(RODAS4, f1, J1, np.array([1.0, 0.5]), 2.0, 20000)
    for name, M in (('RODAS4', RODAS4), ('RODAS4P', RODAS4P)):
        e = [np.abs(run(M, f1, J1, np.array([1.0, 0.5]), 2.0, N) - ref).max() for N in (20, 40, 80, 160)]
        print('%-8s nonstiff order %s' % (name, np.round(np.log2(np.array(e[:-1]) / e[1:]), 2)))
        for lam in (-1e4, -1e8):
            f2 = lambda z: np.array([lam * (z[0] - np.sin(z[1])) + np.cos(z[1]), 1.0])
            J2 = lambda z: np.array([[lam, -lam * np.cos(z[1]) - np.sin(z[1])], [0, 0]])
            e = [abs(run(M, f2, J2, np.zeros(2), 1.0, N)[0] - np.sin(1.0)) for N in (10, 20, 40)]
            print('%-8s Prothero-Robinson lam %g: errors %s' % (name, lam, np.array(e)))
        W, r2, r3 = dense_conditions(M)
        print('%-8s dense-output condition residuals: D2 %.1e, D3 %.1e'
              % (name, np.abs(W @ M['D2'] - r2).max(), np.abs(W @ M['D3'] - r3).max()))
    # derive the RODAS4P set: D3 = (32/7) e5 and D25 = -40/7 are the stiff-limit
    # solution's exact tail (a float64 solve of the full system returns them
    # to ~1e-13); D21..D24 from the four conditions
    W, r2, r3 = dense_conditions(RODAS4P)
    kinf = stiff_limit_stages(RODAS4P)[:5]
    full2 = np.linalg.solve(np.vstack([W, kinf]), np.r_[r2, 0.0])
    full3 = np.linalg.solve(np.vstack([W, kinf]), np.r_[r3, 0.0])
    d25 = -40.0 / 7.0
    head = np.linalg.solve(W[:, :4], r2 - W[:, 4] * d25)
    print('RODAS4P D2 (full solve) %s; D3 (full solve) %s' % (full2, full3))
    print('RODAS4P D2 =', [repr(float(x)) for x in np.r_[head, d25]])
    assert np.allclose(np.r_[head, d25], RODAS4P['D2'], rtol=1e-14, atol=0)
    # interior accuracy (local interpolation error at s = 1/4, 1/2, 3/4)
    for name, M in (('RODAS4', RODAS4), ('RODAS4P', RODAS4P)):
        for lam in (None, -1e4):
            if lam is None:
                f, J, y0 = f1, J1, np.array([1.0, 0.5])
                from scipy.integrate import solve_ivp
                exact = lambda y, dt: solve_ivp(lambda t, z: f1(z), (0, dt), y, rtol=1e-13, atol=1e-14,
                                                method='DOP853').y[:, -1]
            else:
                f = lambda z: np.array([lam * (z[0] - np.sin(z[1])) + np.cos(z[1]), 1.0])
                J = lambda z: np.array([[lam, -lam * np.cos(z[1]) - np.sin(z[1])], [0, 0]])
                y0 = np.zeros(2)
                exact = lambda z, dt: np.array([np.sin(z[1] + dt) + (z[0] - np.sin(z[1])) * np.exp(lam * dt),
                                                z[1] + dt])
            errs = []
            for N in (5, 10, 20, 40):
                y, h, e = y0.copy(), 1.0 / N, 0.0
                for _ in range(N):
                    y1, samp = step(M, f, J, y, h, dense=(0.25, 0.5, 0.75))
                    e = max(e, max(abs(sv[0] - exact(y, s * h)[0]) for s, sv in zip((0.25, 0.5, 0.75), samp)))
                    y = y1
                errs.append(e)
            print('%-8s dense interior error (%s): %s' % (name, 'nonstiff' if lam is None else 'PR %g' % lam,
                                                          np.array(errs)))


if __name__ == '__main__':
    main()
