"""The exact solve's principal pivot tableau (kernel_v2.inc dual_ppt / ppt_pivot), restated in
numpy operation by operation, on random strictly convex dual problems
    min 1/2 f'Hf + b'f,  f >= 0   (H = A + diag(R) positive definite)
and on Delassus-like ones (pyramid rows of one contact are nearly dependent): the block
principal pivoting iterates, done as single rank-1 pivots on the unit-diagonal tableau with
the kernel's one-FMA form (row p stored with P_p - 1, T_ip taken from row p through the sign
symmetry of the tableau of a symmetric H), reach the unique KKT point. The oracle solves the
same iterates with an LDL' factorization per iterate (oracle/pianosim_ref.c dual_solve); the
GPU tests compare the kernel with it directly (test_gpu_solver.py)."""
import numpy as np
import pytest

EXACT_TOL = 2e-5
EXACT_MAXIT = 32


def _pivot(T, q, p, F, dt):
    """One principal pivot in the kernel's form (all lanes at once)."""
    n = len(q)
    P = T[p].copy()
    P[p] = P[p] - dt(1.0)  # atomicAdd(&P[p], -1)
    qp = q[p]
    inv = dt(1.0) / (P[p] + dt(1.0))
    sig = np.array([((F >> i) ^ (F >> p)) & 1 for i in range(n)], bool)
    a = np.where(sig, -P, P)  # T_ip = sig_i sig_p T_pi
    g = (a * inv).astype(dt)
    g[p] = dt(1.0) + inv
    T -= g[:, None] * P[None, :]
    q -= g * qp


def tableau_bpp(H, b, f_warm, dt=np.float64, tol=EXACT_TOL):
    """dual_ppt: scaled tableau, start set from the warm-up forces, BPP exchanges (KKT check
    at `tol` relative: the kernel's 2e-5 in fp32; the oracle's 1e-10 for the fp64 runs)."""
    n = len(b)
    H = H.astype(dt)
    b = b.astype(dt)
    s = (1.0 / np.sqrt(np.diag(H))).astype(dt)
    T = (s[:, None] * H * s[None, :]).astype(dt)
    q = (s * b).astype(dt)
    fs = (f_warm / s).astype(dt)
    F0 = 0
    for i in np.nonzero(fs - (q + T @ fs) > 0)[0]:
        F0 |= 1 << int(i)
    wtol = tol * np.abs(q).max()
    F = 0
    for p in range(n):
        if (F0 >> p) & 1:
            _pivot(T, q, p, F, dt)
            F |= 1 << p
    ninf, backup, iters = n + 1, 3, 0
    for _ in range(EXACT_MAXIT):
        iters += 1
        inF = np.array([(F >> i) & 1 for i in range(n)], bool)
        ftol = tol * (np.abs(q[inF]).max() if inF.any() else 0.0)
        V = [i for i in range(n) if (q[i] < -ftol if inF[i] else q[i] < -wtol)]
        if not V:
            break
        if len(V) < ninf:
            ninf, backup, X = len(V), 3, V
        elif backup > 0:
            backup, X = backup - 1, V
        else:
            X = [max(V)]  # Murty
        for p in X:
            _pivot(T, q, p, F, dt)
            F ^= 1 << p
    inF = np.array([(F >> i) & 1 for i in range(n)], bool)
    return np.where(inF, np.maximum(s * q, 0.0), 0.0).astype(np.float64), iters


def pgs(H, b, sweeps):
    f = np.zeros(len(b))
    for _ in range(sweeps):
        for i in range(len(b)):
            f[i] = max(0.0, f[i] - (H[i] @ f + b[i]) / H[i, i])
    return f


def kkt_residual(H, b, f):
    w = H @ f + b
    return max(-f.min(), -w.min(), np.abs(f * w).max())


def _problem(rng, n, kind):
    if kind == "random":
        A = rng.standard_normal((n, n + 3))
        A = A @ A.T
    else:  # Delassus-like: 4 pyramid rows n +- mu t per contact over a few dofs
        nd = 12
        J = []
        for _ in range((n + 3) // 4):
            nrm, t1, t2 = rng.standard_normal((3, nd))
            mu = 0.8
            J += [nrm + mu * t1, nrm - mu * t1, nrm + mu * t2, nrm - mu * t2]
        J = np.array(J[:n])
        Minv = np.diag(rng.uniform(0.5, 50.0, nd))
        A = J @ Minv @ J.T
    R = 0.05 * np.diag(A) + 1e-6
    return A + np.diag(R), rng.standard_normal(n) * np.sqrt(np.diag(A))


@pytest.mark.parametrize("kind", ["random", "pyramid"])
@pytest.mark.parametrize("n", [4, 12, 33, 48, 64])
def test_tableau_bpp_reaches_the_kkt_point(n, kind):
    rng = np.random.default_rng(n + (0 if kind == "random" else 1000))
    for _ in range(4):
        H, b = _problem(rng, n, kind)
        f, iters = tableau_bpp(H, b, pgs(H, b, 2), tol=1e-10)
        scale = np.abs(b).max() * max(1.0, np.abs(f).max())
        assert kkt_residual(H, b, f) <= 1e-9 * scale, (kkt_residual(H, b, f), iters)
        # strictly convex: the KKT point is unique - PGS run to convergence finds the same one
        g = pgs(H, b, 4000)
        assert np.abs(f - g).max() <= 1e-6 * max(1.0, np.abs(g).max())


@pytest.mark.parametrize("n", [12, 48])
def test_tableau_bpp_in_fp32(n):
    """The kernel's precision: fp32 tableau within 1e-4 relative of the fp64 solution."""
    rng = np.random.default_rng(7 + n)
    for _ in range(4):
        H, b = _problem(rng, n, "pyramid")
        f64, _ = tableau_bpp(H, b, pgs(H, b, 2), tol=1e-10)
        f32, _ = tableau_bpp(H, b, pgs(H, b, 2).astype(np.float32), dt=np.float32)
        assert np.abs(f32 - f64).max() <= 1e-4 * max(1.0, np.abs(f64).max())
