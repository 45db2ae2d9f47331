"""Closed-form known answers for the piano keys, from MuJoCo's documented formulas applied to
the reference's exact piano constants (piano_constants.py:22-85, piano_mjcf.py:25-402,
tasks/base.py:28-31,66). No engine code: each function states the formula it evaluates.

A key is a hinge body about +y at the back edge of its box (anchor = (-half_x, 0, 0) in the
key frame), COM at the box centre, so about the hinge:
  * M = m (L^2 + H^2) / 12 + m (L/2)^2 + armature        (box inertia, parallel axis)
  * qfrc_passive = -k (q - springref) - d v              (joint stiffness, damping)
  * gravity: generalized force m g (L/2) cos q             ((r x m g)_y, r = R_y(q) (L/2, 0, 0))
Integration (mjINT_EULER with implicit joint damping, mj_EulerSkip):
  v' = v + h (M + h d)^-1 (qfrc_smooth + qfrc_constraint),  q' = q + h v'.
Joint-limit soft constraint (MuJoCo "Solver parameters"): distance r (< 0 when violated),
  impedance imp(r) from solimp = (d0, dwidth, width, midpoint, power),
  aref = -b (J v) - k_s imp(r) r,  k_s = 1 / (dwidth^2 tc^2 dampratio^2),  b = 2 / (dwidth tc),
  tc = max(solref[0], 2 h);  regulariser R = (1 - imp) / imp * diagApprox, diagApprox = 1 / M.
"""
from __future__ import annotations

import math

import numpy as np

G = 9.81


def key_params(md, k):
    half_x, half_z = md.key_half[k][0], md.key_half[k][2]
    m = md.key_mass[k]
    M = m * ((2 * half_x) ** 2 + (2 * half_z) ** 2) / 12.0 + m * half_x ** 2 + md.key_armature[k]
    return dict(M=M, m=m, hx=half_x, k=md.key_stiffness[k], d=md.key_damping[k], qref=md.key_springref[k],
                lo=md.key_range[k][0], hi=md.key_range[k][1], h=md.timestep, nsub=md.n_substeps)


def smooth_force(p, q, v, applied=0.0):
    """qfrc_passive + gravity + qfrc_applied on the key dof."""
    return -p["k"] * (q - p["qref"]) - p["d"] * v + p["m"] * G * p["hx"] * math.cos(q) + applied


def free_response(p, q0, v0, control_steps, applied=0.0):
    """q after each control step with no constraint active: the implicit-damping Euler
    recurrence, n_substeps substeps per control step."""
    q, v, out = q0, v0, []
    for _ in range(control_steps):
        for _ in range(p["nsub"]):
            v = v + p["h"] * smooth_force(p, q, v, applied) / (p["M"] + p["h"] * p["d"])
            q = q + p["h"] * v
        out.append(q)
    return np.array(out)


def impedance(solimp, r):
    d0, dw, width, mid, power = solimp
    d0, dw = min(max(d0, 1e-4), 0.9999), min(max(dw, 1e-4), 0.9999)
    x = abs(r) / width
    if x >= 1.0 or width <= 1e-15:
        imp = dw
    else:
        if power == 1.0:
            y = x
        elif x <= mid:
            y = x ** power / mid ** (power - 1)
        else:
            y = 1 - (1 - x) ** power / (1 - mid) ** (power - 1)
        imp = d0 + y * (dw - d0)
    return min(max(imp, 1e-4), 0.9999)


def limit_equilibrium(md, p, side, applied=0.0):
    """Resting penetration r* (< 0) of a key held against its lower (side 0) or upper (side 1)
    limit by the net smooth force. At rest (v = 0, qacc = 0) the constraint force cancels the
    net force tau, f = |tau|, and the soft-constraint solution f = (aref - J a_smooth)/(A + R)
    with A = 1/M gives k_s imp(r) r = -|tau| (1 - imp(r)) / (imp(r) M): solved for r by
    bisection (imp depends on |r|). Returns the resting joint position."""
    solref, solimp = list(md.limit_solref), list(md.limit_solimp)
    dw = min(max(solimp[1], 1e-4), 0.9999)
    tc = max(solref[0], 2 * p["h"])
    ks = 1.0 / (dw * dw * tc * tc * solref[1] * solref[1])

    def q_of(r):
        return p["lo"] + r if side == 0 else p["hi"] - r

    def resid(r):
        tau = smooth_force(p, q_of(r), 0.0, applied)
        tau_push = -tau if side == 0 else tau  # force pushing INTO the limit, > 0
        imp = impedance(solimp, r)
        return ks * imp * r + tau_push * (1 - imp) / (imp * p["M"])

    lo, hi = -0.5, 0.0  # resid(0) > 0 when the key is pushed into the limit; resid(-0.5) < 0
    assert resid(hi) > 0 > resid(lo)
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if resid(mid) > 0:
            hi = mid
        else:
            lo = mid
    return q_of(0.5 * (lo + hi))


def frictionloss_qacc(md, xs, A, fl, v):
    """One dof with a friction-loss row (MuJoCo: J = e_i, pos = 0, bound |f| <= frictionloss,
    solreffriction / solimpfriction; every other row inactive). ``xs`` = the dof's acceleration
    without the row (qacc_smooth: the same state with frictionloss 0), ``A`` = (M^-1)_ii = the
    dof's invweight0 when the configuration is qpos0, ``v`` = the dof's velocity.
    The soft row's reference acceleration is aref = -b v (b = 2 / (dmax timeconst); no
    stiffness term at pos 0), R = (1 - imp) / imp * A, imp = imp(0) = d0. The minimiser of the
    primal cost in the row's quadratic zone is f = -(xs - aref) / (A + R) ("creep": the
    regularised stick); when |f| exceeds the bound the row saturates at f = -fl sign(xs - aref)
    ("slip"). Returns (qacc of the dof = xs + A f, f, regime)."""
    solref, solimp = list(md.friction_solref), list(md.friction_solimp)
    dmax = min(max(solimp[1], 1e-4), 0.9999)
    tc = max(solref[0], 2 * md.timestep)
    aref = -(2.0 / (dmax * tc)) * v
    imp = impedance(solimp, 0.0)
    R = (1 - imp) / imp * A
    f = -(xs - aref) / (A + R)
    regime = "creep"
    if abs(f) > fl:
        f, regime = -fl * np.sign(xs - aref), "slip"
    return xs + A * f, f, regime
