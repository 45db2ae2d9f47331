"""Physics known answers for the oracle (CPU): MuJoCo's documented formulas on the exact piano
model (tests/analytic.py), against the fp64 restatement.

* free response of keys away from their limits: the implicit-damping Euler recurrence with the
  key spring (k = 2, springref -1 deg), damping 0.05, armature 1e-3 and gravity;
* a key resting on its lower limit (the spring's preload beats gravity): the soft-constraint
  equilibrium penetration from solref / solimp;
* a key held against its upper limit by qfrc_applied = 3.0 (the value of the reference's
  piano_with_shadow_hands_test.py:228-242): the same equilibrium on the other side.
The end keys of the keyboard are used: the hands rest around y = +-0.15 and never reach them.
"""
import numpy as np
import pytest

from analytic import free_response, key_params, limit_equilibrium
from helpers import song

END_KEYS = [0, 1, 2, 3, 4, 5, 82, 83, 84, 85, 86, 87]


def _oracle(dp, ref, n=1, **kw):
    task = dp.TaskConfig(**kw)
    md, st, tc = dp.compile_task(song(dp, "twinkle"), task, canonical_actions=False)
    return md, ref.OracleEnv(md, st, tc, n)


def state(n, qkeys):
    q = np.zeros((n, 140))
    q[:, :88] = qkeys
    return dict(qpos=q, qvel=np.zeros((n, 140)), qacc_ws=np.zeros((n, 140)), ctrl=np.zeros((n, 44)),
                sustain=np.zeros(n), t_idx=np.zeros(n, np.int32), last=np.zeros(n, np.uint8))


def free_start(md):
    """Keys at 95% of their range, at rest."""
    return np.array([0.95 * md.key_range[k][1] for k in range(88)])


def test_key_free_response_matches_euler_recurrence(dp, ref):
    # one physics substep per control step: the recurrence is compared substep by substep
    md, env = _oracle(dp, ref, control_timestep=0.005)
    q0 = free_start(md)
    env.set_state(state(1, q0))
    steps = 8
    exp = {k: free_response(key_params(md, k), q0[k], 0.0, steps) for k in END_KEYS}
    for k in END_KEYS:  # the analytic trajectory stays inside the range (no limit row)
        assert (exp[k] > md.key_range[k][0]).all() and (exp[k] < md.key_range[k][1]).all()
    zero = np.zeros((1, 45), np.float32)
    for t in range(steps):
        env.step(zero)
        q = env.get_state()["qpos"][0]
        for k in END_KEYS:
            assert abs(q[k] - exp[k][t]) < 1e-12, (k, t, q[k], exp[k][t])


def test_key_rests_on_lower_limit_at_soft_constraint_equilibrium(dp, ref):
    md, env = _oracle(dp, ref)
    env.set_state(state(1, np.zeros(88)))
    zero = np.zeros((1, 45), np.float32)
    for _ in range(60):  # 3 s
        env.step(zero)
    q = env.get_state()["qpos"][0]
    for k in END_KEYS:
        qs = limit_equilibrium(md, key_params(md, k), side=0)
        assert qs < 0.0  # penetration: the spring preload exceeds the gravity torque
        assert abs(q[k] - qs) < 1e-10, (k, q[k], qs)


def test_key_held_at_upper_limit_by_applied_force(dp, ref):
    md, env = _oracle(dp, ref)
    env.set_state(state(1, np.array([md.key_range[k][1] for k in range(88)])))
    app = np.zeros((1, 140))
    app[0, END_KEYS] = 3.0
    env.set_applied(app)
    zero = np.zeros((1, 45), np.float32)
    for _ in range(40):  # 2 s
        env.step(zero)
    q = env.get_state()["qpos"][0]
    for k in END_KEYS:
        qs = limit_equilibrium(md, key_params(md, k), side=1, applied=3.0)
        assert qs > md.key_range[k][1]
        assert abs(q[k] - qs) < 1e-10, (k, q[k], qs)


def test_equilibrium_formula_self_consistent(dp):
    """The bisection root satisfies the stationarity of the discrete step: with v = 0 at q*,
    one implicit-Euler substep with the soft limit force leaves q* unchanged."""
    md = dp.model.build_model()
    from analytic import impedance, smooth_force
    for k in (0, 1):
        p = key_params(md, k)
        qs = limit_equilibrium(md, p, side=0)
        r = qs - p["lo"]
        imp = impedance(list(md.limit_solimp), r)
        tc = max(md.limit_solref[0], 2 * p["h"])
        dw = md.limit_solimp[1]
        aref = -1.0 / (dw * dw * tc * tc) * imp * r
        R = (1 - imp) / imp / p["M"]
        a_s = smooth_force(p, qs, 0.0) / p["M"]
        f = max(0.0, -(a_s - aref) / (1.0 / p["M"] + R))
        assert abs(a_s + f / p["M"]) < 1e-9 * abs(a_s)


# ------------------------------------------------------------------ joint friction loss
FL_DOFS = (5, 21)  # FFJ3 and THJ5 of each hand: ranges contain 0, so qpos0 has no limit row


def frictionloss_task(dp, fl_by_dof):
    """The authored hand with frictionloss only on the given dofs (both hands), through the MJCF
    path; one physics substep per control step."""
    hand = dp.model.authored_hand()
    dofs = [d._replace(frictionloss=fl_by_dof.get(j, 0.0)) if hasattr(d, "_replace") else
            __import__("dataclasses").replace(d, frictionloss=fl_by_dof.get(j, 0.0)) for j, d in enumerate(hand.dofs)]
    return dp.TaskConfig(hand_xml=dp.mjcf.hand_to_mjcf(hand._replace(dofs=dofs)), control_timestep=0.005)


def frictionloss_state(n, vel):
    """qpos0 (keys up, hands in their default pose, in the air), dof velocities `vel` {dof: v}."""
    s = state(n, np.zeros(88))
    for h in range(2):
        for j, v in vel.items():
            s["qvel"][:, 88 + 26 * h + j] = v
    return s


def frictionloss_cases(dp, run):
    """Known answers of one friction-loss row (analytic.frictionloss_qacc): each dof of FL_DOFS
    alone (one row per hand: the hands are independent) at qpos0, at rest and moving, with the
    bound 10x above the creep force (regularised stick) and at 0.3x of it (slip at the saturated
    force). ``run(task, state) -> qacc_ws [140]`` steps one substep on the oracle or the GPU.
    Returns [(measured, expected, regime)]."""
    from analytic import frictionloss_qacc
    out = []
    task0 = frictionloss_task(dp, {})
    md0, _, _ = dp.compile_task(song(dp, "twinkle"), task0, canonical_actions=False)
    for j in FL_DOFS:
        for v in (0.0, 0.5):
            s = frictionloss_state(1, {j: v})
            xs = run(task0, s)
            _, fu, _ = frictionloss_qacc(md0, xs[88 + j], md0.dof_invweight[0][j], np.inf, v)
            for scale in (10.0, 0.3):
                fl = float(scale * abs(fu))
                task = frictionloss_task(dp, {j: fl})
                md, _, _ = dp.compile_task(song(dp, "twinkle"), task, canonical_actions=False)
                x = run(task, s)
                for h in range(2):
                    i = 88 + 26 * h + j
                    e, f, regime = frictionloss_qacc(md, xs[i], md.dof_invweight[h][j], fl, v)
                    assert regime == ("creep" if scale > 1 else "slip")
                    out.append((x[i], e, regime))
    return out


def test_frictionloss_single_row_known_answers(dp, ref):
    """a hinge with frictionloss under a constant (gravity) torque, below
    the threshold (regularised creep: qacc = (1 - d0) qacc_smooth at rest) and above it (slip:
    qacc = qacc_smooth - A frictionloss sign), at rest and moving (aref = -b v)."""
    def run(task, s):
        md, st, tc = dp.compile_task(song(dp, "twinkle"), task, canonical_actions=False)
        env = ref.OracleEnv(md, st, tc, 1)
        env.set_state(s)
        assert env.contacts(0) == []
        env.step(np.zeros((1, 45), np.float32))
        return env.get_state()["qacc_ws"][0]

    cases = frictionloss_cases(dp, run)
    assert {r for _, _, r in cases} == {"creep", "slip"}
    for got, exp, regime in cases:
        assert abs(got - exp) <= 1e-9 * max(1.0, abs(exp)), (got, exp, regime)
