"""The reference's task-level tests (piano_with_shadow_hands_test.py, shadow_hand_test.py,
piano_test.py) restated against the CPU oracle, plus physics sanity checks of the oracle
(mass matrix, gravity bias) - these pin the oracle before it is trusted as the checker."""
import ctypes as C

import numpy as np
import pytest

from helpers import random_states, song


def make(dp, ref, name="test_task", n=1, **kw):
    ct = kw.pop("control_timestep", 0.01 if name == "test_task" else 0.05)
    task = dp.TaskConfig(control_timestep=ct, **kw)
    seq = song(dp, name)
    md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
    return md, st, tc, ref.OracleEnv(md, st, tc, n)


def test_obs_keys_and_dims(dp, ref):
    for disable in (False, True):
        md, st, tc, env = make(dp, ref, disable_fingering_reward=disable, n_steps_lookahead=0)
        lay = dp.obs_layout(tc)
        assert ("fingering" in lay) == (not disable)
        for k in ("goal", "piano/state", "piano/sustain_state", "rh_shadow_hand/joints_pos",
                  "lh_shadow_hand/joints_pos"):
            assert k in lay
        assert env.obs_dim == max(s.stop for s in lay.values())


def test_obs_dim_benchmark_configs(dp, ref):
    _, _, tc, env = make(dp, ref, "twinkle")
    assert env.obs_dim == 329
    _, _, tc, env = make(dp, ref, "crossing_field", trim_silence=True)
    assert env.obs_dim == 319 and tc.fingering_reward == 0


def test_termination_and_discount(dp, ref):
    """piano_with_shadow_hands_test.py:119-136: T=4 -> three MID then LAST, discount 1."""
    md, st, tc, env = make(dp, ref)
    assert st.T == 4
    env.reset()
    zero = np.zeros((1, 45), np.float32)
    for _ in range(3):
        _, _, disc, stt = env.step(zero)
        assert stt[0] == 1 and disc[0] == 1.0
    _, _, disc, stt = env.step(zero)
    assert stt[0] == 2 and disc[0] == 1.0
    # auto-reset on the next step (dm_env): FIRST
    _, _, _, stt = env.step(zero)
    assert stt[0] == 0


@pytest.mark.parametrize("lookahead", [0, 1, 2, 5])
def test_goal_observable_lookahead(dp, ref, lookahead):
    """piano_with_shadow_hands_test.py:152-192."""
    md, st, tc, env = make(dp, ref, n_steps_lookahead=lookahead)
    lay = dp.obs_layout(tc)
    obs = env.reset()
    zero = np.zeros((1, 45), np.float32)
    T = st.T
    for i in range(T):
        expected = np.zeros((lookahead + 1, 89))
        for j, t in enumerate(range(i, min(i + lookahead + 1, T))):
            expected[j] = st.goal[t]
        np.testing.assert_array_equal(obs[0, lay["goal"]], expected.ravel())
        obs, _, _, _ = env.step(zero)


def test_fingering_observable(dp, ref):
    """piano_with_shadow_hands_test.py:194-226: rh = finger < 5, lh = finger - 5."""
    md, st, tc, env = make(dp, ref)
    lay = dp.obs_layout(tc)
    obs = env.reset()
    zero = np.zeros((1, 45), np.float32)
    for i in range(st.T):
        exp = np.zeros((2, 5))
        for n in range(st.count[i]):
            f = st.fingers[i, n]
            if f < 5:
                exp[0, f] = 1
            else:
                exp[1, f - 5] = 1
        np.testing.assert_array_equal(obs[0, lay["fingering"]], exp.ravel())
        obs, _, _, _ = env.step(zero)


def test_failure_termination(dp, ref):
    """piano_with_shadow_hands_test.py:228-242: qfrc_applied=3 on all keys -> LAST, discount 0."""
    md, st, tc, env = make(dp, ref, wrong_press_termination=True)
    env.reset()
    app = np.zeros((1, 140))
    app[0, :88] = 3.0
    env.set_applied(app)
    _, _, disc, stt = env.step(np.zeros((1, 45), np.float32))
    assert stt[0] == 2 and disc[0] == 0.0


def test_reward_terms_present(dp, ref):
    """piano_with_shadow_hands_test.py:259-272 + the OT term when the song has no fingering."""
    md, st, tc, env = make(dp, ref)
    env.reset()
    env.step(np.zeros((1, 45), np.float32))
    terms = env.reward_terms()[0]
    assert terms[0] == pytest.approx(0.5 * 2.4547089e-4 + 0.5, rel=1e-6)  # goal key not pressed
    assert terms[4] == 0.5  # no forearm collision
    _, _, tc2, env2 = make(dp, ref, "crossing_field", trim_silence=True)
    assert tc2.fingering_reward == 0
    env2.reset()
    env2.step(np.zeros((1, 45), np.float32))
    assert 0.0 <= env2.reward_terms()[0][3] <= 1.0


def test_model_counts_and_orders(dp):
    """shadow_hand_test.py:81-124, piano_test.py:35-64."""
    md = dp.model.build_model()
    assert dp.abi.HAND_NDOF == 24 + 2 and dp.abi.HAND_NACT == 20 + 2
    lo, hi = dp.model.action_spec(md)
    assert lo.shape == (45,) and (hi >= lo).all()
    # joints[0] is WRJ2 (the first Menagerie joint), forearm dofs appended last
    order = list(md.dof_obs_order[0])
    assert order[0] == 2 and order[-2:] == [0, 1]
    # fingertip site bodies: th, ff, mf, rf, lf distal
    assert len(set(md.site_body[0])) == 5
    # forearm_tx range spans the piano (tasks/base.py:160-164)
    np.testing.assert_allclose(list(md.dof_range[0][0]), [-0.6105 - 0.15, 0.6105 - 0.15], atol=1e-9)


def test_mass_matrix_and_gravity_bias(dp, ref):
    """Oracle dynamics vs finite differences of the potential energy and body COM
    kinematics (independent of the recursive algorithms)."""
    md, st, tc, env = make(dp, ref, "twinkle")
    L = ref.lib()
    L.ref_debug_dynamics.argtypes = [C.c_void_p, C.c_int, ref._f64p, ref._f64p]
    L.ref_debug_com.argtypes = [C.c_void_p, C.c_int, ref._f64p]
    env.reset()
    rng = np.random.RandomState(1)
    q, _ = random_states(md, 1, rng)
    s = env.get_state()
    s["qpos"][0] = q[0]
    s["qvel"][0] = 0
    env.set_state(s)
    M = np.zeros(140 * 140)
    b = np.zeros(140)
    L.ref_debug_dynamics(env._h, 0, M, b)
    M = M.reshape(140, 140)
    assert np.abs(M - M.T).max() == 0
    assert np.linalg.eigvalsh(M).min() > 0

    def coms(qq):
        s["qpos"][0] = qq
        env.set_state(s)
        c = np.zeros(150)
        L.ref_debug_com(env._h, 0, c)
        return c.reshape(2, 25, 3)

    def potential(qq):
        c = coms(qq)
        u = sum(md.body_mass[h][bb] * 9.81 * c[h, bb, 2] for h in range(2) for bb in range(25))
        for k in range(88):
            u += md.key_mass[k] * 9.81 * (md.key_pos[k][2] - md.key_half[k][0] * np.sin(qq[k]))
        return u

    eps = 1e-6
    g = np.array([(potential(q[0] + eps * e) - potential(q[0] - eps * e)) / (2 * eps) for e in np.eye(140)])
    np.testing.assert_allclose(b, g, atol=1e-7)
    # translational part of M from COM Jacobians; the remainder must be PSD
    J = np.zeros((2, 25, 3, 140))
    for i in range(88, 140):
        e = np.zeros(140)
        e[i] = eps
        J[..., i] = (coms(q[0] + e) - coms(q[0] - e)) / (2 * eps)
    Mt = sum(md.body_mass[h][bb] * J[h, bb].T @ J[h, bb] for h in range(2) for bb in range(25))
    assert np.linalg.eigvalsh(M[88:, 88:] - Mt[88:, 88:]).min() > -1e-7


def test_oracle_random_rollout_is_stable(dp, ref):
    md, st, tc, env = make(dp, ref, "twinkle", n=2)
    env.reset()
    lo, hi = dp.model.action_spec(md)
    rng = np.random.RandomState(12345)
    for _ in range(60):
        obs, rew, disc, stt = env.step(rng.uniform(lo, hi, (2, 45)).astype(np.float32))
    s = env.get_state()
    assert np.isfinite(s["qpos"]).all() and np.abs(s["qvel"]).max() < 200
    assert np.isfinite(rew).all()


def test_threaded_cpu_baseline_matches_serial(dp, ref):
    """bench.py's all-cores CPU baseline (OpenMP over envs) steps exactly the serial loop."""
    outs = []
    for threads in (1, 4):
        md, st, tc, env = make(dp, ref, "twinkle", n=12)
        env.reset()
        lo, hi = dp.model.action_spec(md)
        rng = np.random.RandomState(3)
        for _ in range(8):
            res = env.step(rng.uniform(lo, hi, (12, 45)).astype(np.float32), threads=threads)
        outs.append((res, env.get_state()))
    for a, b in zip(outs[0][0], outs[1][0]):
        np.testing.assert_array_equal(a, b)
    for k in outs[0][1]:
        np.testing.assert_array_equal(outs[0][1][k], outs[1][1][k])
