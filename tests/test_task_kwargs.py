"""PianoTask keyword arguments the reference forwards through PianoWithShadowHands' **kwargs
(piano_with_shadow_hands.py:65, tasks/base.py:96-107), on the CPU checker and the host model
compiler (the GPU side: tests/test_gpu_task_kwargs.py):

* gravity_compensation (tasks/base.py:185-186, mujoco_utils' compensate_gravity: gravcomp 1 on
  every hand body): with zero controls at qpos0 the hands feel no net force and stay exactly at
  rest, where without it they sag under gravity; the keys keep their gravity;
* attachment_yaw (tasks/base.py:174-181): the hand roots turned about world z by +yaw (right) and
  -yaw (left), so every fingertip at reset is the yaw-0 one rotated about its hand's root;
* primitive_fingertip_collisions (shadow_hand.py:95,144-152): palm boxes with capsule (True) or
  convex-hull (False, the reference's default) distal colliders; None keeps the authored
  all-capsule hand; exclusive with hand_xml.
"""
import math

import numpy as np
import pytest

from helpers import song


def _oracle(dp, ref, n=1, **kw):
    md, st, tc = dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(**kw), canonical_actions=False)
    return md, ref.OracleEnv(md, st, tc, n)


def test_gravity_compensation_holds_the_hands_at_rest(dp, ref):
    out = {}
    for gc in (False, True):
        md, o = _oracle(dp, ref, gravity_compensation=gc)
        assert md.hand_gravcomp == (1.0 if gc else 0.0)
        o.reset()
        for _ in range(5):
            o.step(np.zeros((1, 45), np.float32))  # ctrl 0 = every position target at qpos0
        out[gc] = o.get_state()["qpos"][0]
        assert o.contact_count()[0] == 0
    assert np.abs(out[True][88:]).max() == 0.0            # no net force on any hand dof
    assert np.abs(out[False][88:]).max() > 1e-3            # gravity pulls the hands down
    np.testing.assert_array_equal(out[True][:88], out[False][:88])  # keys: gravity unchanged


@pytest.mark.parametrize("yaw", [12.0, -30.0])
def test_attachment_yaw_turns_the_hands_about_their_roots(dp, ref, yaw):
    _, o0 = _oracle(dp, ref)
    _, o1 = _oracle(dp, ref, attachment_yaw=yaw)
    o0.reset()
    o1.reset()
    t0, t1 = o0.fingertips()[0], o1.fingertips()[0]  # [hand][finger][xyz], hand 0 = right
    for h, sign in ((0, 1.0), (1, -1.0)):
        root = np.array(dp.model.HAND_POSITIONS[h])
        a = math.radians(sign * yaw)
        Rz = np.array([[math.cos(a), -math.sin(a), 0.0], [math.sin(a), math.cos(a), 0.0], [0.0, 0.0, 1.0]])
        np.testing.assert_allclose(t1[h], (t0[h] - root) @ Rz.T + root, atol=1e-12)


def test_primitive_fingertip_collisions_selects_the_collider_kinds(dp):
    kinds = {}
    for flag in (None, True, False):
        md, _, _ = dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(primitive_fingertip_collisions=flag))
        kinds[flag] = [int(t) for t in md.xgeom_type[0]]
    box, hull = dp.abi.GEOM_BOX, dp.abi.GEOM_HULL
    assert not any(kinds[None])                                   # authored: capsules only
    assert kinds[True].count(box) == 3 and hull not in kinds[True]  # palm boxes, capsule tips
    assert kinds[False].count(box) == 3 and kinds[False].count(hull) == 5  # + 5 hull fingertips
    # the flag compiles the same model as the box / hull hand handed over as MJCF
    a, _, _ = dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(primitive_fingertip_collisions=False))
    b, _, _ = dp.compile_task(song(dp, "twinkle"),
                              dp.TaskConfig(hand_xml=dp.mjcf.hand_to_mjcf(dp.mjcf.box_hull_hand())))
    for f in ("xgeom_type", "xgeom_pos", "xgeom_quat", "hull_vert", "body_pos", "dof_axis", "n_xpairs"):
        np.testing.assert_allclose(np.asarray(getattr(a, f)), np.asarray(getattr(b, f)), atol=1e-9, err_msg=f)
    with pytest.raises(ValueError, match="exclusive"):
        dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(primitive_fingertip_collisions=True, hand_xml="x.xml"))


def test_reduced_action_space_spec_and_obs(dp):
    """shadow_hand_test.py:89-99: the reduced hand has NU + n_forearm - 3 actuators (19 a hand:
    A_THJ5, A_THJ1, A_LFJ5 removed), so the task's action is 2 x 19 + sustain; THJ2 and its
    actuator are narrowed to (0, 0.698132); joints_pos drops the three joints (23 a hand)."""
    full, _, tcf = dp.compile_task(song(dp, "twinkle"), dp.TaskConfig())
    md, _, tc = dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(reduced_action_space=True))
    lo, hi = dp.model.action_spec(md)
    assert len(lo) == 2 * (20 + 2 - 3) + 1 == dp.model.action_dim(md) == 39
    assert dp.abi.obs_dim(tc, md) == dp.abi.obs_dim(tcf, full) - 6
    lay = dp.obs_layout(tc, md)
    assert lay["rh_shadow_hand/joints_pos"].stop - lay["rh_shadow_hand/joints_pos"].start == 23
    hand = dp.model.authored_hand()
    names = [d.name for d in hand.dofs]
    for h in range(2):
        locked = {names[j] for j in range(26) if md.dof_locked[h][j]}
        assert locked == {"THJ5", "THJ1", "LFJ5"}
        kept = [names[md.dof_obs_order[h][i]] for i in range(md.n_obs_joints[h])]
        assert kept == [names[j] for j in hand.obs_order if names[j] not in locked]  # order kept
        j2 = names.index("THJ2")
        assert tuple(md.dof_range[h][j2]) == dp.model.REDUCED_THUMB_RANGE
    cols = dp.model.action_columns(md)
    acts = hand.acts
    for h, a, c in cols:
        kind, target = acts[a][0], acts[a][1]
        assert kind == 1 or names[target] not in ("THJ5", "THJ1", "LFJ5")
        if kind == 0 and names[target] == "THJ2":
            assert (lo[c], hi[c]) == dp.model.REDUCED_THUMB_RANGE
    assert sorted(c for _, _, c in cols) == list(range(38)) and (lo[-1], hi[-1]) == (0.0, 1.0)
    # the full layout is unchanged (n_action = 0: 45 columns)
    assert full.n_action == 0 and dp.model.action_dim(full) == 45


def test_forearm_dofs(dp):
    """forearm_dofs keeps a subset of the forearm slides (shadow_hand.py:270-311); the others
    lock. Unknown names raise (shadow_hand_test.py:78-80), as do the reference's forearm_tz /
    roll / pitch / yaw, which need more than this kernel's 26 dof slots per hand."""
    for fd, na in ((("forearm_tx",), 43), (("forearm_ty",), 43), ((), 41), (("forearm_tx", "forearm_ty"), 45)):
        md, _, _ = dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(forearm_dofs=fd))
        assert dp.model.action_dim(md) == na
        for h in range(2):
            assert [bool(md.dof_locked[h][j]) for j in range(2)] == [n not in fd for n in ("forearm_tx", "forearm_ty")]
    for bad in (("invalid",), ("forearm_roll",), ("forearm_ty", "forearm_tx")):
        with pytest.raises(ValueError, match="forearm_dofs"):
            dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(forearm_dofs=bad))


def test_locked_dofs_are_the_reference_hand_without_those_joints(dp, ref):
    """A removed joint (reduced_action_space) is a locked dof slot: the reduced model's mass
    matrix is the full one restricted to the kept dofs (MuJoCo's M of a body tree without the
    joint: its Jacobian column gone) with an identity row for the slot, the bias of the kept dofs
    is the same at the same state, the constraint regularisers use the reduced M's inverse
    (mj_setConst), and under random actions with contacts the slot never moves."""
    import ctypes as C
    from helpers import random_states
    full, st, tcf = dp.compile_task(song(dp, "crossing_field"), dp.TaskConfig(trim_silence=True), canonical_actions=False)
    red, st2, tcr = dp.compile_task(song(dp, "crossing_field"), dp.TaskConfig(trim_silence=True, reduced_action_space=True),
                                    canonical_actions=False)
    lk = [88 + 26 * h + j for h in range(2) for j in range(26) if red.dof_locked[h][j]]
    kept = [i for i in range(140) if i not in lk]
    L = ref.lib()
    L.ref_debug_dynamics.argtypes = [C.c_void_p, C.c_int, ref._f64p, ref._f64p]
    rng = np.random.RandomState(3)
    q, v = random_states(full, 1, rng)
    q[0, lk] = 0.0
    v[0, lk] = 0.0
    mats = []
    for md, s_, tc in ((full, st, tcf), (red, st2, tcr)):
        env = ref.OracleEnv(md, s_, tc, 1)
        env.reset()
        s = env.get_state()
        s["qpos"][0], s["qvel"][0] = q[0], v[0]
        env.set_state(s)
        M, b = np.zeros(140 * 140), np.zeros(140)
        L.ref_debug_dynamics(env._h, 0, M, b)
        mats.append((M.reshape(140, 140), b))
    (Mf, bf), (Mr, br) = mats
    np.testing.assert_allclose(Mr[np.ix_(kept, kept)], Mf[np.ix_(kept, kept)], rtol=0, atol=1e-15)
    np.testing.assert_array_equal(Mr[np.ix_(lk, lk)], np.eye(len(lk)))
    assert not Mr[np.ix_(lk, kept)].any()
    np.testing.assert_allclose(br[kept], bf[kept], rtol=0, atol=1e-12)
    # dof_invweight (mj_setConst at qpos0) = the diagonal of the reduced M's inverse
    env0 = ref.OracleEnv(full, st, tcf, 1)
    env0.reset()
    M0, b0 = np.zeros(140 * 140), np.zeros(140)
    L.ref_debug_dynamics(env0._h, 0, M0, b0)
    M0 = M0.reshape(140, 140)
    for h in range(2):
        keep_h = [j for j in range(26) if not red.dof_locked[h][j]]
        idx = [88 + 26 * h + j for j in keep_h]
        want = np.diag(np.linalg.inv(M0[np.ix_(idx, idx)]))
        np.testing.assert_allclose([red.dof_invweight[h][j] for j in keep_h], want, rtol=1e-9)
        assert not np.allclose([full.dof_invweight[h][j] for j in keep_h], want, rtol=1e-6)  # it differs
    env = ref.OracleEnv(red, st2, tcr, 8)
    env.reset()
    lo, hi = dp.model.action_spec(red)
    ncon = 0
    for _ in range(30):
        env.step(rng.uniform(lo, hi, (8, len(lo))).astype(np.float32))
        ncon += int(env.contact_count().sum())
    qq = env.get_state()["qpos"]
    assert ncon > 0 and np.abs(qq[:, lk]).max() == 0.0 and np.abs(qq[:, kept[88:]]).max() > 0.1
