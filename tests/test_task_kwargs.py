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
