"""The constraint solve and the caps, on the oracle (CPU).

* The specification's primal Newton solve (MuJoCo's default solver, with friction-loss rows and
  no row cap) equals the dual problem solved by projected Gauss-Seidel run to convergence from a
  cold start (friction-loss forces boxed to +-frictionloss) - an independent method for the same
  unique solution - on random-action states of the benchmark song.
* Newton converges in every substep; the contact cap never binds; rows are uncapped.
* randomize_hand_positions: the counter-based U(-0.05, 0.05) draws and the hand shift.
"""
import numpy as np
import pytest

from helpers import song

KEYS = ("qpos", "qvel", "qacc_ws", "ctrl", "sustain", "t_idx", "last")


def _env(dp, ref, n, name="crossing_field", seed=0, **kw):
    kw.setdefault("trim_silence", name != "twinkle")
    md, st, tc = dp.compile_task(song(dp, name), dp.TaskConfig(**kw), canonical_actions=False)
    return md, st, tc, ref.OracleEnv(md, st, tc, n, seed=seed)


def _rollout(ref, env, md, steps, rng):
    lo, hi = [np.asarray(x) for x in __import__("importlib").import_module(
        "diffusion-piano_amd").model.action_spec(md)]
    env.reset()
    for _ in range(steps):
        env.step(rng.uniform(lo, hi, (env.n, 45)).astype(np.float32))
    return lo, hi


def test_exact_solve_is_the_converged_solution(dp, ref):
    md, st, tc, env = _env(dp, ref, 16)
    rng = np.random.RandomState(3)
    lo, hi = _rollout(ref, env, md, 12, rng)
    gaps = []
    try:
        for _ in range(4):
            s = env.get_state()
            a = rng.uniform(lo, hi, (16, 45)).astype(np.float32)
            env.step(a)
            q_exact = env.get_state()["qpos"]
            env.set_state(s)
            ref.set_solver(1, 1e-13, 200000)  # converged PGS
            env.step(a)
            ref.set_solver(0)
            gaps.append(np.abs(env.get_state()["qpos"] - q_exact).max())
    finally:
        ref.set_solver(0)
    assert max(gaps) < 1e-9, gaps


def test_pgs_solver_is_retired(dp):
    with pytest.raises(ValueError, match="retired"):
        dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(constraint_solver="pgs"))
    _, _, tc = dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(constraint_solver="exact"))
    assert tc.solver == 1 and tc.solver_iterations == 0 and tc.solver_refine == 1


def test_solver_refine_option(dp):
    """TaskConfig.solver_refine reaches ps_task_cfg.solver_refine (0 none, 1 coupled substeps,
    2 every substep); other values raise (ps_create rejects them too)."""
    for r in (0, 1, 2):
        _, _, tc = dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(solver_refine=r))
        assert tc.solver_refine == r
    with pytest.raises(ValueError, match="solver_refine"):
        dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(solver_refine=3))


def test_newton_converges_and_no_row_cap(dp, ref):
    """The Newton solve converges in every substep of a random-action rollout (never at its
    iteration cap); the contact cap (20) does not bind; constraint rows are not capped - the
    52 friction-loss rows alone are most of round 2's 64-row cap; with key limits and contacts the
    substeps carry up to ~200 rows."""
    md, st, tc, env = _env(dp, ref, 16)
    ref.stats_reset()
    _rollout(ref, env, md, 40, np.random.RandomState(5))
    s = ref.stats()
    assert s["substeps"] == 16 * 40 * 10
    assert s["contact_cap_substeps"] == 0
    assert s["newton"][63] == 0
    assert s["newton"][:63].sum() == s["substeps"]
    assert s["iterations"] / s["substeps"] < 8
    rows = np.nonzero(s["rows"])[0]
    assert rows.min() >= 52 and rows.max() > 150  # 52 friction rows always, + limits + contacts
    found = s["found"]
    assert np.nonzero(found)[0].max() < tc.max_contacts
    assert s["warnings"] == 0


def test_frictionloss_rows_act(dp, ref):
    """With the Menagerie frictionloss the dynamics differ measurably from frictionloss 0 (the
    rows are in the solve), and a zero frictionloss model equals the solve without those rows."""
    md, st, tc, env = _env(dp, ref, 4)
    md0, _, _ = dp.compile_task(song(dp, "crossing_field"), dp.TaskConfig(trim_silence=True), canonical_actions=False)
    np.ctypeslib.as_array(md0.dof_frictionloss)[:] = 0.0
    env0 = ref.OracleEnv(md0, st, tc, 4)
    rng = np.random.RandomState(2)
    lo, hi = _rollout(ref, env, md, 6, rng)
    env0.set_state(env.get_state())
    a = rng.uniform(lo, hi, (4, 45)).astype(np.float32)
    env.step(a)
    env0.step(a)
    gap = np.abs(env.get_state()["qvel"] - env0.get_state()["qvel"]).max()
    assert gap > 1e-3, gap


# ------------------------------------------------------------------ randomize_hand_positions
def test_hand_offset_draws(ref):
    d = np.array([[ref.hand_offset_draw(7, e, ep) for ep in range(64)] for e in range(64)])
    assert (d >= -0.05).all() and (d < 0.05).all()
    assert abs(d.mean()) < 0.005 and abs(d.std() - 0.1 / np.sqrt(12)) < 0.003  # U(-0.05, 0.05)
    assert ref.hand_offset_draw(7, 3, 5) == d[3, 5]  # a pure function of (seed, env, episode)
    assert ref.hand_offset_draw(8, 3, 5) != d[3, 5]
    assert len(np.unique(d)) >= d.size - 4  # 24-bit draws: a few birthday collisions at most


def test_hand_offsets_keyed_by_global_env(dp, ref):
    """draws keyed by global env id - env g gets the same hand offset whether the job
    runs on one handle (world 1) or is sharded over two (env_offset = shard start)."""
    seq = song(dp, "twinkle")
    md, st, tc = dp.compile_task(seq, dp.TaskConfig(randomize_hand_positions=True), canonical_actions=False)
    whole = ref.OracleEnv(md, st, tc, 6, seed=5)
    halves = [ref.OracleEnv(md, st, tc, 3, seed=5, env_offset=off) for off in (0, 3)]
    for e in (whole, *halves):
        e.reset()
        e.reset()  # second episode
    dy = whole.hand_offset()[0]
    np.testing.assert_array_equal(np.concatenate([h.hand_offset()[0] for h in halves]), dy)
    np.testing.assert_array_equal(dy.astype(np.float32),
                                  np.array([ref.hand_offset_draw(5, g, 1) for g in range(6)], np.float32))


def test_randomized_reset_shifts_both_hands(dp, ref):
    md, st, tc, env = _env(dp, ref, 4, name="twinkle", seed=11, randomize_hand_positions=True)
    _, _, _, base = _env(dp, ref, 4, name="twinkle", seed=11)
    env.reset()
    base.reset()
    dy, ep = env.hand_offset()
    assert (ep == 1).all()
    exp = np.array([ref.hand_offset_draw(11, e, 0) for e in range(4)], np.float32)
    np.testing.assert_array_equal(dy.astype(np.float32), exp)
    tips, tips0 = env.fingertips(), base.fingertips()
    np.testing.assert_allclose(tips[..., 1] - tips0[..., 1], np.broadcast_to(dy[:, None, None], (4, 2, 5)),
                               atol=1e-12)
    np.testing.assert_allclose(tips[..., [0, 2]], tips0[..., [0, 2]], atol=1e-12)
    env.reset()  # the next episode draws again
    dy2, ep2 = env.hand_offset()
    assert (ep2 == 2).all() and not np.array_equal(dy2, dy)
    bdy, _ = base.hand_offset()
    assert (bdy == 0).all()
