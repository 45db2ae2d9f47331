"""The constraint solve and the caps, on the oracle (CPU).

* The specification's exact dual solve (warm-up PGS + block principal pivoting) equals PGS run
  to convergence from a cold start - an independent method for the same unique solution (the
  one MuJoCo's solvers converge to) - on random-action states of the benchmark song.
* Round 1's truncated solver (20 cold-start PGS sweeps) is measurably NOT that solution.
* The contact cap never binds in a random-action rollout, the coupled-row cap only rarely.
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


def test_round1_pgs20_is_not_converged(dp, ref):
    """The study behind the solver change (profiles/r02_solver_study.json): 20 cold-start PGS
    sweeps leave a one-control-step qpos gap far above the fp32 parity tolerance."""
    md, st, tc, env = _env(dp, ref, 16)
    _, _, tc_pgs, env_pgs = _env(dp, ref, 16, constraint_solver="pgs")
    assert tc.solver == 1 and tc_pgs.solver == 0 and tc_pgs.pgs_iterations == 20
    rng = np.random.RandomState(3)
    lo, hi = _rollout(ref, env, md, 12, rng)
    s = env.get_state()
    env_pgs.set_state(s)
    a = rng.uniform(lo, hi, (16, 45)).astype(np.float32)
    env.step(a)
    env_pgs.step(a)
    gap = np.abs(env.get_state()["qpos"] - env_pgs.get_state()["qpos"]).max()
    assert gap > 1e-4, gap


def test_caps_rarely_bind_in_random_rollouts(dp, ref):
    """The contact cap (20) never binds; the coupled-row cap (64 = one row per lane) binds in
    ~1e-4 of the substeps under uniform random actions, where position targets at the joint
    ranges push many hand joints past their limits at once (profiles/r02_solver_study.json
    has the rates over longer rollouts)."""
    md, st, tc, env = _env(dp, ref, 16)
    ref.stats_reset()
    _rollout(ref, env, md, 40, np.random.RandomState(5))
    s = ref.stats()
    assert s["substeps"] == 16 * 40 * 10
    assert s["contact_cap_substeps"] == 0
    assert s["row_cap_substeps"] <= 2e-3 * s["substeps"]
    assert s["pdas"][63] == 0  # the exact solve never hit its iteration cap
    found = s["found"]
    assert np.nonzero(found)[0].max() < tc.max_contacts


def test_exact_solver_needs_no_sweeps(dp, ref):
    """The warm-up only picks the start set: with 0 or 8 sweeps the solution is the same."""
    md, st, tc0, env0 = _env(dp, ref, 8, pgs_iterations=0)
    _, _, tc8, env8 = _env(dp, ref, 8, pgs_iterations=8)
    rng = np.random.RandomState(9)
    lo, hi = _rollout(ref, env8, md, 10, rng)
    env0.set_state(env8.get_state())
    a = rng.uniform(lo, hi, (8, 45)).astype(np.float32)
    env0.step(a)
    env8.step(a)
    assert np.abs(env0.get_state()["qpos"] - env8.get_state()["qpos"]).max() < 1e-9


# ------------------------------------------------------------------ randomize_hand_positions
def test_hand_offset_draws(ref):
    d = np.array([[ref.hand_offset_draw(7, e, ep) for ep in range(64)] for e in range(64)])
    assert (d >= -0.05).all() and (d < 0.05).all()
    assert abs(d.mean()) < 0.005 and abs(d.std() - 0.1 / np.sqrt(12)) < 0.003  # U(-0.05, 0.05)
    assert ref.hand_offset_draw(7, 3, 5) == d[3, 5]  # a pure function of (seed, env, episode)
    assert ref.hand_offset_draw(8, 3, 5) != d[3, 5]
    assert len(np.unique(d)) >= d.size - 4  # 24-bit draws: a few birthday collisions at most


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
