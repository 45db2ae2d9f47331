"""Task-layer cases on the GPU that round 1 left untested:

* the ot_fingering reward with 11-16 simultaneous goal keys (the kernel's transposed K > 10
  Hungarian) against the oracle; more than PS_MAX_NOTES goal keys is a ps_create error;
* Guren (config 4's song, fingering reward) at 4096 envs: duplicated action streams agree
  bitwise, 256 sampled envs match the oracle;
* config 1: one Twinkle env, 500 random steps (RandomState(12345), three auto-resets),
  teacher-forced against the oracle step by step;
* randomize_hand_positions: the GPU's draws are the oracle's bit for bit, and the shifted
  hands step alike;
* VectorizedPianoEnv returns observations / rewards a driver may keep across steps;
* diverged envs (NaN / |x| > 1e10 qpos or qvel): reset and flagged per env like MuJoCo's
  mj_checkPos / mj_checkVel, the same as the oracle; Environment raises PhysicsError.
"""
import numpy as np
import pytest

from helpers import Floor, assert_parity, song

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

KEYS = ("qpos", "qvel", "qacc_ws", "ctrl", "sustain", "t_idx", "last")


def _gs(g):
    return {k: v.cpu().numpy() for k, v in g.get_state().items()}


def chord_song(dp, sizes, dur=0.5):
    """A song of chords (no fingering -> ot_fingering reward): chord i has sizes[i] keys."""
    m = dp.music
    seq = m.NoteSequence(title="chords")
    t = 0.0
    for n in sizes:
        base = 40 + (int(t * 10) % 7)
        for j in range(n):
            seq.notes.append(m.Note(base + 2 * j, t, t + dur, 80, 0))
        t += dur
    seq.total_time = t
    return seq


def test_ot_reward_with_11_to_16_goal_keys(dp, ref):
    seq = chord_song(dp, [12, 16, 11, 14, 4])
    task = dp.TaskConfig()
    md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
    assert tc.fingering_reward == 0 and int((st.goal[:, :88] != 0).sum(1).max()) == 16
    n = 16
    g = dp.BatchedPianoEnv(n, seq, task, device="cuda:0", canonical_actions=False)
    o = ref.OracleEnv(md, st, tc, n)
    lo, hi = dp.model.action_spec(md)
    rng = np.random.RandomState(4)
    g.reset()
    o.reset()
    errs, ks = [], []
    for t in range(st.T - 1):
        a = rng.uniform(lo, hi, (n, 45)).astype(np.float32)
        o.set_state({k: v for k, v in _gs(g).items() if k in KEYS})
        g.step(torch.from_numpy(a).cuda())
        o.step(a)
        errs.append(np.abs(g.reward_terms().cpu().numpy()[:, 3] - o.reward_terms()[:, 3]))
        ks.append(int((st.goal[t, :88] != 0).sum()))
    assert max(ks) == 16 and any(10 < k < 16 for k in ks)
    e = np.concatenate(errs)
    assert np.percentile(e, 99) < 1e-3, e.max()


def test_more_goal_keys_than_supported_is_an_error(dp):
    seq = chord_song(dp, [4, 4])
    md, st, tc = dp.compile_task(seq, dp.TaskConfig(), canonical_actions=False)
    st.goal[1, 20:37] = 1.0  # 17 goal keys in one step (count stays as built)
    with pytest.raises(dp.PianosimError, match="goal keys"):
        dp.BatchedPianoEnv(2, st, dp.TaskConfig(), device="cuda:0")


def test_guren_at_4096_envs(dp, ref):
    N = 4096
    seq = song(dp, "guren")
    task = dp.TaskConfig(trim_silence=True)
    g = dp.BatchedPianoEnv(N, seq, task, device="cuda:0", canonical_actions=False)
    md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
    assert tc.fingering_reward == 1 and st.T == 287
    lo, hi = (torch.tensor(x, device="cuda:0", dtype=torch.float32) for x in dp.model.action_spec(md))
    gen = torch.Generator(device="cuda:0").manual_seed(8)
    g.reset()
    for _ in range(20):
        u = torch.rand(N // 2, 45, device="cuda:0", generator=gen)
        a = lo + torch.cat([u, u]) * (hi - lo)
        obs, rew, disc, stt = g.step(a)
    s = g.get_state()
    assert torch.isfinite(s["qpos"]).all() and torch.isfinite(rew).all()
    assert torch.equal(s["qpos"][: N // 2], s["qpos"][N // 2:]) and torch.equal(obs[: N // 2], obs[N // 2:])
    # 256 sampled envs, teacher-forced for 4 steps against the oracle (1024 env-steps)
    idx = np.arange(0, N, N // 256)
    o, o2 = ref.OracleEnv(md, st, tc, len(idx)), Floor(ref, md, st, tc, len(idx))
    prng = np.random.RandomState(6)
    lay = dp.obs_layout(tc)
    eqs, ers, fl = [], [], []
    for _ in range(4):
        sg = _gs(g)
        o.set_state({k: sg[k][idx] for k in KEYS})
        o2.set_state({k: sg[k][idx] for k in KEYS}, prng)
        a = lo + torch.rand(N, 45, device="cuda:0", generator=gen) * (hi - lo)
        og, rg, _, tg = g.step(a)
        oo, ro, _, to = o.step(a.cpu().numpy()[idx])
        o2.step(a.cpu().numpy()[idx])
        np.testing.assert_array_equal(tg.cpu().numpy()[idx], to)
        eqs.append(np.abs(g.get_state()["qpos"].cpu().numpy()[idx] - o.get_state()["qpos"]).max(axis=1))
        fl.append(o2.dev(o.get_state()["qpos"]))
        ers.append(np.abs(rg.cpu().numpy()[idx] - ro))
        np.testing.assert_array_equal(og.cpu().numpy()[idx][:, lay["fingering"]], oo[:, lay["fingering"]])
    eq, er = np.concatenate(eqs), np.concatenate(ers)
    assert_parity(eq, np.concatenate(fl), "guren, 4096 envs")
    assert np.percentile(er, 99) < 1e-3, er.max()


def test_config1_single_env_500_random_steps(dp, ref):
    """BASELINE config 1 (suite_test.py:22-56 style): RoboPianist-debug-TwinkleTwinkleLittleStar-v0,
    actions U[spec] from RandomState(12345), 500 steps = three auto-resets (T = 161)."""
    env = dp.load("RoboPianist-debug-TwinkleTwinkleLittleStar-v0", seed=12345)
    core = env.core
    md, st, tc = dp.compile_task(song(dp, "twinkle"), core.task, canonical_actions=False)
    o = ref.OracleEnv(md, st, tc, 1)
    lo, hi = dp.model.action_spec(md)
    spec = env.action_spec()
    rng = np.random.RandomState(12345)
    ts = env.reset()
    o.reset()
    assert ts.first()
    firsts, errs, rerr = 0, [], []
    for i in range(500):
        a = rng.uniform(spec.minimum, spec.maximum).astype(np.float32)
        a_spec = (lo + (a.astype(np.float64) + 1.0) * 0.5 * (hi - lo)).astype(np.float32)
        o.set_state({k: v for k, v in _gs(core).items() if k in KEYS})
        ts = env.step(a)
        _, ro, do, so = o.step(a_spec[None])
        assert int(ts.step_type) == int(so[0]), i
        if ts.first():
            firsts += 1
            assert ts.reward is None and ts.discount is None
        else:
            rerr.append(abs(ts.reward - float(ro[0])))
            assert ts.discount == float(do[0])
        errs.append(np.abs(_gs(core)["qpos"] - o.get_state()["qpos"]).max())
    assert firsts == 3
    errs, rerr = np.array(errs), np.array(rerr)
    assert np.median(errs) < 1e-5 and np.percentile(errs, 99) < 1e-4, (np.median(errs), np.percentile(errs, 99), errs.max())
    assert np.percentile(rerr, 99) < 1e-3, rerr.max()


def test_randomize_hand_positions_parity(dp, ref):
    n = 32
    seq = song(dp, "twinkle")
    task = dp.TaskConfig(randomize_hand_positions=True)
    md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
    g = dp.BatchedPianoEnv(n, seq, task, device="cuda:0", canonical_actions=False, seed=99)
    o = ref.OracleEnv(md, st, tc, n, seed=99)
    g.reset()
    o.reset()
    dg, eg = (x.cpu().numpy() for x in g.hand_offset())
    do, eo = o.hand_offset()
    np.testing.assert_array_equal(dg, do.astype(np.float32))  # bitwise: same Philox bits, same fma
    np.testing.assert_array_equal(eg, eo)
    assert np.abs(dg).max() > 0.01
    np.testing.assert_allclose(g.fingertips().cpu().numpy(), o.fingertips(), atol=2e-6)
    lo, hi = dp.model.action_spec(md)
    rng = np.random.RandomState(1)
    errs = []
    for _ in range(6):
        a = rng.uniform(lo, hi, (n, 45)).astype(np.float32)
        o.set_state({k: v for k, v in _gs(g).items() if k in KEYS})
        g.step(torch.from_numpy(a).cuda())
        o.step(a)
        errs.append(np.abs(_gs(g)["qpos"] - o.get_state()["qpos"]).max(axis=1))
    e = np.concatenate(errs)
    assert np.median(e) < 1e-5 and np.percentile(e, 99) < 1e-4, (np.median(e), np.percentile(e, 99), e.max())
    # an auto-reset draws the next episode's shift
    g.set_state({"t_idx": np.full(n, st.T - 1, np.int32)})
    g.step(torch.zeros(n, 45, device="cuda:0"))
    _, _, _, stt = g.step(torch.zeros(n, 45, device="cuda:0"))
    assert (stt.cpu().numpy() == 0).all()
    d2, e2 = (x.cpu().numpy() for x in g.hand_offset())
    assert (e2 == 2).all()
    exp = np.array([ref.hand_offset_draw(99, i, 1) for i in range(n)], np.float32)
    np.testing.assert_array_equal(d2, exp)


def test_sharded_handles_equal_one_handle_bitwise(dp):
    """SURVEY 8(e) on the kernel: a job of N envs on one handle equals the same job sharded over
    two handles (env_offset = 0 and N/2, as bench.py's ranks create them) bit for bit under
    randomize_hand_positions - the Philox draws are keyed by the global env id, and an env's
    step depends on nothing but its own row."""
    n = 64
    seq = song(dp, "twinkle")
    task = dp.TaskConfig(randomize_hand_positions=True)
    whole = dp.BatchedPianoEnv(n, seq, task, device="cuda:0", seed=21)
    halves = [dp.BatchedPianoEnv(n // 2, seq, task, device="cuda:0", seed=21, env_offset=off) for off in (0, n // 2)]
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    outs = [whole.reset()] + [h.reset() for h in halves]
    np.testing.assert_array_equal(outs[0].cpu().numpy(), torch.cat(outs[1:]).cpu().numpy())
    for t in range(40):
        a = torch.rand(n, 45, device="cuda:0", generator=gen) * 2 - 1
        if t == 20:  # episodes end at different steps: every env auto-resets into a new draw
            tt = (np.arange(n) % 7 + dp.compile_task(seq, task)[1].T - 7).astype(np.int32)
            whole.set_state({"t_idx": tt})
            for i, h in enumerate(halves):
                h.set_state({"t_idx": tt[i * n // 2:(i + 1) * n // 2]})
        rw = whole.step(a)
        rh = [h.step(a[i * n // 2:(i + 1) * n // 2]) for i, h in enumerate(halves)]
        for j in range(4):
            np.testing.assert_array_equal(rw[j].cpu().numpy(), torch.cat([r[j] for r in rh]).cpu().numpy())
    dw, ew = (x.cpu().numpy() for x in whole.hand_offset())
    dh = np.concatenate([x.hand_offset()[0].cpu().numpy() for x in halves])
    eh = np.concatenate([x.hand_offset()[1].cpu().numpy() for x in halves])
    np.testing.assert_array_equal(dw, dh)
    np.testing.assert_array_equal(ew, eh)
    assert (ew >= 2).any() and np.abs(dw).max() > 0.01
    sw = whole.get_state()
    sh = [h.get_state() for h in halves]
    for k in ("qpos", "qvel", "qacc_ws", "ctrl"):
        np.testing.assert_array_equal(sw[k].cpu().numpy(), torch.cat([x[k] for x in sh]).cpu().numpy())


def test_vectorized_env_outputs_survive_the_next_step(dp):
    env = dp.VectorizedPianoEnv(8, song(dp, "twinkle"))
    o0 = env.reset()
    keep0 = {k: v.clone() for k, v in o0.items()}
    a = torch.rand(8, 45, device="cuda:0") * 2 - 1
    o1, r1, d1 = env.step(a)
    keep1 = {k: v.clone() for k, v in o1.items()}
    r1c = r1.clone()
    o2, r2, d2 = env.step(torch.rand(8, 45, device="cuda:0") * 2 - 1)
    for k in o0:
        assert torch.equal(o0[k], keep0[k]) and torch.equal(o1[k], keep1[k])
    assert torch.equal(r1, r1c)
    assert not torch.equal(o1["piano/state"], o2["piano/state"]) or not torch.equal(r1, r2)


def test_non_finite_actions_do_not_stall_the_launch(dp):
    """A policy that emits NaN / inf actions poisons only its own envs: the launch completes
    (the OT assignment is bounded against non-finite costs - an unbounded Hungarian search on
    lane 0 would never return) and every other env steps exactly as it does without them."""
    N = 64
    task = dp.TaskConfig(trim_silence=True)  # Crossing Field: ot_fingering reward (Hungarian)
    a = torch.rand(4, N, 45, device="cuda:0", generator=torch.Generator(device="cuda:0").manual_seed(9)) * 2 - 1
    bad = a.clone()
    bad[:, :4] = float("nan")
    bad[:, 4:6] = float("inf")
    outs = []
    for acts in (a, bad):
        g = dp.BatchedPianoEnv(N, song(dp, "crossing_field"), task, device="cuda:0")
        g.reset()
        for t in range(4):
            obs, rew, disc, st = g.step(acts[t])
        torch.cuda.synchronize()
        outs.append((g.get_state()["qpos"].cpu().numpy(), obs.cpu().numpy(), rew.cpu().numpy()))
    (q0, o0, r0), (q1, o1, r1) = outs
    assert np.array_equal(q0[6:], q1[6:]) and np.array_equal(o0[6:], o1[6:]) and np.array_equal(r0[6:], r1[6:])


def _poison(s):
    """env 0: NaN hand joint, env 1: inf key angle, env 2: |qvel| > 1e10 (mj_checkPos / checkVel)."""
    s = {k: v.copy() for k, v in s.items()}
    s["qpos"][0, 100] = np.nan
    s["qpos"][1, 7] = np.inf
    s["qvel"][2, 120] = 3e10
    return s


def test_diverged_envs_reset_and_flagged(dp, ref):
    """MuJoCo resets a diverged env's data and raises a warning (mj_checkPos / mj_checkVel); the
    kernel does the same per env and counts it (ps_warnings), like the oracle; the other envs
    step bit-identically to an unpoisoned run, and the reset envs match the oracle's."""
    N = 16
    seq = song(dp, "crossing_field")
    task = dp.TaskConfig(trim_silence=True)
    md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
    lo, hi = dp.model.action_spec(md)
    rng = np.random.RandomState(4)
    acts = [rng.uniform(lo, hi, (N, 45)).astype(np.float32) for _ in range(5)]
    o = ref.OracleEnv(md, st, tc, N)
    o.reset()
    for a in acts[:3]:
        o.step(a)
    s0 = o.get_state()
    runs = []
    for poison in (False, True):
        g = dp.BatchedPianoEnv(N, seq, task, device="cuda:0", canonical_actions=False)
        g.reset()
        g.set_state(_poison(s0) if poison else s0)
        for a in acts[3:]:
            g.step(torch.from_numpy(a).cuda())
        runs.append((_gs(g), g.warnings().cpu().numpy()))
    (sc, wc), (sp, wp) = runs
    assert (wc == 0).all()
    exp = np.zeros((N, 3), np.int32)
    exp[0, 0] = exp[1, 0] = exp[2, 1] = 1
    np.testing.assert_array_equal(wp, exp)
    for k in ("qpos", "qvel"):
        assert np.isfinite(sp[k]).all()
        np.testing.assert_array_equal(sp[k][3:], sc[k][3:])
    o.set_state(_poison(s0))
    for a in acts[3:]:
        o.step(a)
    np.testing.assert_array_equal(o.warnings(), exp)
    e = np.abs(sp["qpos"][:3] - o.get_state()["qpos"][:3]).max()
    assert e < 1e-4, e


def test_environment_raises_physics_error(dp):
    """composer.Environment.step: a physics warning raises PhysicsError by default; with
    raise_exception_on_physics_error=False the step ends the episode (LAST, reward 0, discount
    0) and the next step resets (FIRST)."""
    for raise_ in (True, False):
        env = dp.envs.Environment(song(dp, "twinkle"), dp.TaskConfig(), raise_exception_on_physics_error=raise_)
        env.reset()
        a = np.zeros(45, np.float32)
        assert env.step(a).mid()
        q = env.core.get_state()["qvel"]
        q[0, 90] = float("nan")
        env.core.set_state({"qvel": q})
        if raise_:
            with pytest.raises(dp.PhysicsError, match="BADQVEL"):
                env.step(a)
        else:
            ts = env.step(a)
            assert ts.last() and ts.reward == 0.0 and ts.discount == 0.0
            assert env.step(a).first()
            assert env.step(a).mid()
