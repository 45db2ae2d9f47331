"""The Newton constraint solve on the GPU against the oracle's (friction-loss rows, uncapped
rows, hands coupled through hand-hand contacts), the solver counters, and bitwise repeatability
of contacts sharing a key.

Tolerances (fp32 kernel vs fp64 oracle, same state and action, one control step):
helpers.assert_parity - qpos median < 1e-5, p99 < 1e-4 over the well-conditioned env-steps
(the checker's own 1e-7 rad sensitivity below 1e-5), and p99 over all within max(1e-4, 2x that
sensitivity's p99) - on the bench song, the replays of coupled-hand and heavy-contact env-steps
(the stiffest Hessians, fp32 LDL') and the whole-C-block states."""
import numpy as np
import pytest

from helpers import PARITY_MAX_CEIL, PARITY_P99_CEIL, PARITY_P99_CEIL_UNREFINED, Floor, assert_parity, song

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

KEYS = ("qpos", "qvel", "qacc_ws", "ctrl", "sustain", "t_idx", "last")


def _pair(dp, ref, name, n, **kw):
    kw.setdefault("trim_silence", name != "twinkle")
    task = dp.TaskConfig(**kw)
    seq = song(dp, name)
    md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
    return md, dp.BatchedPianoEnv(n, seq, task, device="cuda:0", canonical_actions=False), ref.OracleEnv(md, st, tc, n)


def _teacher_forced(md, g, o, o2, steps, rng, warm=6):
    """-> (qpos error, checker sensitivity) per env-step; o2 steps from the perturbed state."""
    lo, hi = dp_action_spec(md)
    prng = np.random.RandomState(1)
    o.reset()
    for _ in range(warm):
        o.step(rng.uniform(lo, hi, (o.n, 45)).astype(np.float32))
    s = o.get_state()
    g.set_state({k: s[k] for k in KEYS})
    errs, floor = [], []
    for _ in range(steps):
        a = rng.uniform(lo, hi, (o.n, 45)).astype(np.float32)
        sg = {k: v.cpu().numpy() for k, v in g.get_state().items()}
        o.set_state({k: sg[k] for k in KEYS})
        o2.set_state({k: sg[k] for k in KEYS}, prng)
        g.step(torch.from_numpy(a).cuda())
        o.step(a)
        o2.step(a)
        qo = o.get_state()["qpos"]
        errs.append(np.abs(g.get_state()["qpos"].cpu().numpy() - qo).max(axis=1))
        floor.append(o2.dev(qo))
    return np.concatenate(errs), np.concatenate(floor)


def dp_action_spec(md):
    import importlib
    return importlib.import_module("diffusion-piano_amd").model.action_spec(md)


def test_exact_solver_teacher_forced_bench_song(dp, ref):
    md, g, o = _pair(dp, ref, "crossing_field", 64)
    o2 = Floor(ref, *dp.compile_task(song(dp, "crossing_field"), dp.TaskConfig(trim_silence=True),
                                     canonical_actions=False), 64)
    e, f = _teacher_forced(md, g, o, o2, 16, np.random.RandomState(21))
    assert_parity(e, f, "bench song")


def test_solver_stats_and_caps(dp):
    """Counters of the bench workload: Newton iterations per substep (~4-5: the oracle's mean
    from a cold start is 4.7), never the iteration cap, no non-positive pivot, the contact cap
    (~1e-6 of the substeps) almost never binding; ~40% of the substeps couple the hands."""
    N = 4096
    g = dp.BatchedPianoEnv(N, song(dp, "crossing_field"), dp.TaskConfig(trim_silence=True), device="cuda:0")
    g.reset()
    gen = torch.Generator(device="cuda:0").manual_seed(5)
    st = []
    for _ in range(15):
        g.step(torch.rand(N, 45, device="cuda:0", generator=gen) * 2 - 1)
        st.append(g.solver_stats().cpu().numpy())
    st = np.stack(st)
    it = st[..., 0] / 10.0
    subs = st[..., 0].size * 10
    print(f"Newton iterations/substep {it.mean():.2f}, cap {st[..., 2].sum()}, coupled {st[..., 4].sum() / subs:.3f}, "
          f"bad pivots {st[..., 5].sum()}, max rows {st[..., 3].max()}")
    assert 1.0 < it.mean() < 10.0, it.mean()
    assert st[..., 1].sum() <= 1e-4 * subs  # narrow phase found >= max_contacts (20) contacts
    assert st[..., 2].sum() <= 1e-4 * subs  # Newton iteration cap
    assert st[..., 5].sum() == 0            # non-positive pivots
    assert 0.1 < st[..., 4].sum() / subs < 0.9
    assert st[..., 3].max() <= 96


def _replay(dp, ref, select, steps=14, N=2048, seed=7, **kw):
    """Roll N GPU envs; replay on the oracle the env-steps `select(stats, state)` picks (kw: more
    TaskConfig options of the GPU env)."""
    md, g, _ = _pair(dp, ref, "crossing_field", N, **kw)
    lo, hi = dp_action_spec(md)
    rng = np.random.RandomState(seed)
    g.reset()
    states, acts, outs = [], [], []
    for _ in range(steps):
        s0 = {k: v.cpu().numpy() for k, v in g.get_state().items()}
        a = rng.uniform(lo, hi, (N, 45)).astype(np.float32)
        g.step(torch.from_numpy(a).cuda())
        pick = np.nonzero(select(g.solver_stats().cpu().numpy()) & (s0["last"] == 0))[0][:64]
        if len(pick):
            q1 = g.get_state()["qpos"].cpu().numpy()
            states.append({k: s0[k][pick] for k in KEYS})
            acts.append(a[pick])
            outs.append(q1[pick])
    n = sum(len(x) for x in acts)
    st = {k: np.concatenate([s[k] for s in states]) for k in KEYS} if n else None
    if not n:
        return n, None, None
    seq = song(dp, "crossing_field")
    _, sttab, tc = dp.compile_task(seq, dp.TaskConfig(trim_silence=True), canonical_actions=False)
    o, o2 = ref.OracleEnv(md, sttab, tc, n), Floor(ref, md, sttab, tc, n)
    o.set_state(st)
    o2.set_state(st, np.random.RandomState(seed))
    acts = np.concatenate(acts)
    o.step(acts)
    o2.step(acts)
    qo = o.get_state()["qpos"]
    return n, np.abs(np.concatenate(outs) - qo).max(axis=1), o2.dev(qo)


def test_newton_heavy_states(dp, ref):
    """States with 10+ contacts in a substep (40+ contact rows besides the 52 friction-loss rows:
    round 2 dropped rows past 64) replayed on the oracle."""
    n, e, f = _replay(dp, ref, lambda st: st[:, 3] > 40)
    assert n >= 4, f"only {n} heavy env-steps"
    assert_parity(e, f, "heavy env-steps")


def test_newton_coupled_hands(dp, ref):
    """Env-steps whose every substep coupled the hands (hand-hand contact: the C-block
    elimination after both hands' independent pivots) replayed on the oracle."""
    n, e, f = _replay(dp, ref, lambda st: st[:, 4] >= 10)
    assert n >= 16, f"only {n} coupled env-steps"
    assert_parity(e, f, "coupled env-steps")


def test_unrefined_solve_coupled_hands(dp, ref):
    """TaskConfig(solver_refine=0), the option without the refining Newton step (the default,
    1, adds one in the converged piece on coupled substeps): the coupled replays keep round 5's
    all-sample ceiling 2e-4 (measured 1.6e-4; refined ~8e-5)."""
    n, e, f = _replay(dp, ref, lambda st: st[:, 4] >= 10, solver_refine=0)
    assert n >= 16, f"only {n} coupled env-steps"
    assert_parity(e, f, "coupled env-steps, solver_refine=0", p99_ceil=PARITY_P99_CEIL_UNREFINED)


def test_solver_refine_heavy_states(dp, ref):
    """The same on the heavy-contact replays with every substep refined (solver_refine=2)."""
    n, e, f = _replay(dp, ref, lambda st: st[:, 3] > 40, solver_refine=2)
    assert n >= 4, f"only {n} heavy env-steps"
    assert_parity(e, f, "heavy env-steps, solver_refine=2", p99_ceil=1e-4)


def test_newton_coupled_hands_full_block(dp, ref, monkeypatch):
    """The same on the 28-column C block (taken when a hand has more than 16 C dofs; forced here
    for every coupled substep by the test hook). Held at round 5's all-sample ceiling: the forced
    wide template refines less well than the fitted ones (measured p99 1.0e-4 unrefined, 1.4e-4
    refined, against the checker's floor p99 1.8e-4)."""
    monkeypatch.setenv("PIANOSIM_DEBUG_FULL_COUPLED", "1")
    n, e, f = _replay(dp, ref, lambda st: st[:, 4] >= 10, steps=8)
    assert n >= 8, f"only {n} coupled env-steps"
    assert_parity(e, f, "coupled env-steps, whole C block", p99_ceil=PARITY_P99_CEIL_UNREFINED)


def _overlap_states(md, rng):
    """The right hand slid along the keyboard (forearm_tx) and raised (forearm_ty) onto the left
    one, every position actuator held at its joint: hand-hand contacts across many fingers
    couple more than 28 dofs of both hands. -> (state dict, actions)."""
    lo, hi = dp_action_spec(md)
    # side by side (forearm_tx), and the right hand raised (forearm_ty) over the left one: flat
    # hands stacked at the height where they touch along the fingers
    grid = [(tx, ty) for tx in np.linspace(-0.30, -0.12, 37) for ty in (0.0, 0.02, 0.04, 0.06)]
    grid += [(tx, ty) for tx in np.linspace(-0.32, -0.28, 5) for ty in np.linspace(0.0, 0.06, 61)]
    per = 4
    N = per * len(grid)
    q = np.zeros((N, 140))
    q[:, 88:] = rng.normal(0.0, 0.02, (N, 52))
    for h in range(2):  # inside the joint ranges
        for j in range(26):
            lo_j, hi_j = md.dof_range[h][j]
            q[:, 88 + 26 * h + j] = np.clip(q[:, 88 + 26 * h + j], lo_j, hi_j)
    q[:, 88] = np.repeat([g[0] for g in grid], per)      # rh forearm_tx (qpos: 88 keys, rh 26, lh 26)
    q[:, 89] = np.repeat([g[1] for g in grid], per)      # rh forearm_ty
    q[:, 88 + 26] = 0.0
    q[:, 89 + 26] = 0.0
    # actions hold every position actuator at its joint (tendon actuators: the two-joint sum)
    a = np.zeros((N, 45), np.float32)
    for h in range(2):
        for u in range(22):
            kind, tgt = int(md.act_kind[h][u]), int(md.act_target[h][u])
            val = q[:, 88 + 26 * h + tgt] if kind == 0 else sum(
                md.tendon_coef[h][tgt][k] * q[:, 88 + 26 * h + md.tendon_dof[h][tgt][k]] for k in range(2))
            a[:, 22 * h + u] = np.clip(val, lo[22 * h + u], hi[22 * h + u])
    st = {"qpos": q.astype(np.float32), "qvel": np.zeros((N, 140), np.float32),
          "qacc_ws": np.zeros((N, 140), np.float32), "ctrl": np.zeros((N, 44), np.float32),
          "sustain": np.zeros(N, np.float32), "t_idx": np.full(N, 5, np.int32), "last": np.zeros(N, np.uint8)}
    return st, a


def test_newton_whole_c_block_overlapping_hands(dp, ref):
    """The right hand slid along the keyboard (forearm_tx) and raised (forearm_ty) onto the left
    one: hand-hand contacts across many fingers couple more than 28 dofs of both hands
    (PS_STAT_MAX_CDOFS), which the 16-column C block cannot hold, so the whole-block solve (both
    hands' C blocks in slot layout) runs. Overlapping hands are mostly violent (explosive contact
    forces: the checker itself moves by ~1e-2 under a 1e-7 rad perturbation of the joints), so
    the GPU is held to the checker's own sensitivity there (median within the sensitivity's
    median, p99 within 2x its p99), and to the parity gate (median < 1e-5, p99 < 1e-4) on the
    states whose sensitivity is below 1e-5; one control step from the same state."""
    seq = song(dp, "crossing_field")
    task = dp.TaskConfig(trim_silence=True)
    md, sttab, tc = dp.compile_task(seq, task, canonical_actions=False)
    rng = np.random.RandomState(11)
    st, a = _overlap_states(md, rng)
    N = len(a)
    g = dp.BatchedPianoEnv(N, seq, task, device="cuda:0", canonical_actions=False)
    g.set_state(st)
    g.step(torch.from_numpy(a).cuda())
    stats = g.solver_stats().cpu().numpy()
    warn = g.warnings().cpu().numpy()
    big = np.nonzero((stats[:, 6] > 28) & (stats[:, 1] == 0) & (warn.sum(1) == 0))[0]
    print(f"max coupled dofs {stats[:, 6].max()}, env-steps above 28 without the contact cap: {len(big)} of {N}")
    assert len(big) >= 8, f"only {len(big)} env-steps with more than 28 coupled dofs"
    sub = {k: x[big] for k, x in st.items()}
    o, o2 = ref.OracleEnv(md, sttab, tc, len(big)), Floor(ref, md, sttab, tc, len(big))
    o.set_state(sub)
    o2.set_state(sub, rng)
    o.step(a[big])
    o2.step(a[big])
    qo = o.get_state()["qpos"]
    floor = o2.dev(qo)
    e = np.abs(g.get_state()["qpos"].cpu().numpy()[big] - qo).max(axis=1)
    calm = floor < 1e-5
    print(f"{calm.sum()} calm of {len(big)}; qpos err median {np.median(e):.2e} p99 {np.percentile(e, 99):.2e} "
          f"max {e.max():.2e}, the checker's sensitivity median {np.median(floor):.2e} p99 {np.percentile(floor, 99):.2e}")
    # measured (r05): median 9.2e-6, p99 7.2e-4, max 7.7e-4 against the checker's own sensitivity
    # median 9.2e-3 / p99 6.5e-2: absolute gates at ~2x the measured values (a gate
    # relative to that sensitivity alone would let a 1000x regression of this path pass)
    assert np.median(e) < 2e-5, (np.median(e), np.median(floor))
    assert np.percentile(e, 99) < 2e-3 and e.max() < PARITY_MAX_CEIL, (np.percentile(e, 99), e.max())
    if calm.any():
        ec = e[calm]
        assert np.median(ec) < 1e-5 and np.percentile(ec, 99) < 1e-4, (np.median(ec), np.percentile(ec, 99), ec.max())


def _one_substep(dp, ref, st, a, select, **kw):
    """One physics substep (control_timestep = the physics timestep) from the same states on the
    GPU and the checker, on the states whose GPU solver counters `select` picks (no physics
    warning). -> (GPU counters of the picked states, qpos L-inf error, qacc L-inf error relative
    to the checker's largest |qacc|, at least 1)."""
    seq = song(dp, "crossing_field")
    task = dp.TaskConfig(trim_silence=True, control_timestep=0.005, **kw)
    md, sttab, tc = dp.compile_task(seq, task, canonical_actions=False)
    assert md.n_substeps == 1
    N = len(a)
    g = dp.BatchedPianoEnv(N, seq, task, device="cuda:0", canonical_actions=False)
    g.set_state(st)
    g.step(torch.from_numpy(a).cuda())
    stats = g.solver_stats().cpu().numpy()
    warn = g.warnings().cpu().numpy()
    pick = np.nonzero(select(stats) & (warn.sum(1) == 0))[0]
    if not len(pick):
        return stats[pick], np.zeros(0), np.zeros(0)
    sub = {k: np.asarray(x)[pick] for k, x in st.items()}
    o = ref.OracleEnv(md, sttab, tc, len(pick))
    o.set_state(sub)
    o.step(a[pick])
    so = o.get_state()
    sg = {k: v.cpu().numpy()[pick] for k, v in g.get_state().items()}
    eq = np.abs(sg["qpos"] - so["qpos"]).max(axis=1)
    v0 = np.asarray(sub["qvel"], np.float64)
    h = float(md.timestep)
    acc_o, acc_g = (so["qvel"] - v0) / h, (sg["qvel"].astype(np.float64) - v0) / h
    ea = np.abs(acc_g - acc_o).max(axis=1) / np.maximum(np.abs(acc_o).max(axis=1), 1.0)
    return stats[pick], eq, ea


def test_one_substep_whole_c_block(dp, ref):
    """the whole-C-block template (more than 28 coupled dofs of both hands) held to
    the one-substep gate - one substep is far better conditioned than a control step (no 10-fold
    compounding through the soft contacts), so the fp32 solve is measured, not the chaos. These
    are violent states (overlapping hands: |qacc| up to ~1e4), so the gate is on qacc relative to
    its largest magnitude: median < 5e-5, p99 < 5e-4 (measured r05: 1.3e-5 / 1.05e-4); qpos median
    < 5e-6, p99 < 5e-5 (2.4e-6 / 3.6e-5). The GPU counters must show the path: more than 28
    coupled dofs."""
    md = dp.compile_task(song(dp, "crossing_field"), dp.TaskConfig(trim_silence=True), canonical_actions=False)[0]
    st, a = _overlap_states(md, np.random.RandomState(11))
    stats, eq, ea = _one_substep(dp, ref, st, a, lambda s: (s[:, 6] > 28) & (s[:, 1] == 0))
    msg = (f"{len(eq)} states, coupled dofs max {stats[:, 6].max() if len(eq) else 0}: qpos err median "
           f"{np.median(eq):.2e} p99 {np.percentile(eq, 99):.2e} max {eq.max():.2e}; qacc rel err median "
           f"{np.median(ea):.2e} p99 {np.percentile(ea, 99):.2e} max {ea.max():.2e}")
    print(msg)
    assert len(eq) >= 8 and stats[:, 6].max() > 28, msg
    assert np.median(eq) < 5e-6 and np.percentile(eq, 99) < 5e-5, msg
    assert np.median(ea) < 5e-5 and np.percentile(ea, 99) < 5e-4, msg


def _contact_rich_states(dp, ref, n=4096, seed=7):
    """Random hand poses pushed toward flexion (the upper 40% of every joint range), one control
    step of the checker to settle the initial penetrations (max_contacts 24). -> (state, actions)."""
    from helpers import random_states
    task = dict(trim_silence=True, max_contacts=24)
    md, st, tc = dp.compile_task(song(dp, "crossing_field"), dp.TaskConfig(**task), canonical_actions=False)
    rng = np.random.RandomState(seed)
    o = ref.OracleEnv(md, st, tc, n)
    o.reset()
    s0 = o.get_state()
    q, v = random_states(md, n, rng)
    lo = np.array([md.dof_range[h][j][0] for h in range(2) for j in range(26)])
    hi = np.array([md.dof_range[h][j][1] for h in range(2) for j in range(26)])
    q[:, 88:] = lo + (hi - lo) * rng.uniform(0.6, 1.0, (n, 52))
    s0["qpos"], s0["qvel"] = q, v * 0.0
    la, ha = dp_action_spec(md)
    a = np.repeat(((la + ha) / 2)[None], n, 0).astype(np.float32)
    o.set_state(s0)
    o.step(a)  # settle
    return md, st, tc, o, a


def test_one_substep_full_contact_capacity(dp, ref):
    """states at 22-24 contacts in the substep (max_contacts 24 = MAXCON; 88+ contact
    rows, the contact lanes past 64 direction rows) held to the one-substep gate: qpos median
    < 1e-6, p99 < 5e-5; qacc relative p99 < 1e-3. The GPU counters must show the path: 88 or
    more contact rows (PS_STAT_MAX_ROWS = 4 x contacts) in the picked states."""
    md, sttab, tc, o, a = _contact_rich_states(dp, ref)
    s1 = o.get_state()
    cand = np.nonzero(o.contact_count() >= 21)[0]
    assert len(cand) >= 8, f"only {len(cand)} states with >= 21 contacts"
    states = {k: np.asarray(s1[k])[cand] for k in KEYS}
    stats, eq, ea = _one_substep(dp, ref, states, a[cand], lambda s: s[:, 3] >= 88, max_contacts=24)
    msg = (f"{len(eq)} of {len(cand)} states at >= 22 contacts on the GPU (rows max {stats[:, 3].max() if len(eq) else 0}): "
           f"qpos err median {np.median(eq) if len(eq) else 0:.2e} p99 {np.percentile(eq, 99) if len(eq) else 0:.2e}; "
           f"qacc rel err median {np.median(ea) if len(eq) else 0:.2e} p99 {np.percentile(ea, 99) if len(eq) else 0:.2e}")
    print(msg)
    assert len(eq) >= 8 and stats[:, 3].min() >= 88, msg
    assert np.median(eq) < 2e-6 and np.percentile(eq, 99) < 5e-5, msg
    assert np.percentile(ea, 99) < 1e-3, msg


def test_same_key_contacts_bitwise_repeatable(dp, ref):
    """A state with several contacts on one key (found with the oracle) replicated into 2048
    envs: every env - different workgroup, different dispatch slot - gives bitwise the same
    step, so the LDS float atomics that accumulate a key's row terms are deterministic."""
    md, st, tc = dp.compile_task(song(dp, "crossing_field"), dp.TaskConfig(trim_silence=True), canonical_actions=False)
    o = ref.OracleEnv(md, st, tc, 64)
    o.reset()
    lo, hi = dp.model.action_spec(md)
    rng = np.random.RandomState(2)
    pick = None
    for _ in range(60):
        o.step(rng.uniform(lo, hi, (64, 45)).astype(np.float32))
        for i in range(64):
            keys = [c[1] for c in o.contacts(i) if c[0] == 0]
            if keys and max(keys.count(k) for k in set(keys)) >= 3:
                pick = i
                break
        if pick is not None:
            break
    assert pick is not None, "no state with 3 contacts on one key"
    s = o.get_state()
    N = 2048
    rep = {k: np.repeat(s[k][pick:pick + 1], N, axis=0) for k in KEYS}
    g = dp.BatchedPianoEnv(N, song(dp, "crossing_field"), dp.TaskConfig(trim_silence=True), device="cuda:0",
                           canonical_actions=False)
    g.set_state(rep)
    a = torch.from_numpy(np.repeat(rng.uniform(lo, hi, (1, 45)).astype(np.float32), N, axis=0)).cuda()
    for _ in range(3):
        obs, rew, disc, stt = g.step(a)
        q = g.get_state()["qpos"]
        assert torch.equal(q, q[:1].expand_as(q))
        assert torch.equal(obs, obs[:1].expand_as(obs)) and torch.equal(rew, rew[:1].expand_as(rew))


def test_full_contact_capacity_teacher_forced(dp, ref):
    """max_contacts = 24 (MAXCON) with 22-24 contacts in a substep: every contact's direction-row
    dots come from its own lane (a lane per direction row stopped at 64 rows = 21
    contacts, and the 22nd+ took another contact's tangent J.v). States: _contact_rich_states,
    those still at >= 22 contacts after the settling step; one teacher-forced control step, GPU vs
    checker. The GPU counters must show the >= 22-contact path in the step (88+ contact rows in
    some substep) for at least a quarter of the states. Contact-rich states are ill-conditioned
    (the checker moves by ~1e-2 at p99 under a 1e-7 rad perturbation): qpos median within 2x the
    checker's own, p99 within 2x its own and below 5e-3, max below helpers.PARITY_MAX_CEIL
    (test_one_substep_full_contact_capacity holds the same path to the substep gate)."""
    md, st, tc, o, a = _contact_rich_states(dp, ref)
    pick = np.nonzero(o.contact_count() >= 22)[0]
    assert len(pick) >= 8, f"only {len(pick)} states with >= 22 contacts"
    n = len(pick)
    s1 = o.get_state()
    states = {k: np.asarray(s1[k])[pick] for k in KEYS}
    seq = song(dp, "crossing_field")
    task = dp.TaskConfig(trim_silence=True, max_contacts=24)
    g = dp.BatchedPianoEnv(n, seq, task, device="cuda:0", canonical_actions=False)
    o1, o2 = ref.OracleEnv(md, st, tc, n), Floor(ref, md, st, tc, n)
    g.reset()
    g.set_state(states)
    o1.set_state(states)
    o2.set_state(states, np.random.RandomState(2))
    g.step(torch.from_numpy(a[:n]).cuda())
    o1.step(a[:n])
    o2.step(a[:n])
    rows = g.solver_stats().cpu().numpy()[:, 3]
    qo = o1.get_state()["qpos"]
    e = np.abs(g.get_state()["qpos"].cpu().numpy() - qo).max(axis=1)
    f = o2.dev(qo)
    msg = (f"{n} states, {int((rows >= 88).sum())} reached 88+ contact rows on the GPU (max {rows.max()}): "
           f"qpos err median {np.median(e):.2e} p99 {np.percentile(e, 99):.2e} max {e.max():.2e}; the checker's "
           f"sensitivity median {np.median(f):.2e} p99 {np.percentile(f, 99):.2e}")
    print(msg)
    assert (rows >= 88).sum() >= max(4, n // 4), msg
    assert np.median(e) <= max(1e-5, 2.0 * np.median(f)), msg
    # measured (r05): p99 3.0e-3, max 9.5e-3 against the checker's own p99 1.1e-2
    assert np.percentile(e, 99) <= min(2.0 * np.percentile(f, 99), 5e-3) and e.max() <= PARITY_MAX_CEIL, msg
