"""qpos drift of the fp32 HIP step against the fp64 oracle (BASELINE.json's second metric).

Reported, from identical (qpos, qvel, qacc_warmstart, ctrl):
  * teacher-forced: the oracle is re-synced to the GPU state before every control step,
    so the error is one step's fp32-vs-fp64 difference;
  * free-running: both sides start from reset and step the same action sequence for
    1000 control steps (episodes auto-reset every T steps on both sides).
Three action sources: zero actions (no contact), the reference's recorded Twinkle action
trace (tests/data/twinkle_twinkle_actions.npy, examples/ of the reference, 158x45 canonical
actions, replayed cyclically; env i starts 20 i actions into it, so the envs visit different
states) and uniform random actions. Two workloads: "bench" - the one bench.py's headline times
(Crossing Field, the reference's default box / convex-hull colliders,
PianoTask(primitive_fingertip_collisions=False)) - and "twinkle" (Twinkle, the authored
all-capsule hand; the report of rounds 1-5).

Bounded here: teacher-forced qpos (helpers.assert_parity for the capsule hand: median < 1e-5,
p99 < 1e-4 over the env-steps the checker itself resolves to 1e-5 under a limit-preserving
1e-7 rad perturbation, p99 over all within max(1e-4, 2x that sensitivity); the box / hull hand
by helpers.assert_flip_rates, the same median and well-conditioned clauses plus flip rates) and
free-running zero-action drift (< 1e-4 over 1000 steps). Free-running drift under contact-rich actions is chaotic
(a fp32 rounding difference in a stiff contact grows ~x1e3 in ~20 steps), so it is recorded,
not bounded; see DESIGN.md "Parity". When PIANOSIM_REPORT is set the numbers are written
there as JSON (profiles/r01_drift.json is one such report).
"""
import json
import os

import numpy as np
import pytest

from helpers import DATA, PARITY_P99_CEIL_UNREFINED, Floor, assert_flip_rates, assert_parity, song

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
KEYS = ("qpos", "qvel", "qacc_ws", "ctrl", "sustain", "t_idx", "last")
STEPS = 1000
N = 8


WORKLOADS = {  # name -> (song, TaskConfig kwargs, report key)
    "bench": ("crossing_field", dict(trim_silence=True, primitive_fingertip_collisions=False),
              "Crossing Field, box/hull hand (bench.py's headline workload)"),
    "twinkle": ("twinkle", {}, "Twinkle, authored all-capsule hand"),
}


def _task(dp, workload):
    name, kw, _ = WORKLOADS[workload]
    return song(dp, name), dp.TaskConfig(**kw)


def _envs(dp, ref, workload):
    seq, task = _task(dp, workload)
    md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
    g = dp.BatchedPianoEnv(N, seq, task, device="cuda:0", canonical_actions=False)
    o = ref.OracleEnv(md, st, tc, N)
    return md, g, o


def _gq(g):
    return g.get_state()["qpos"].cpu().numpy()


def _run(dp, ref, kind, workload):
    trace = np.load(DATA / "twinkle_twinkle_actions.npy").astype(np.float32) if kind == "trace" else None
    md, g, o = _envs(dp, ref, workload)
    lo, hi = dp.model.action_spec(md)
    rng = np.random.RandomState(12345)

    def action(t):
        if kind == "zero":
            return np.zeros((N, 45), np.float32)
        if kind == "trace":
            a = trace[(t + 20 * np.arange(N)) % len(trace)]  # canonical [-1, 1] -> spec units
            return (lo + (a + 1) * 0.5 * (hi - lo)).astype(np.float32)
        return rng.uniform(lo, hi, (N, 45)).astype(np.float32)

    g.reset()
    o.reset()
    free, tf = [], []
    for t in range(STEPS):
        a = action(t)
        g.step(torch.from_numpy(a).cuda())
        o.step(a)
        free.append(float(np.abs(_gq(g) - o.get_state()["qpos"]).max()))
    # teacher-forced: re-sync every step; o2 from the perturbed state (the checker's sensitivity)
    g.reset()
    o.reset()
    o2 = Floor(ref, *dp.compile_task(*_task(dp, workload), canonical_actions=False), N, k=3)  # (8 envs: cheap)
    prng = np.random.RandomState(4)
    floor = []
    for t in range(200):
        a = action(t)
        s = {k: v.cpu().numpy() for k, v in g.get_state().items()}
        o.set_state({k: s[k] for k in KEYS})
        o2.set_state({k: s[k] for k in KEYS}, prng)
        g.step(torch.from_numpy(a).cuda())
        o.step(a)
        o2.step(a)
        qo = o.get_state()["qpos"]
        tf.append(np.abs(_gq(g) - qo).max(axis=1))
        floor.append(o2.dev(qo))
    tf, floor = np.concatenate(tf), np.concatenate(floor)
    at = lambda k: free[k - 1]
    return {"free_running_qpos_linf": {str(k): at(k) for k in (1, 5, 10, 20, 50, 100, 161, 500, 1000)},
            "free_running_max_over_1000": max(free),
            "teacher_forced_qpos_linf": {"median": float(np.median(tf)), "p99": float(np.percentile(tf, 99)),
                                         "max": float(tf.max()), "samples": int(tf.size),
                                         "p99_well_conditioned": float(np.percentile(tf[floor < 1e-5], 99))
                                         if (floor < 1e-5).any() else None,
                                         "well_conditioned_samples": int((floor < 1e-5).sum()),
                                         "fp64_self_1e-7_p99": float(np.percentile(floor, 99))},
            "_tf": tf, "_floor": floor}


@pytest.fixture(scope="module")
def report():
    import sys
    from helpers import ROOT
    sys.path.insert(0, str(ROOT))
    from bench import lib_sha
    rep = {"envs": N, "steps": STEPS, "oracle": "fp64 C restatement (oracle/pianosim_ref.c)",
           "perturbation": "hand joints N(0, 1e-7) rad, each kept on its side of its limits (helpers.perturbed)",
           "lib_sha": lib_sha(), "workloads": {k: v[2] for k, v in WORKLOADS.items()}}
    yield rep
    path = os.environ.get("PIANOSIM_REPORT")
    if path:
        with open(path, "w") as f:
            json.dump(rep, f, indent=1)


@pytest.mark.parametrize("workload", ["bench", "twinkle"])
def test_drift_zero_action(dp, ref, report, workload):
    r = _run(dp, ref, "zero", workload)
    r.pop("_tf"), r.pop("_floor")
    report.setdefault(workload, {})["zero_action"] = r
    assert r["free_running_max_over_1000"] < 1e-4, r
    assert r["teacher_forced_qpos_linf"]["max"] < 1e-5, r


@pytest.mark.parametrize("workload", ["bench", "twinkle"])
@pytest.mark.parametrize("kind", ["trace", "random"])
def test_drift_contact_rich(dp, ref, report, kind, workload):
    r = _run(dp, ref, kind, workload)
    tf, floor = r.pop("_tf"), r.pop("_floor")
    report.setdefault(workload, {})[f"{kind}_actions"] = r
    if workload == "bench":  # MPR face switches: the box / hull hand's gate
        assert_flip_rates(tf, floor, f"{workload}: {kind} actions, teacher-forced")
    elif kind == "trace":  # the reference's Twinkle trace: its top 1% are steps the checker itself
        # moves by 2e-5 - 2e-4 under the perturbation and the GPU by 1-3x that (refining every
        # substep: p99 1.42e-4 -> 1.16e-4): 3x the floor, round 5's ceiling
        assert_parity(tf, floor, f"{workload}: {kind} actions, teacher-forced", p99_ceil=PARITY_P99_CEIL_UNREFINED,
                      floor_factor=3.0)
    else:
        assert_parity(tf, floor, f"{workload}: {kind} actions, teacher-forced")
    assert np.isfinite(r["free_running_max_over_1000"])
