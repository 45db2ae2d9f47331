"""Chaos floor of the free-running drift metric (BASELINE.json: qpos L-inf drift over 1000
steps): the fp64 CPU restatement against ITSELF with the hand joint positions perturbed by
N(0, delta) at the start of every episode, on the drift test's action sources and workloads
(tests/test_gpu_drift.py: "bench" = Crossing Field with the reference's default box / hull
colliders, "twinkle" = Twinkle with the all-capsule hand). If a 1e-12 perturbation of an fp64
run grows past 1e-4 within an episode, no implementation that is not bit-identical to the
checker (fp32 on a GPU, or MuJoCo itself run with another BLAS or summation order) can hold the
free-running drift under 1e-4 on that workload; the teacher-forced (one-step) error is then the
meaningful parity number.

The perturbation keeps every joint on its side of its limits (helpers.perturb_joints): at
qpos0 22 of the 52 hand joints rest exactly ON a limit, and a move below it switches that
limit's row on - a discontinuity of the step, not chaos, whose size does not depend on delta
(round 5's version perturbed by +-delta and measured exactly that: the same step-1 difference
for delta 1e-12 and 1e-7). The record keeps the step-1 difference of each delta: for a chaos
measurement it scales with delta.

Usage: python tools/chaos_floor.py [out.json] [workload ...]   (CPU only, a few minutes)
"""
import importlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))

import ref  # noqa: E402  (the CPU checker)
from helpers import DATA, perturb_joints, song  # noqa: E402

N, STEPS = 8, 1000
KEYS = ("qpos", "qvel", "qacc_ws", "ctrl", "sustain", "t_idx", "last")
CHECK = (1, 5, 10, 20, 50, 100, 161, 500, 1000)


WORKLOADS = {"bench": ("crossing_field", dict(trim_silence=True, primitive_fingertip_collisions=False)),
             "twinkle": ("twinkle", {})}


def run(dp, kind, delta, workload):
    name, kw = WORKLOADS[workload]
    md, st, tc = dp.compile_task(song(dp, name), dp.TaskConfig(**kw), canonical_actions=False)
    a_env, b_env = ref.OracleEnv(md, st, tc, N), ref.OracleEnv(md, st, tc, N)
    lo, hi = dp.model.action_spec(md)
    rng = np.random.RandomState(12345)
    prng = np.random.RandomState(7)
    trace = np.load(DATA / "twinkle_twinkle_actions.npy").astype(np.float32)
    a_env.reset(); b_env.reset()
    out, worst = {}, 0.0
    for t in range(STEPS):
        s = b_env.get_state()
        fresh = s["t_idx"] == 0
        if fresh.any():  # perturb the hand joints of every env starting an episode
            s["qpos"][fresh, 88:] = perturb_joints(s["qpos"][fresh, 88:], prng, delta, md)
            b_env.set_state({k: s[k] for k in KEYS})
        if kind == "zero":
            a = np.zeros((N, 45), np.float32)
        elif kind == "trace":  # env i starts 20 i actions into the trace (tests/test_gpu_drift.py)
            x = trace[(t + 20 * np.arange(N)) % len(trace)]
            a = (lo + (x + 1) * 0.5 * (hi - lo)).astype(np.float32)
        else:
            a = rng.uniform(lo, hi, (N, 45)).astype(np.float32)
        a_env.step(a); b_env.step(a)
        d = float(np.abs(a_env.get_state()["qpos"] - b_env.get_state()["qpos"]).max())
        worst = max(worst, d)
        if t + 1 in CHECK:
            out[str(t + 1)] = d
    return {"qpos_linf_at_step": out, "max_over_1000": worst}


def oracle_sha():
    """The physics the floor is measured on (bench.py's oracle_sha: the checker's source and the
    compiled default model); bench.py drops a floor whose hash differs."""
    from bench import oracle_sha as sha
    return sha()


def main():
    dp = importlib.import_module("diffusion-piano_amd")
    rep = {"checker": "fp64 C restatement vs itself, hand qpos perturbed by N(0, delta) at each episode start, "
                      "every joint kept on its side of its limits (helpers.perturb_joints)",
           "envs": N, "steps": STEPS, "oracle_sha": oracle_sha(),
           "workloads": {k: f"{v[0]} {v[1]}" for k, v in WORKLOADS.items()}}
    path = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "profiles" / "chaos_floor.json"
    for w in sys.argv[2:] or list(WORKLOADS):
        rep[w] = {}
        for kind in ("zero", "trace", "random"):
            for delta in (1e-12, 1e-7):
                rep[w][f"{kind}/delta={delta:g}"] = r = run(dp, kind, delta, w)
                print(w, kind, delta, r["qpos_linf_at_step"]["1"], r["max_over_1000"], flush=True)
    path.write_text(json.dumps(rep, indent=1))
    print("wrote", path)


if __name__ == "__main__":
    main()
