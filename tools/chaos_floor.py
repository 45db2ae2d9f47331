"""Chaos floor of the free-running drift metric (BASELINE.json: qpos L-inf drift over 1000
steps): the fp64 CPU restatement against ITSELF with the hand joint positions perturbed by
delta at the start of every episode, on the drift test's action sources. If a 1e-12
perturbation of an fp64 run grows past 1e-4 within an episode, no implementation that is
not bit-identical to the checker (fp32 on a GPU, or MuJoCo itself run with another BLAS or
summation order) can hold the free-running drift under 1e-4 on that workload; the
teacher-forced (one-step) error is then the meaningful parity number.

Usage: python tools/chaos_floor.py [out.json]   (CPU only, ~1-2 min)
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
from helpers import DATA, song  # noqa: E402

N, STEPS = 8, 1000
KEYS = ("qpos", "qvel", "qacc_ws", "ctrl", "sustain", "t_idx", "last")
CHECK = (1, 5, 10, 20, 50, 100, 161, 500, 1000)


def run(dp, kind, delta):
    md, st, tc = dp.compile_task(song(dp, "twinkle"), dp.TaskConfig(), canonical_actions=False)
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
            s["qpos"][fresh, 88:] += delta * prng.choice([-1.0, 1.0], size=(int(fresh.sum()), 52))
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
    rep = {"checker": "fp64 C restatement vs itself, hand qpos perturbed by +-delta at each episode start",
           "envs": N, "steps": STEPS, "song": "twinkle", "oracle_sha": oracle_sha()}
    for kind in ("zero", "trace", "random"):
        for delta in (1e-12, 1e-7):
            rep[f"{kind}/delta={delta:g}"] = run(dp, kind, delta)
            print(kind, delta, rep[f"{kind}/delta={delta:g}"]["max_over_1000"], flush=True)
    path = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "profiles" / "chaos_floor.json"
    path.write_text(json.dumps(rep, indent=1))
    print("wrote", path)


if __name__ == "__main__":
    main()
