"""Solver and cap study on the fp64 oracle (CPU only; no GPU).

Three questions on the benchmark workloads (random uniform actions):
* is the specification's exact dual solve (warm-up PGS sweeps + block principal pivoting)
  the converged solution? - checked against PGS run to convergence from a cold start (until
  no force moves by more than 1e-12 relative), an independent method for the same unique
  solution (the one MuJoCo's default Newton solver converges to);
* how far was round 1's truncated solver (20 cold-start PGS sweeps) from it?
* how often do the contact cap (max_contacts) and the coupled-row cap (PS_MAX_ROWS) bind?

Method: roll N envs forward with the specification; at every `--every`-th control step run
ONE control step from the state with each solver and compare qpos / qvel (L-inf per env).
Solves per substep and the cap histograms are collected over the specification's steps.

usage: python tools/solver_study.py [--out profiles/r02_solver_study.json] [--envs 64] [--steps 200]
"""
from __future__ import annotations

import argparse
import importlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))

KEYS = ("qpos", "qvel", "qacc_ws", "ctrl", "sustain", "t_idx", "last")


def pct(x, q):
    return float(np.percentile(x, q)) if len(x) else None


def _lf(d):
    return {"median": pct(d, 50), "p90": pct(d, 90), "p99": pct(d, 99), "max": float(d.max())}


def study(dp, ref, name, kw, n, steps, every, warmup, seed):
    from helpers import song
    seq = song(dp, name)
    md, st, tc = dp.compile_task(seq, dp.TaskConfig(pgs_iterations=warmup, **kw), canonical_actions=False)
    _, _, tc_pgs = dp.compile_task(seq, dp.TaskConfig(constraint_solver="pgs", **kw), canonical_actions=False)
    lo, hi = dp.model.action_spec(md)
    env = ref.OracleEnv(md, st, tc, n)          # the specification (exact dual solve)
    legacy = ref.OracleEnv(md, st, tc_pgs, n)   # round-1 solver: PGS, 20 cold-start sweeps
    env.reset()
    rng = np.random.RandomState(seed)
    ref.set_solver(0)
    tot = None

    def spec_step(a):  # one specification step; its counters are added to tot
        nonlocal tot
        s0 = ref.stats()
        env.step(a)
        s1 = ref.stats()
        d = {k: s1[k] - s0[k] for k in s1}
        tot = d if tot is None else {k: tot[k] + d[k] for k in tot}

    d_conv, d_pgs = ([], []), ([], [])
    t_exact = t_conv = 0.0
    for t in range(steps):
        a = rng.uniform(lo, hi, (n, 45)).astype(np.float32)
        if t % every != every - 1:
            spec_step(a)
            continue
        s = env.get_state()
        keep = s["last"] == 0
        t0 = time.perf_counter()
        spec_step(a)
        t_exact += time.perf_counter() - t0
        s_spec = env.get_state()
        env.set_state(s)
        ref.set_solver(1, 1e-12, 200000)   # converged PGS (independent check)
        t0 = time.perf_counter()
        env.step(a)
        t_conv += time.perf_counter() - t0
        ref.set_solver(0)
        s_conv = env.get_state()
        legacy.set_state(s)
        legacy.step(a)
        s_pgs = legacy.get_state()
        for dst, other in ((d_conv, s_conv), (d_pgs, s_pgs)):
            dst[0].append(np.abs(s_spec["qpos"] - other["qpos"]).max(axis=1)[keep])
            dst[1].append(np.abs(s_spec["qvel"] - other["qvel"]).max(axis=1)[keep])
        env.set_state(s_spec)  # continue the specification rollout
    stt = tot
    found, rowreq, pd = stt["found"], stt["rowreq"], stt["pdas"]
    subs = int(found.sum())
    mean = lambda h: float((np.arange(len(h)) * h).sum() / max(1, h.sum()))

    def q(h, p):
        c = np.cumsum(h)
        return int(np.searchsorted(c, p * c[-1]))

    cat = lambda x: np.concatenate(x)
    return {
        "song": name, "envs": n, "control_steps": steps, "warmup_sweeps": warmup,
        "samples": int(len(cat(d_conv[0]))),
        "exact_vs_converged_pgs_one_control_step": {"qpos_linf": _lf(cat(d_conv[0])), "qvel_linf": _lf(cat(d_conv[1])),
                                                    "cpu_s_exact": t_exact, "cpu_s_converged_pgs": t_conv},
        "exact_vs_pgs20_one_control_step": {"qpos_linf": _lf(cat(d_pgs[0])), "qvel_linf": _lf(cat(d_pgs[1]))},
        "exact_solver": {"solves_per_substep_hist": {int(i): int(pd[i]) for i in np.nonzero(pd)[0]},
                         "mean_solves": mean(pd[:63]), "iteration_cap_hits": int(pd[63])},
        "caps": {
            "max_contacts": tc.max_contacts, "max_rows": 64, "substeps": subs,
            "contacts_found": {"mean": mean(found), "p99": q(found, 0.99), "p999": q(found, 0.999),
                               "max": int(np.nonzero(found)[0].max()) if subs else 0},
            "rows_requested": {"mean": mean(rowreq), "p99": q(rowreq, 0.99), "p999": q(rowreq, 0.999),
                               "max": int(np.nonzero(rowreq)[0].max()) if subs else 0},
            "substeps_contacts_dropped": stt["contact_cap_substeps"],
            "substeps_rows_dropped": stt["row_cap_substeps"],
        },
    }


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default=str(ROOT / "profiles" / "r02_solver_study.json"))
    p.add_argument("--envs", type=int, default=64)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--every", type=int, default=20)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--songs", default="crossing_field,twinkle,guren")
    args = p.parse_args()
    dp = importlib.import_module("diffusion-piano_amd")
    import ref
    ref.build()
    kws = {"twinkle": {}, "crossing_field": dict(trim_silence=True), "guren": dict(trim_silence=True)}
    out = {"what": "the specification's exact dual solve vs PGS run to convergence (independent check) and vs "
                   "the round-1 solver (PGS, 20 cold-start sweeps): one control step teacher-forced from "
                   "random-action rollout states (specification rollout); solves per substep and cap "
                   "histograms over the specification rollout",
           "results": []}
    for name in args.songs.split(","):
        r = study(dp, ref, name, kws[name], args.envs, args.steps, args.every, args.warmup, 12345)
        print(json.dumps(r), flush=True)
        out["results"].append(r)
    Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
