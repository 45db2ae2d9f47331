"""How well does a perturbed fp64 checker run measure a state's sensitivity (the "floor" of the
parity gates)? Development aid (round 6): for each env-step of a teacher-forced comparison it
records the GPU's qpos error against the checker and the checker's own move under K
independent perturbations of several kinds:

  q     hand joints N(0, 1e-7) rad, each kept on its side of its limits (helpers.perturbed)
  qv    the same plus every velocity moved by N(0, 1e-7 max(|v|, 1)) - the fp32 rounding scale of
        the state the GPU carries between its substeps (friction-loss and contact zones depend on
        velocity; a position-only perturbation never probes that)

and prints, per floor definition (kind, K = 1..3: max over the first K samples), the gate's
numbers: well-conditioned count (floor < 1e-5) and the GPU's p99 over them, the all-sample p99,
the floor p99, flip rates. Cases: trace (Twinkle, capsule hand, the reference's action trace,
16 envs x 200 steps), bench (Crossing Field, box/hull hand, 4096 staggered envs, 256 sampled x 6
steps), random (Twinkle, capsule hand, random actions, 16 x 200).

usage: python tools/floor_study.py [case ...]   (GPU; PIANOSIM_REFINE = TaskConfig.solver_refine)
writes gpurun_out/floor_study_<case>.npz"""
import dataclasses
import importlib
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "oracle"))
dp = importlib.import_module("diffusion-piano_amd")
import ref  # noqa: E402  (the CPU checker)
from helpers import DATA, perturb_joints, song  # noqa: E402
from bench import load_song, stagger_episodes  # noqa: E402

KEYS = ("qpos", "qvel", "qacc_ws", "ctrl", "sustain", "t_idx", "last")
REFINE = int(os.environ.get("PIANOSIM_REFINE", "1"))
K = 3
THREADS = int(os.environ.get("FLOOR_THREADS", "16"))


def perturb(s, rng, kind, md):
    s = dict(s)
    q = np.array(s["qpos"], np.float64)
    q[:, 88:] = perturb_joints(q[:, 88:], rng, 1e-7, md)
    s["qpos"] = q
    if kind == "qv":
        v = np.array(s["qvel"], np.float64)
        s["qvel"] = v + rng.normal(0.0, 1.0, v.shape) * 1e-7 * np.maximum(np.abs(v), 1.0)
    return s


def run(case):
    if case == "bench":
        seq, task = load_song(dp, "crossing_field")
        task = dataclasses.replace(task, primitive_fingertip_collisions=False, solver_refine=REFINE)
        N, n, steps, warm = 4096, 256, 6, 12
    else:
        seq, task = song(dp, "twinkle"), dp.TaskConfig(solver_refine=REFINE)
        N = n = 16
        steps, warm = 200, 0
    md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
    g = dp.BatchedPianoEnv(N, seq, task, device="cuda:0", seed=12345, canonical_actions=False)
    o = ref.OracleEnv(md, st, tc, n)
    o2 = ref.OracleEnv(md, st, tc, n)
    lo, hi = dp.model.action_spec(md)
    rng, prng = np.random.RandomState(31), np.random.RandomState(32)
    trace = np.load(DATA / "twinkle_twinkle_actions.npy").astype(np.float32)
    idx = np.sort(rng.choice(N, n, replace=False))
    g.reset()
    if case == "bench":
        stagger_episodes(g, 0, g.song.T)
    for _ in range(warm):
        g.step(torch.from_numpy(rng.uniform(lo, hi, (N, 45)).astype(np.float32)).cuda())
    rec = {"err": [], "stats": [], "ncon": [], "act": [], "qg": []}
    states = []
    for kind in ("q", "qv"):
        rec[f"floor_{kind}"] = []
    for t in range(steps):
        if case == "trace":
            x = trace[(t + 10 * np.arange(N)) % len(trace)]
            a = (lo + (x + 1) * 0.5 * (hi - lo)).astype(np.float32)
        else:
            a = rng.uniform(lo, hi, (N, 45)).astype(np.float32)
        s = {k: v.cpu().numpy()[idx] for k, v in g.get_state().items() if k in KEYS}
        states.append(s)
        rec["act"].append(a[idx])
        o.set_state(s)
        g.step(torch.from_numpy(a).cuda())
        o.step(a[idx], THREADS)
        qo = o.get_state()["qpos"]
        qg = g.get_state()["qpos"].cpu().numpy()[idx]
        rec["qg"].append(qg)
        rec["err"].append(np.abs(qg - qo).max(axis=1))
        rec["stats"].append(g.solver_stats().cpu().numpy()[idx])
        rec["ncon"].append(o.contact_count())
        for kind in ("q", "qv"):
            fs = []
            for _ in range(K):
                o2.set_state(perturb(s, prng, kind, md))
                o2.step(a[idx], THREADS)
                fs.append(np.abs(o2.get_state()["qpos"] - qo).max(axis=1))
            rec[f"floor_{kind}"].append(np.stack(fs, 1))
    out = {k: np.concatenate(v) for k, v in rec.items()}
    st_all = {k: np.concatenate([x[k] for x in states]) for k in KEYS}
    Path("gpurun_out").mkdir(exist_ok=True)
    np.savez(f"gpurun_out/floor_study_{case}_r{REFINE}.npz", **out, **{"s_" + k: v for k, v in st_all.items()})
    # the env-steps the 3-sample floors call well-conditioned where the GPU moved by > 1e-4: the
    # checker with many more perturbations - does it reach the GPU's deviation itself?
    e = out["err"]
    f3 = np.maximum(out["floor_q"].max(axis=1), out["floor_qv"].max(axis=1))
    sus = np.nonzero((f3 < 1e-5) & (e > 1e-4))[0]
    if len(sus):
        KK = 48
        sub = {k: v[sus] for k, v in st_all.items()}
        acts = out["act"][sus]
        os_ = ref.OracleEnv(md, st, tc, len(sus))
        os_.set_state(sub)
        os_.step(acts, THREADS)
        q0 = os_.get_state()["qpos"]
        fk = []
        for k in range(KK):
            os_.set_state(perturb(sub, prng, "qv" if k % 2 else "q", md))
            os_.step(acts, THREADS)
            fk.append(np.abs(os_.get_state()["qpos"] - q0).max(axis=1))
        fk = np.stack(fk, 1)
        reach = fk.max(axis=1) >= 0.5 * e[sus]
        print(json.dumps({"case": case, "suspicious": int(len(sus)), "of_well": int((f3 < 1e-5).sum()),
                          "checker_reaches_half_gpu_err_within_48": int(reach.sum()),
                          "frac_perturbations_flipping": [float(np.mean(fk[i] > 1e-5)) for i in range(len(sus))],
                          "gpu_err": [float(x) for x in e[sus]], "checker_max48": [float(x) for x in fk.max(axis=1)]}),
              flush=True)
    e = out["err"]
    summary = {"case": case, "refine": REFINE, "n": int(e.size), "median": float(np.median(e)),
               "p99": float(np.percentile(e, 99)), "max": float(e.max())}
    for kind in ("q", "qv"):
        for k in range(1, K + 1):
            f = out[f"floor_{kind}"][:, :k].max(axis=1)
            calm = f < 1e-5
            summary[f"{kind}{k}"] = {"n_well": int(calm.sum()),
                                     "p99_well": float(np.percentile(e[calm], 99)) if calm.any() else None,
                                     "floor_p99": float(np.percentile(f, 99)),
                                     "flip_gpu_floor_1e-3": [float(np.mean(e > 1e-3)), float(np.mean(f > 1e-3))],
                                     "flip_gpu_floor_1e-4": [float(np.mean(e > 1e-4)), float(np.mean(f > 1e-4))]}
    print(json.dumps(summary), flush=True)
    # the worst env-steps the q3 floor calls well-conditioned, with their features
    f = out["floor_qv"].max(axis=1)
    order = np.argsort(-e)
    for i in order[:20]:
        print("err %.2e floor_q %s floor_qv %s stats %s ncon %d" % (
            e[i], np.array2string(out["floor_q"][i], precision=1), np.array2string(out["floor_qv"][i], precision=1),
            out["stats"][i].tolist(), out["ncon"][i]), flush=True)


if __name__ == "__main__":
    ref.build()
    for c in sys.argv[1:] or ["trace", "bench", "random"]:
        run(c)
