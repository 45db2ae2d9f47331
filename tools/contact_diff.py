"""GPU vs checker contact lists on the benched workload, collision only (development aid,
round 6). bench.py's workload (Crossing Field, box / hull colliders, 4096 staggered envs, random
actions) is rolled on the GPU with contact recording on; after the last step the GPU's contact
list of each env (its task-layer collision pass at the end state) is compared with the
checker's collision pass at the SAME state (ref.OracleEnv.set_state runs kinematics + collide on
the fp32 state it is given). A contact present on one side only, or one whose distance differs
by more than 1e-5 m, normal by 1e-3 or point by 1e-4 m, is counted by pair kind; the worst ones
are printed with both sides' numbers and the pair's collider ids.

usage: python tools/contact_diff.py [steps] [envs]   (GPU)"""
import dataclasses
import importlib
import json
import sys
from collections import Counter
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]
dp = importlib.import_module("diffusion-piano_amd")
import ref  # noqa: E402  (the CPU checker)
from bench import load_song, stagger_episodes  # noqa: E402

KEYS = ("qpos", "qvel", "qacc_ws", "ctrl", "sustain", "t_idx", "last")


def kind_of(c, ncap=40):
    kind, key, g1, g2 = c[:4]
    a = "x" if g1 >= ncap else "c"
    if key >= 0 or g2 < 0:
        return f"{a}-key" if key >= 0 else f"{a}-base"
    return f"{a}-{'x' if g2 >= ncap else 'c'}"


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    mode = sys.argv[3] if len(sys.argv) > 3 else "bench"
    if mode == "bench":
        seq, task = load_song(dp, "crossing_field")
        task = dataclasses.replace(task, primitive_fingertip_collisions=False)
    else:  # "random": random joint states of the all-capsule hand (tests/helpers.random_states)
        from helpers import random_states, song
        seq, task = song(dp, "twinkle"), dp.TaskConfig(control_timestep=0.005)
    md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
    g = dp.BatchedPianoEnv(N, seq, task, device="cuda:0", seed=12345, canonical_actions=False)
    g.record_contacts(True)
    lo, hi = dp.model.action_spec(md)
    rng = np.random.RandomState(3)
    g.reset()
    if mode == "bench":
        stagger_episodes(g, 0, g.song.T)
        for _ in range(steps):
            g.step(torch.from_numpy(rng.uniform(lo, hi, (N, 45)).astype(np.float32)).cuda())
    else:
        q, v = random_states(md, N, rng, vscale=0.1)
        q[:, :88] = np.clip(q[:, :88], 0.0, None)
        g.set_state(dict(qpos=q, qvel=v, qacc_ws=np.zeros_like(q), ctrl=np.zeros((N, 44)), sustain=np.zeros(N),
                         t_idx=np.zeros(N, np.int32), last=np.zeros(N, np.uint8)))
        g.step(torch.zeros(N, 45, device="cuda:0"))
    s = {k: v.cpu().numpy() for k, v in g.get_state().items() if k in KEYS}
    cg = g.contacts()
    o = ref.OracleEnv(md, st, tc, N)
    o.set_state(s)
    tot, cnt, worst, rows = Counter(), Counter(), [], []
    for i in range(N):
        co = o.contacts_full(i)
        used = set()
        for c in co:
            k = kind_of(c)
            tot[k] += 1
            match = [j for j, x in enumerate(cg[i]) if x[:4] == c[:4] and j not in used]
            if not match:
                cnt[("cpu_only", k)] += 1
                worst.append((abs(c[4]) + 1.0, i, "cpu_only", c[:5], None))
                continue
            j = min(match, key=lambda j: np.abs(cg[i][j][5] - c[5]).max())
            used.add(j)
            x = cg[i][j]
            dd, dpos, dn = abs(x[4] - c[4]), np.abs(x[5] - c[5]).max(), np.abs(x[6] - c[6]).max()
            if dd > 1e-5 or dpos > 1e-4 or dn > 1e-3:
                cnt[("diff", k)] += 1
                rows.append([i, *c[:4], x[4], *x[5], *x[6], c[4], *c[5], *c[6]])
                worst.append((dn + dd * 100, i, "diff", c[:5], (x[4], dpos, dn, np.round(c[6], 4).tolist(),
                                                                np.round(x[6], 4).tolist())))
        for j, x in enumerate(cg[i]):
            if j not in used and not [c for c in co if c[:4] == x[:4]]:
                cnt[("gpu_only", kind_of(x))] += 1
                worst.append((abs(x[4]) + 1.0, i, "gpu_only", x[:5], None))
    print(json.dumps({"envs": N, "steps": steps, "contacts_by_kind": dict(tot),
                      "mismatches": {f"{a}/{b}": v for (a, b), v in sorted(cnt.items())}}), flush=True)
    Path("gpurun_out").mkdir(exist_ok=True)
    np.savez("gpurun_out/contact_diff.npz", rows=np.array(rows, np.float64), **{"s_" + k: v for k, v in s.items()})
    worst.sort(key=lambda w: -w[0])
    for w in worst[:40]:
        print(w[1:], flush=True)


if __name__ == "__main__":
    ref.build()
    main()
