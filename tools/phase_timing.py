"""Per-phase cycle breakdown from the -DPS_TIMING diagnostic build (run with
PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so). Shares, not absolute speed."""
import ctypes as C, importlib, sys
from pathlib import Path
import numpy as np, torch
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
dp = importlib.import_module("diffusion-piano_amd")
lib = importlib.import_module("diffusion-piano_amd._lib")
from helpers import song, tool_hand_kwargs
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
L = lib.load()
L.ps_debug_timing.argtypes = [C.c_void_p, C.c_void_p]
NAME = sys.argv[2] if len(sys.argv) > 2 else "crossing_field"
g = dp.BatchedPianoEnv(N, song(dp, NAME), dp.TaskConfig(trim_silence=NAME != "twinkle", **tool_hand_kwargs()), device="cuda:0")
g.reset()
L.ps_debug_timing(g._h, None)
gen = torch.Generator(device="cuda:0").manual_seed(1)
stats = []
for i in range(10):
    g.step(torch.rand(N, 45, device="cuda:0", generator=gen) * 2 - 1)
    stats.append(g.solver_stats().cpu().numpy())
st = np.stack(stats)  # [10, N, 4]
NPH = 56
out = np.zeros((N, NPH), np.uint64)
L.ps_debug_timing(g._h, out.ctypes.data)
names = {24: "kin:prologue", 25: "kin:levels", 0: "kin:rest", 26: "dyn:CRB levels", 27: "dyn:M rows", 1: "dyn:rest",
         11: "coll:piano cnt", 7: "coll:piano wr", 2: "coll:pairs", 18: "newton:prep", 3: "factor", 4: "solve_smooth",
         46: "nt:setup-keys", 47: "nt:setup-park", 48: "nt:setup-dofrows", 49: "nt:setup-keyrows",
         50: "nt:setup-contacts", 12: "nt:setup-rest", 51: "nt:rows", 13: "nt:grad", 14: "nt:hessian", 15: "nt:factor", 16: "nt:solve", 17: "nt:linesearch",
         8: "nt:J'f", 6: "integrate", 5: "final+task", 32: "xpiano:cand", 33: "xpiano:refine", 34: "xpiano:narrow",
         35: "xpairs:sphere", 36: "xpairs:refine", 37: "xpairs:narrow"}
tot = out[:, [i for i in names]].astype(np.float64).sum(axis=1)
for i, n in names.items():
    v = out[:, i].astype(np.float64)
    print(f"{n:14s} {v.mean()/10:12.0f} cycles/env-step  {100*v.sum()/tot.sum():5.1f}%")
print(f"total {tot.mean()/10:.0f} cycles/env-step per wave; mean rows/substep {out[:,9].mean()/100:.1f} mean contacts {out[:,10].mean()/100:.2f}")
solves = st[..., 0] / 10.0
print(f"Newton: iterations per substep mean {solves.mean():.3f}, max over env-steps {st[..., 0].max()} per step; "
      f"contact-cap substeps {int(st[..., 1].sum())}, iteration-cap substeps {int(st[..., 2].sum())}, "
      f"max contact rows {int(st[..., 3].max())}, coupled substeps {st[..., 4].sum() / (10 * st[..., 4].size):.3f}")
# iterations by substep (timing-build counters 19-23): the first substep starts cold, the later
# ones from the previous substep's zones (one iteration when that piece holds)
c = out[:, 19:24].astype(np.float64).sum(axis=0)
m = out[:, 28:32].astype(np.float64).sum(axis=0)  # box / hull narrow-phase rounds (timing build)
# (since round 6 the piano and hand-hand box / hull pairs are one list: one refine pass and one
# series of rounds, counted in the hand-hand slots - xpiano:refine / narrow and the piano round
# counters stay 0; xpiano:cand is the piano candidates, xpairs:sphere the hand-hand spheres)
if m[1] > 0 or m[3] > 0:
    print(f"box/hull narrow phase: piano {m[1] / N / 100:.2f} rounds/substep, {m[0] / max(m[1], 1):.1f} MPR steps of the "
          f"slowest lane per round; piano + hand-hand {m[3] / N / 100:.2f} rounds/substep, {m[2] / max(m[3], 1):.1f} steps")
h = out[:, 38:46].astype(np.float64).sum(axis=0)
if h[0] > 0:
    print(f"box/hull pairs per substep: {h[7] / N / 100:.2f} listed (piano candidates + hand-hand past the spheres), "
          f"{h[0] / N / 100:.2f} past the enclosing capsules (substeps with any: {h[4] / N / 100:.3f}), {h[1] / N / 100:.3f} "
          f"with a contact; MPR steps per pair {h[2] / max(h[0], 1):.2f} (contact pairs {h[3] / max(h[1], 1):.2f}, others "
          f"{(h[2] - h[3]) / max(h[0] - h[1], 1):.2f}); piano hull pairs per substep (before round 6) {h[5] / N / 100:.2f}, "
          f"{h[6] / N / 100:.3f} with a contact")
if c[1] > 0 and c[4] > 0:
    print(f"Newton by substep: first {c[0] / c[1]:.2f} iterations, later {c[2] / c[4]:.2f} "
          f"(guessed piece held in {100 * c[3] / c[4]:.1f}% of the later substeps)")
# the per-env spread sets the tail of a launch (4096 envs = 2 rounds of 2048 slots)
per = tot / 10
q = np.percentile(per, [50, 90, 99, 100])
top = per >= q[2]
print(f"per-env cycles/env-step p50 {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} max {q[3]:.0f}; "
      f"rows/substep: all {out[:,9].mean()/100:.1f}, top 1% {out[top,9].mean()/100:.1f}")
for i, n in names.items():
    v = out[top, i].astype(np.float64)
    print(f"  top1% {n:14s} {v.mean()/10:12.0f}")
# the slowest envs, phase by phase (what sets a launch's tail at one round of workgroups)
worst = np.argsort(per)[-3:][::-1]
print("slowest envs (cycles/env-step):", ", ".join(f"{per[w]:.0f}" for w in worst),
      "| Newton iterations per step:", ", ".join(str(int(st[:, w, 0].sum() / 10)) for w in worst),
      "| max contact rows:", ", ".join(str(int(st[:, w, 3].max())) for w in worst))
for i, n in names.items():
    print(f"  worst {n:14s} " + " ".join(f"{out[w, i] / 10:10.0f}" for w in worst))
