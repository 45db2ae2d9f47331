"""Per-step launch tail from the -DPS_TIMING build (PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so).
When N envs fit the resident slots in one round (N <= 2048), a launch lasts as long as its
slowest env: this prints, step by step, the mean and the max per-env cycles and the phase split
of the slowest env against the mean. usage: python tools/tail_timing.py [N] [song]"""
import ctypes as C, importlib, sys
from pathlib import Path
import numpy as np, torch
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
dp = importlib.import_module("diffusion-piano_amd")
lib = importlib.import_module("diffusion-piano_amd._lib")
from helpers import song, tool_hand_kwargs
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
NAME = sys.argv[2] if len(sys.argv) > 2 else "twinkle"
STEPS = 20
L = lib.load()
L.ps_debug_timing.argtypes = [C.c_void_p, C.c_void_p]
g = dp.BatchedPianoEnv(N, song(dp, NAME), dp.TaskConfig(trim_silence=NAME != "twinkle", **tool_hand_kwargs()), device="cuda:0")
g.reset()
gen = torch.Generator(device="cuda:0").manual_seed(1)
for _ in range(3):
    g.step(torch.rand(N, 45, device="cuda:0", generator=gen) * 2 - 1)
L.ps_debug_timing(g._h, None)
names = {24: "kin:prologue", 25: "kin:levels", 0: "kin:rest", 26: "dyn:CRB levels", 27: "dyn:M rows", 1: "dyn:rest",
         11: "coll:piano cnt", 7: "coll:piano wr", 2: "coll:pairs", 18: "newton:prep", 3: "factor", 4: "solve_smooth",
         46: "nt:setup-keys", 47: "nt:setup-park", 48: "nt:setup-dofrows", 49: "nt:setup-keyrows",
         50: "nt:setup-contacts", 12: "nt:setup-rest", 51: "nt:rows", 13: "nt:grad", 14: "nt:hessian", 15: "nt:factor", 16: "nt:solve", 17: "nt:linesearch",
         8: "nt:J'f", 6: "integrate", 5: "final+task"}  # the slots of phase_timing.py (Newton solve)
idx = list(names)
out = np.zeros((N, 56), np.uint64)
means, maxes, worst_rows, mean_rows, ms, piv = [], [], [], [], [], []
for s in range(STEPS):
    a = torch.rand(N, 45, device="cuda:0", generator=gen) * 2 - 1
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.step(a)
    e1.record()
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1))
    L.ps_debug_timing(g._h, out.ctypes.data)
    ph = out[:, idx].astype(np.float64)
    tot = ph.sum(axis=1)
    live = tot > 0
    w = int(np.argmax(tot))
    means.append(ph[live].mean(axis=0))
    maxes.append(ph[w])
    worst_rows.append(out[w, 9] / 10.0)
    mean_rows.append(out[live, 9].mean() / 10.0)
    piv.append((out[live, 22].mean(), out[w, 22]))  # principal pivots per env-step (dual_ppt)
means, maxes = np.array(means), np.array(maxes)
mt, xt = means.sum(axis=1), maxes.sum(axis=1)
print(f"# tools/tail_timing.py {N} {NAME}: {STEPS} steps, per-step mean env vs slowest env (cycles per env-step)")
print(f"launch ms (timing build) mean {np.mean(ms):.3f}; mean env {mt.mean():.0f}, slowest env {xt.mean():.0f} "
      f"(ratio {xt.mean() / mt.mean():.2f}, per step min {np.min(xt / mt):.2f} max {np.max(xt / mt):.2f}); "
      f"rows/substep mean env {np.mean(mean_rows):.1f}, slowest env {np.mean(worst_rows):.1f}")
print(f"(slot 22, unused since the Newton solve) mean env {np.mean([a for a, b in piv]):.1f}, slowest env {np.mean([b for a, b in piv]):.1f}")
print(f"{'phase':18s} {'mean env':>10s} {'slowest':>10s} {'excess':>10s}")
for j, i in enumerate(idx):
    print(f"{names[i]:18s} {means[:, j].mean():10.0f} {maxes[:, j].mean():10.0f} {maxes[:, j].mean() - means[:, j].mean():10.0f}")
