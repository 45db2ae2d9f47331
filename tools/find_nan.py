"""Run N envs with random actions; dump the first env/step whose state turns non-finite."""
import importlib, sys
from pathlib import Path
import numpy as np, torch
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
dp = importlib.import_module("diffusion-piano_amd")
from helpers import song
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
g = dp.BatchedPianoEnv(N, song(dp, "twinkle"), dp.TaskConfig(), device="cuda:0", canonical_actions=False)
lo = torch.tensor(g.action_lo, device="cuda:0", dtype=torch.float32); hi = torch.tensor(g.action_hi, device="cuda:0", dtype=torch.float32)
g.reset()
gen = torch.Generator(device="cuda:0").manual_seed(12345)
found = 0
maxv = []
for t in range(80):
    s0 = g.get_state()
    a = lo + torch.rand(N, 45, device="cuda:0", generator=gen) * (hi - lo)
    obs, rew, disc, st = g.step(a)
    s1 = g.get_state()
    bad = ~(torch.isfinite(s1["qpos"]).all(1) & torch.isfinite(s1["qvel"]).all(1) & torch.isfinite(rew) & (s1["qvel"].abs().max(1).values < 1e3))
    maxv.append(float(s1["qvel"][torch.isfinite(s1["qvel"]).all(1)].abs().max()))
    if bad.any():
        idx = torch.nonzero(bad).flatten().cpu().numpy()
        print(f"step {t}: {len(idx)} bad envs, first {idx[:10]}")
        if not found:
            e = int(idx[0])
            np.savez("gpurun_out/nan_case.npz", **{k: v[e].cpu().numpy() for k, v in s0.items()}, action=a[e].cpu().numpy(), step=t, env=e,
                     after_q=s1["qpos"][e].cpu().numpy(), after_v=s1["qvel"][e].cpu().numpy(), ncon=g.contact_count()[e].item())
        found += len(idx)
        if found > 50: break
print("max |qvel| per step (finite envs):", np.round(maxv[:10], 1), "...", np.round(maxv[-5:], 1))
