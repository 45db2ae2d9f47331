"""Debug aid: run the twinkle teacher-forced workload with a PS_CHECK_A build (prints MFMA vs
scalar Delassus mismatches from the kernel)."""
import importlib, sys
from pathlib import Path
import numpy as np, torch
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
dp = importlib.import_module("diffusion-piano_amd")
from helpers import song
for name, n in (("twinkle", 256), ("crossing_field", 1024)):
    g = dp.BatchedPianoEnv(n, song(dp, name), dp.TaskConfig(trim_silence=name != "twinkle"), device="cuda:0")
    g.reset()
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    for i in range(12):
        g.step(torch.rand(n, 45, device="cuda:0", generator=gen) * 2 - 1)
    torch.cuda.synchronize()
    print(name, "max rows", int(g.solver_stats().cpu().numpy()[:, 3].max()), flush=True)
