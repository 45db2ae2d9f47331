"""Development aid: the state after K steps of a fixed random-action rollout of the library the
loader binds (PIANOSIM_LIB), saved for a bitwise comparison of two builds.
usage: PIANOSIM_LIB=... python tools/ab_state.py out.npz [N] [K]   (PIANOSIM_HAND: collider set)"""
import importlib
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
dp = importlib.import_module("diffusion-piano_amd")
from helpers import song, tool_hand_kwargs  # noqa: E402

out = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
g = dp.BatchedPianoEnv(N, song(dp, "crossing_field"), dp.TaskConfig(trim_silence=True, **tool_hand_kwargs()),
                       device="cuda:0")
g.reset()
gen = torch.Generator(device="cuda:0").manual_seed(77)
rews = []
for _ in range(K):
    _, r, _, _ = g.step(torch.rand(N, 45, device="cuda:0", generator=gen) * 2 - 1)
    rews.append(r.cpu().numpy())
s = {k: v.cpu().numpy() for k, v in g.get_state().items()}
np.savez(out, rew=np.stack(rews), **s)
print(out, "done")
