"""Debug aid: GPU vs checker contact lists on the box/hull test hand after one control step
from the same random states (ps_record_contacts / ps_contacts)."""
import importlib
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]
dp = importlib.import_module("diffusion-piano_amd")
import ref  # noqa: E402
from helpers import box_hull_hand, random_states, song  # noqa: E402

n = 8
hand = box_hull_hand(dp)
if len(sys.argv) > 1 and sys.argv[1] == "hulls":
    hand = hand._replace(xgeoms=[x for x in hand.xgeoms if x.kind == "hull"])
task = dp.TaskConfig(hand_xml=dp.mjcf.hand_to_mjcf(hand), control_timestep=0.005)
seq = song(dp, "twinkle")
md, st, tc = dp.compile_task(seq, task, canonical_actions=False)
g = dp.BatchedPianoEnv(n, seq, task, device="cuda:0", canonical_actions=False)
g.record_contacts(True)
o = ref.OracleEnv(md, st, tc, n)
rng = np.random.RandomState(1)
q, v = random_states(md, n, rng, vscale=0.1)
s = dict(qpos=q, qvel=v, qacc_ws=np.zeros_like(q), ctrl=np.zeros((n, 44)), sustain=np.zeros(n),
         t_idx=np.zeros(n, np.int32), last=np.zeros(n, np.uint8))
g.set_state(s)
o.set_state(s)
a = np.zeros((n, 45), np.float32)
g.step(torch.from_numpy(a).cuda())
o.step(a)
qg = g.get_state()["qpos"].cpu().numpy()
qo = o.get_state()["qpos"]
cg = g.contacts()
for i in range(n):
    e = np.abs(qg[i] - qo[i])
    co = o.contacts_full(i)
    print(f"env {i}: err {e.max():.3e} at {int(e.argmax())} ncon gpu {len(cg[i])} cpu {len(co)}")
    for c in co:
        match = [x for x in cg[i] if x[:4] == c[:4]]
        best = min(match, key=lambda x: np.abs(x[5] - c[5]).max()) if match else None
        if best is None:
            print("   CPU only", c[:5], np.round(c[5], 4), np.round(c[6], 3))
        else:
            dp_ = np.abs(best[5] - c[5]).max()
            dn = np.abs(best[6] - c[6]).max()
            if dp_ > 1e-4 or dn > 1e-3 or abs(best[4] - c[4]) > 1e-5:
                print("   DIFF", c[:5], "gpu dist", best[4], "dpos", dp_, "dn", dn, np.round(c[6], 3), np.round(best[6], 3))
    for x in cg[i]:
        if not [c for c in co if c[:4] == x[:4]]:
            print("   GPU only", x[:5], np.round(x[5], 4), np.round(x[6], 3))
