"""Phase clock stamps of the fused PPO minibatch kernel (diagnostic build libpianorl_timing.so,
-DMLP_TIMING): one reference-schedule update on 4096 Twinkle envs, then the stamps of the last
minibatch's tile-0 workgroups (actor, critic) of mlp_rows_kernel, or of member 0 of mlp_split_kernel's
tile-0 groups (the default for these shapes; PIANORL_MLP_SPLIT=0 selects the other). With the product library
(PIANORL_LIB=.../libpianorl.so) it only runs the update, for rocprofv3's kernel trace."""
import ctypes as C
import importlib
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
os.environ.setdefault("PIANORL_LIB", str(ROOT / "diffusion-piano_amd" / "libpianorl_timing.so"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

dp = importlib.import_module("diffusion-piano_amd")
ppo = importlib.import_module("diffusion-piano_amd.ppo")
lib = importlib.import_module("diffusion-piano_amd._lib")

agent = ppo.PPOAgent(329, 45, batch_size=128, ppo_epochs=1, use_wandb=False, checkpoint_dir="/tmp/ppo_t", graphs=False)
N = 1024
S = torch.randn(N, 329, device="cuda")
A = torch.rand(N, 45, device="cuda") * 2 - 1
R = torch.randn(N, device="cuda")
D = torch.zeros(N, device="cuda")
agent.update(S, A, R, torch.zeros(N, device="cuda"), torch.randn(N, 329, device="cuda"), D)
torch.cuda.synchronize()
L = lib.load_rl()
if not hasattr(L, "prl_mlp_timing_get"):
    sys.exit(0)  # product build (kernel durations come from rocprofv3 around this script)
out = (C.c_uint64 * 64)()
L.prl_mlp_timing_get.argtypes = [C.c_void_p]
assert L.prl_mlp_timing_get(out) == 0
t = np.array(out[:], dtype=np.int64).reshape(2, 32)
names = {0: "start", 21: "L0 gemm", 1: "fwd L0", 22: "L1 gemm", 2: "fwd L1", 23: "L2 gemm", 3: "fwd L2", 5: "out+head", 7: "out dX",
         8: "L2 ln-bwd", 11: "L2 dX", 12: "L1 ln-bwd", 15: "L1 dX", 16: "L0 ln-bwd", 19: "L0", 20: "end",
         # mlp_split_kernel (member 0 of tile 0): the exchanges' signal -> data-in-LDS spans
         30: "idx rows", 31: "state tile", 4: "out gemm",
         24: "x0 exch", 25: "x1 exch", 26: "x2 exch", 27: "x3 exch", 28: "x4 exch", 29: "x5 exch"}
for net in range(2):
    prev = t[net, 0]
    print("actor" if net == 0 else "critic", "total", t[net, 20] - t[net, 0], "cycles")
    order = [0, 30, 31, 21, 24, 1, 22, 25, 2, 23, 26, 3, 4, 5, 7, 27, 8, 11, 28, 12, 15, 29, 16, 19, 20]
    for i in order:
        if i == 0 or t[net, i] == 0:
            continue
        print(f"   {names[i]:12s} {t[net, i] - prev:8d}")
        prev = t[net, i]
