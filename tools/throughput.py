"""Quick GPU throughput sweep over env counts and songs (development aid; bench.py is the
contract). usage: python tools/throughput.py [song] [N ...]"""
import importlib
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
dp = importlib.import_module("diffusion-piano_amd")
from helpers import song, tool_hand_kwargs  # noqa: E402


def throughput(name, n, steps=20):
    import os
    its = os.environ.get("PIANOSIM_NEWTON_ITERS")  # Newton iteration cap (default: the library's)
    task = dp.TaskConfig(trim_silence=name != "twinkle", solver_iterations=None if its is None else int(its),
                         **tool_hand_kwargs())  # PIANOSIM_HAND: the collider set (bench.py --hand)
    g = dp.BatchedPianoEnv(n, song(dp, name), task, device="cuda:0")
    g.reset()
    gen = torch.Generator(device="cuda:0").manual_seed(12345)
    acts = [torch.rand(n, 45, device="cuda:0", generator=gen) * 2 - 1 for _ in range(steps)]
    for i in range(3):
        g.step(acts[i])
    rates = []
    for _ in range(5):  # median of 5 timed blocks (the box's clocks wander by a few %)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            g.step(acts[i])
        torch.cuda.synchronize()
        rates.append(n * steps / (time.perf_counter() - t0))
    r = sorted(rates)[2]
    lib = Path(dp._lib.LIB_PATH).name
    print(f"{name:15s} N={n:6d}: {r:12,.0f} env-steps/s ({n / r * 1e3:.3f} ms/step) "
          f"[min {min(rates):,.0f} max {max(rates):,.0f}] {lib} iters={task.solver_iterations}", flush=True)


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "twinkle"
    for n in [int(x) for x in sys.argv[2:]] or [1024, 4096, 16384]:
        throughput(name, n)
