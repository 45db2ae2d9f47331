"""Algorithmic FLOPs per env-step, counted by running the fp64 oracle's
counting build (oracle/flops.cpp: every add/sub, mul, div, sqrt/transcendental with no zero
operand) over random-action rollouts of the bench configs. Writes profiles/flops.json, which
bench.py turns into its `valu_roofline` (FP32 vector peak). CPU only.
usage: python tools/count_flops.py [envs] [steps]"""
import importlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))
dp = importlib.import_module("diffusion-piano_amd")
import ref  # noqa: E402  (measurement infrastructure, not the product)
from helpers import song  # noqa: E402


def count(name, n, steps, seed=12345):
    task = dp.TaskConfig(trim_silence=name != "twinkle")
    md, st, tc = dp.compile_task(song(dp, name), task, canonical_actions=False)
    env = ref.OracleEnv(md, st, tc, n, counting=True)
    env.reset()
    lo, hi = dp.model.action_spec(md)
    rng = np.random.RandomState(seed)
    ref.flops_reset()
    t0 = time.perf_counter()
    ncon = 0
    for _ in range(steps):
        env.step(rng.uniform(lo, hi, (n, 45)).astype(np.float32))
        ncon += int(env.contact_count().sum())
    c = ref.flops_get().astype(np.float64) / (n * steps)
    return {"song": name, "envs": n, "steps": steps, "episode_T": int(st.T),
            "flops_per_env_step": float(c.sum()),
            "add_sub": float(c[0]), "mul": float(c[1]), "div": float(c[2]), "sqrt_transc_minmax": float(c[3]),
            "mean_contacts_at_step_end": ncon / (n * steps), "seconds": time.perf_counter() - t0}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 340
    out = {"method": "oracle/flops.cpp counting build: fp64 ops with no zero operand (dense rows' "
                     "structural zeros skipped), FMA = 2, sqrt/div/transcendental = 1; uniform "
                     "random actions, resets included", "configs": {}}
    for name in ("crossing_field", "twinkle"):
        r = count(name, n, steps)
        out["configs"][name] = r
        print(json.dumps(r), flush=True)
    (ROOT / "profiles" / "flops.json").write_text(json.dumps(out, indent=1) + "\n")
