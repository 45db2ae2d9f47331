"""Phase ablation timing (results are wrong with skips; timing only)."""
import os, subprocess, sys
masks = {"full": 0, "no-kin": 1, "no-dyn": 2, "no-collide": 4, "no-factor": 8, "no-solve_smooth": 16,
         "no-constraints": 32, "no-pgs-iters": 64, "only-integrate": 1|2|4|8|16|32|64}
for name, m in masks.items():
    env = dict(os.environ, PIANOSIM_SKIP=str(m))
    out = subprocess.run([sys.executable, "tools/gpu_probe.py", "tp"], env=env, capture_output=True, text=True)
    lines = [l for l in out.stdout.splitlines() if "N=4096" in l]
    print(f"{name:18s} {lines[0] if lines else out.stderr[-300:]}", flush=True)
