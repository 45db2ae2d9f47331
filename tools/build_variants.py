"""Build variant step libraries for GPU A/B runs (development aid): the product flags of
__graft_entry__._hipcc_lib plus -D switches, in parallel.

usage: python tools/build_variants.py name=-DPS_X=1,-DPS_Y=2 [name=...]
writes diffusion-piano_amd/libpianosim_<name>.so (select with PIANOSIM_LIB=...)."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as ge  # noqa: E402

FLAGS = ["-fno-hip-fp32-correctly-rounded-divide-sqrt", "-falign-loops=64", "-mllvm", "-amdgpu-sched-strategy=max-ilp"]


def main(specs):
    procs = []
    for spec in specs:
        name, _, defs = spec.partition("=")
        out = ge.PKG / f"libpianosim_{name}.so"
        cmd = [ge.HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-value", *FLAGS,
               *[d for d in defs.split(",") if d], "-o", str(out), str(ge.PKG / "csrc" / "pianosim.hip")]
        procs.append((name, subprocess.Popen(cmd)))
    bad = [n for n, p in procs if p.wait() != 0]
    if bad:
        sys.exit(f"failed: {bad}")


if __name__ == "__main__":
    main(sys.argv[1:])
