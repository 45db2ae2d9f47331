# Build diffusion-piano_amd/libpianosim_base.so from the step-kernel sources of a git revision
# (default HEAD), the "before" side of tools/ab.sh. Runs on the CPU side (hipcc cross-compiles).
# usage: bash tools/build_base.sh [rev]
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p "$T/pkg/csrc" "$T/include"
for f in pianosim.hip kernel_v2.inc newton.inc devmodel.h prims.h collide_x.h; do
  git -C "$ROOT" show "$REV:diffusion-piano_amd/csrc/$f" > "$T/pkg/csrc/$f"
done
git -C "$ROOT" show "$REV:include/pianosim.h" > "$T/include/pianosim.h"
cd "$T/pkg/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-value \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -falign-loops=64 \
  -o "$ROOT/diffusion-piano_amd/libpianosim_base.so" pianosim.hip
rm -rf "$T"
echo "built libpianosim_base.so from $REV"
