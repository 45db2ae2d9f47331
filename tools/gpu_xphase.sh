# Development aid: hull-kernel phase split with and without its box/hull collision sections
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in "$@"; do
  PIANOSIM_HULL=1 PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field > gpurun_out/xphase_$L.txt 2>&1 || exit 5
  echo "== $L"; grep -v amdgpu.ids gpurun_out/xphase_$L.txt | sed -n 1,29p
done
