# Development aid: Newton variants - parity probe (bench / trace / random), throughput, and the
# iteration counts of their -DPS_TIMING builds (libX_timing.so next to libX.so when present).
# usage (on the box, via gpurun): bash tools/gpu_nt_variants.sh libA.so libB.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ntv.txt
for L in "$@"; do
  PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 300 python -u tools/parity_probe.py bench trace random >> gpurun_out/ntv.txt 2> gpurun_out/ntv_$L.err || exit 9
  PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 >> gpurun_out/ntv.txt 2>&1 || exit 6
  T=${L%.so}_timing.so
  if [ -f diffusion-piano_amd/$T ]; then
    PIANOSIM_LIB=diffusion-piano_amd/$T timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field > gpurun_out/ntv_phase_$L.txt 2>&1 || exit 5
    grep -E "^total|^Newton" gpurun_out/ntv_phase_$L.txt | sed "s/^/$L /" >> gpurun_out/ntv.txt
  fi
done
grep -v amdgpu.ids gpurun_out/ntv.txt
