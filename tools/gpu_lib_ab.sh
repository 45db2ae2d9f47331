# Development aid: step-kernel builds A/B (args: lib file names in diffusion-piano_amd/) -
# parity probe, capsule-hand and box/hull-hand throughput per build, interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/libab.txt
for L in "$@"; do
  PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 300 python -u tools/parity_probe.py bench trace >> gpurun_out/libab.txt 2> gpurun_out/libab_$L.err || exit 9
done
for rep in 1 2; do
  for L in "$@"; do
    PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 >> gpurun_out/libab.txt 2>&1 || exit 6
    PIANOSIM_HULL=1 PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 200 python tools/throughput.py crossing_field 4096 | sed "s/^/hull /" >> gpurun_out/libab.txt 2>&1 || exit 7
  done
done
grep -v amdgpu.ids gpurun_out/libab.txt
