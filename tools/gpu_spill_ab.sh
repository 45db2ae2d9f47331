# Development aid: capsule-hand throughput of Newton-template variant libraries (timing only:
# libv_dec = every substep through the decoupled template, physics NOT the reference's).
set -o pipefail
cd $GRAFT_REPO_ROOT
for l in libpianosim.so libv_dec.so libv_no28.so; do
  PIANOSIM_LIB=diffusion-piano_amd/$l timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 2>&1 | grep -v amdgpu.ids || exit 4
done
