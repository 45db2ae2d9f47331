# Development aid: capsule kernel with / without the collision-time parking (libv_pk: parked)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in libpianosim.so libv_pk.so libpianosim.so libv_pk.so; do
  PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 2>&1 | grep -v amdgpu.ids || exit 4
done
for L in libpianosim_timing.so libv_pk_timing.so; do
  PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field > gpurun_out/pk_$L.txt 2>&1 || exit 5
  echo "== $L"; grep -v amdgpu.ids gpurun_out/pk_$L.txt | sed -n 1,22p
done
