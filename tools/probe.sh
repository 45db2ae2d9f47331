# occupancy probe (development aid): throughput of experiment builds side by side
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/probe.txt
for L in ${LIBS:-libpianosim.so}; do
  PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 200 python tools/throughput.py crossing_field ${NS:-1024 4096 16384} >> gpurun_out/probe.txt 2>&1 || exit 6
done
cat gpurun_out/probe.txt
