# Parity probe + throughput of several prebuilt step-kernel libraries on one box (development aid).
# usage (on the box, via gpurun): bash tools/gpu_variants.sh libA.so libB.so ...  (names under diffusion-piano_amd/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/variants.jsonl
for L in "$@"; do
  PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 300 python -u tools/parity_probe.py ${CASES:-} >> gpurun_out/variants.jsonl 2> gpurun_out/variants_$L.err || exit 9
  PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 200 python tools/throughput.py crossing_field ${NS:-4096} >> gpurun_out/variants_tp.txt 2>&1 || exit 6
done
cat gpurun_out/variants.jsonl gpurun_out/variants_tp.txt
