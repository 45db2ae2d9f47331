# Development aid (round 5): Newton refinement variants (PS_NT_REFINE=2: a polish step for coupled
# substeps; PS_EXP_POLISH: for all) against the default build: parity probe, throughput, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_refine2.txt
: > $O
PIANOSIM_LIB=diffusion-piano_amd/libpianosim_cpol.so timeout -k 10 900 python -u tools/parity_probe.py bench coupled trace heavy guren random > gpurun_out/ab_cpol_probe.jsonl 2>/dev/null || exit 6
timeout -k 10 900 python -u tools/parity_probe.py bench coupled heavy hull > gpurun_out/ab_new_probe.jsonl 2>/dev/null || exit 6
for rep in 1 2; do
  for L in new cpol polish; do
    F=libpianosim_$L.so; [ $L = new ] && F=libpianosim.so
    PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/hull $L /" >> $O || exit 5
    PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/capsule $L /" >> $O || exit 5
  done
done
(PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field) > gpurun_out/ab_xgR_phase.txt 2>/dev/null || exit 7
echo DONE
