# Diagnostics of the step kernel on one box (development aid): phase split + solver counters
# of the -DPS_TIMING build, and throughput of the current build vs libpianosim_base.so (built
# beforehand from an earlier commit; run with the round-1 PGS solver).
# usage (on the box, via gpurun): bash tools/gpu_diag.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$SKIP_PHASE" ] || PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field > gpurun_out/diag_phase.txt 2>&1 || exit 5
cat gpurun_out/diag_phase.txt | head -24
: > gpurun_out/diag_tp.txt
if [ -f diffusion-piano_amd/libpianosim_base.so ]; then
  PIANOSIM_SOLVER=pgs PIANOSIM_LIB=diffusion-piano_amd/libpianosim_base.so timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 >> gpurun_out/diag_tp.txt 2>&1 || exit 6
fi
timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 >> gpurun_out/diag_tp.txt 2>&1 || exit 6
PIANOSIM_SOLVER=pgs timeout -k 10 200 python tools/throughput.py crossing_field 4096 >> gpurun_out/diag_tp.txt 2>&1 || exit 6
cat gpurun_out/diag_tp.txt
