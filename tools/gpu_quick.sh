# GPU tests (optionally a selection) + throughput, one box (development aid).
# usage (on the box, via gpurun): bash tools/gpu_quick.sh [pytest selection]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${1:-tests}
timeout -k 10 600 python -u -m pytest $SEL -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
if [ $RC -gt 1 ]; then exit 9; fi
timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 > gpurun_out/quick_tp.txt 2>&1 || exit 6
cat gpurun_out/quick_tp.txt
PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field > gpurun_out/diag_phase.txt 2>&1 || exit 5
head -24 gpurun_out/diag_phase.txt
