# Development aid: the GPU suite (all tests, failures listed), then throughput of the capsule
# and the box / hull hands and the hull hand's phase split.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -s > gpurun_out/pytest_gpu.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|^FAILED|: n [0-9]+, median|max coupled|calm of" gpurun_out/pytest_gpu.log | head -60
if [ $RC -gt 1 ]; then exit 9; fi
timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 > gpurun_out/tp.txt 2>&1 || exit 6
PIANOSIM_HULL=1 timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 >> gpurun_out/tp.txt 2>&1 || exit 6
grep N= gpurun_out/tp.txt
PIANOSIM_HULL=1 PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field > gpurun_out/hull_phase.txt 2>&1 || exit 5
head -26 gpurun_out/hull_phase.txt
