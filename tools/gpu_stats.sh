# Development aid (round 5): hull phase timing with the hand-hand pair statistics, and the whole
# GPU suite without -x (every gate's printed numbers).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
(PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field) > gpurun_out/st_hull_phase.txt 2>/dev/null || exit 7
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/st_tests.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/st_tests.log
echo DONE
