# Development aid (round 5): the whole GPU suite without -x (every gate's printed numbers), the
# throughput of the current build (hull / primitive / capsule hands) and the hull phase split.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-ck}
mkdir -p gpurun_out
for H in hull primitive authored; do
  PIANOSIM_HAND=$H timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/$H /" >> gpurun_out/${P}_tp.txt || exit 5
done
(PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field) > gpurun_out/${P}_hull_phase.txt 2>/dev/null || exit 7
if [ -z "$NOTEST" ]; then
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests -m gpu ${TESTK:+-k "$TESTK"} > gpurun_out/${P}_tests.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/${P}_tests.log
fi
echo DONE
