# Development round on one box: a test selection, throughput, phase split (outputs under gpurun_out/).
# usage (on the box, via gpurun): bash tools/gpu_dev.sh "<pytest selection>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${1:-tests}
timeout -k 10 600 python -u -m pytest $SEL -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/dev_pytest.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/dev_pytest.log
grep -E "passed|failed|^E  .*Error|^E  .*assert" gpurun_out/dev_pytest.log | tail -24
if [ $RC -gt 1 ]; then exit 9; fi
timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 16384 > gpurun_out/dev_tp.txt 2>&1 || exit 6
cat gpurun_out/dev_tp.txt
PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field > gpurun_out/dev_phase.txt 2>&1 || exit 5
head -26 gpurun_out/dev_phase.txt
