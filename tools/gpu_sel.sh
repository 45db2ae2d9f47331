# Development aid: a pytest selection on the GPU, failures and parity summaries listed.
# usage (on the box, via gpurun): bash tools/gpu_sel.sh <pytest selection ...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -q -m gpu --timeout 300 --timeout-method thread -s > gpurun_out/pytest_sel.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/pytest_sel.log
grep -E "passed|failed|^FAILED|: n [0-9]+, median|max coupled|calm of|^E  " gpurun_out/pytest_sel.log | head -60
if [ $RC -gt 1 ]; then exit 9; fi
