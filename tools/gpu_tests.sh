# Development aid: run a subset of the GPU suite on the box with per-step time limits.
# usage (from gpurun): bash tools/gpu_tests.sh <tag> <pytest args...>
#   writes gpurun_out/<tag>_tests.log; the drift report (when test_gpu_drift runs) to
#   gpurun_out/<tag>_drift.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
shift
export PIANOSIM_REPORT=gpurun_out/${tag}_drift.json
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread "$@" > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${tag}_tests.log
exit $rc
