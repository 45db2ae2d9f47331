# Development aid: the parity gates' data (tests with their printed statistics, no -x), the
# parity probe over every case, and the bench line. usage: bash tools/gpu_probe.sh <prefix>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-r05_p}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_solver.py tests/test_gpu_colliders.py tests/test_gpu_task_kwargs.py tests/test_gpu_ppo.py} > gpurun_out/${P}_tests.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/${P}_tests.log
if [ $RC -gt 1 ]; then exit 9; fi
if [ -z "$NOPROBE" ]; then
timeout -k 10 900 python -u tools/parity_probe.py > gpurun_out/${P}_probe.jsonl 2> gpurun_out/${P}_probe.err || exit 3
fi
timeout -k 10 400 python bench.py > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || exit 4
echo DONE
