# Parity diagnosis of the trace-action case (development aid), then the solver tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PROBE_DIAG=1 timeout -k 10 300 python -u tools/parity_probe.py > gpurun_out/diag_trace.txt 2> gpurun_out/diag_trace.err || exit 8
cat gpurun_out/diag_trace.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_task_kwargs.py tests/test_gpu_task_cases.py -q -m gpu --timeout 300 --timeout-method thread -s > gpurun_out/pytest_sel.log 2>&1
echo "PYTEST_EXIT $?" >> gpurun_out/pytest_sel.log
grep -E "passed|failed|max coupled|env-steps:|Error|assert" gpurun_out/pytest_sel.log | head -40
